#!/bin/bash
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --output-format csv -d gpurun_out/blasnames -o run -- python3 tools/probes/blas_kernel_names.py > gpurun_out/blasnames.log 2>&1 || { tail -20 gpurun_out/blasnames.log; exit 1; }
f=$(find gpurun_out/blasnames -name "*kernel_trace.csv" | head -1)
python3 - "$f" <<'PY'
import csv, sys
seen = {}
for r in csv.DictReader(open(sys.argv[1])):
    n = r["Kernel_Name"]
    k = (n, r.get("Workgroup_Size_X", r.get("Workgroup_Size", "")), r.get("Grid_Size_X", r.get("Grid_Size", "")), r.get("LDS_Block_Size", r.get("Lds_Size", "")), r.get("VGPR_Count", ""), r.get("Accum_VGPR_Count", ""), r.get("SGPR_Count", ""))
    seen[k] = seen.get(k, 0) + 1
for k, c in seen.items():
    print(c, "|", " | ".join(str(x) for x in k[1:]), "|", k[0][:400])
print(list(csv.DictReader(open(sys.argv[1])))[0].keys())
PY
