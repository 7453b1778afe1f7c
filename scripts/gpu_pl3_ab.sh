#!/bin/bash
# Main-loop A/B in the step: FAN_GEMM_PL=2 (default: the 4096^2 bwd-weight with the wire epilogue on the 8-wave
# pipelined kernel) vs 3 (4-wave kernel for every 256x256 GEMM, i.e. also that bwd-weight). Alternated, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/pl3ab
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
for m in 2 3; do
FAN_GEMM_PL=$m timeout -k 10 200 python bench.py --ref-mb 0 --steps 40 > $O/b_${m}_$i.jsonl 2>/dev/null || exit 1
echo "pl=$m $(tail -1 $O/b_${m}_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
done
FAN_GEMM_PL=3 timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --ref-mb 0 > $O/prof.log 2>&1 && echo prof done
