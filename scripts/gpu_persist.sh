#!/bin/bash
# Persistent 4-wave GEMM: numerics (bit-identical to one workgroup per tile; kernel suite), timing probe, flagship A/B
# (FAN_GEMM_PERSIST=256 default vs 0) alternated on one box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/persist
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_gemm_ragged.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head -8; exit $rc; }
timeout -k 10 200 python tools/probes/persist_probe.py > $O/probe.jsonl 2>&1 && grep '^{' $O/probe.jsonl || exit 1
for i in 1 2 3; do
for c in 256 0; do
FAN_GEMM_PERSIST=$c timeout -k 10 200 python bench.py --ref-mb 0 --steps 40 > $O/bench_${c}_$i.jsonl 2>/dev/null || exit 1
echo "persist=$c $(tail -1 $O/bench_${c}_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
done
