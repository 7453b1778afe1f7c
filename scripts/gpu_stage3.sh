#!/bin/bash
# 3-stage 256x128 pipelined GEMM: numerics (kernel + ragged suites, persistent grid caps), classifier-forward probe
# (hot / cold operands), flagship bench x3 with kernel statistics.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/stage3
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_gemm_ragged.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head -8; exit $rc; }
timeout -k 10 200 python tools/probes/fwd2_out_probe.py > $O/fwd2.jsonl 2>&1 && grep '^{' $O/fwd2.jsonl || exit 1
for i in 1 2 3; do
timeout -k 10 200 python bench.py --ref-mb 0 --steps 40 > $O/bench_$i.jsonl 2>/dev/null || exit 1
echo "$(tail -1 $O/bench_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["value"], d["ms_per_step"])')"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --ref-mb 0 > $O/prof.log 2>&1 && echo prof done
