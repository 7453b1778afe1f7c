#!/bin/bash
# Packed ReLU masks: numerics on every tile / loop / split-K path, epilogue cost probe, flagship A/B (FAN_RELU_BITS
# 1 vs 0 alternated) and an in-step A/B of the narrow bwd-weight plan (256x256 split 4 vs 256x128 split 2).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/bits
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_relu_bits.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > gpurun_out/bits/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/bits/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/bits/pytest.log | head -8; exit $rc; }
timeout -k 10 200 python tools/probes/epi_cost_probe.py > gpurun_out/bits/epi.jsonl 2>&1 && cat gpurun_out/bits/epi.jsonl | grep '^{' || exit 1
for i in 1 2; do
for b in 1 0; do
FAN_RELU_BITS=$b timeout -k 10 200 python bench.py --ref-mb 0 --steps 40 > gpurun_out/bits/bench_b${b}_$i.jsonl 2>/dev/null || exit 1
echo "bits=$b $(tail -1 gpurun_out/bits/bench_b${b}_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
FAN_GEMM_PLAN="1024x4096x8192=256,128,2;4096x1024x8192=256,128,2" timeout -k 10 200 python bench.py --ref-mb 0 --steps 40 > gpurun_out/bits/bench_p128_$i.jsonl 2>/dev/null || exit 1
echo "bits=1 bwdw 256x128/s2 $(tail -1 gpurun_out/bits/bench_p128_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
