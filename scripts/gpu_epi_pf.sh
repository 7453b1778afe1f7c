#!/bin/bash
# ReLU-mask epilogue with the activation loads prefetched two 16-row blocks ahead + register-resident softmax-xent:
# numerics, epilogue cost probe, flagship bench x3 and its kernel statistics.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/epipf
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_gemm_ragged.py -x -q --timeout 120 --timeout-method thread > gpurun_out/epipf/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/epipf/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/epipf/pytest.log | head -8; exit $rc; }
timeout -k 10 200 python tools/probes/epi_cost_probe.py > gpurun_out/epipf/epi.jsonl 2>&1 && grep '^{' gpurun_out/epipf/epi.jsonl || exit 1
for i in 1 2 3; do
timeout -k 10 200 python bench.py --ref-mb 0 --steps 40 > gpurun_out/epipf/bench_$i.jsonl 2>/dev/null || exit 1
echo "$(tail -1 gpurun_out/epipf/bench_$i.jsonl | cut -c1-250)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/epipf/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --ref-mb 0 > gpurun_out/epipf/prof.log 2>&1 && echo prof done
