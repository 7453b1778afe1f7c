#!/bin/bash
# GEMM kernel tests, then ping-pong vs one-role main loop A/B on the MLP shapes (MB 8192), then the flagship bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_prepack.py -x -q --timeout 120 \
  --timeout-method thread > gpurun_out/pytest_kernels.log 2>&1; rc=$?; tail -15 gpurun_out/pytest_kernels.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/gemm_bench.py --mb ${MB:-8192} --ab --rounds 5 ${GEMM_ARGS:-} > gpurun_out/gemm_ab.log 2>&1; rc=$?
cut -c1-420 gpurun_out/gemm_ab.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-400
