#!/bin/bash
# Tightened GEMM tests, then a marker + kernel trace of the forced multi-rank path with the C++ engine's roctx ranges.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_gemm_ragged.py -x -q --timeout 200 --timeout-method thread > gpurun_out/pytest_kernels.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_kernels.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)|assert" gpurun_out/pytest_kernels.log | head; exit $rc; }
FAN_ROCTX=1 timeout -k 10 300 rocprofv3 --marker-trace --kernel-trace --output-format csv -d gpurun_out/prof_roctx -o run -- python3 bench.py --force-dist --steps 5 --warmup 2 --ref-mb 0 --no-trace > gpurun_out/prof_roctx.log 2>&1 || { tail -20 gpurun_out/prof_roctx.log; exit 1; }
ls gpurun_out/prof_roctx
