#!/bin/bash
# GEMM kernel tests + GEMM bench vs hipBLASLt (rebuilds the extension first if a source is newer).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
if [ -n "$(find csrc -newer fpga_ai_nic_amd/_C.so -type f 2>/dev/null)" ]; then python tools/build_ext.py -j 16 || exit 1; fi
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py -x -q > gpurun_out/pytest_kernels.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_kernels.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/gemm_bench.py ${GEMM_ARGS:-} > gpurun_out/gemm_bench.log 2>&1; rc=$?; cat gpurun_out/gemm_bench.log | cut -c1-400; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-300
