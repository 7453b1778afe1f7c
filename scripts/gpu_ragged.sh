#!/bin/bash
# Edge-tile GEMMs: ragged-shape tests first (fast fail), then the whole GPU suite, the flagship bench (aligned fast
# path unchanged?) and GEMM timings vs hipBLASLt on the MLP and ragged shape sets.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_gemm_ragged.py -x -v --timeout 120 --timeout-method thread > gpurun_out/pytest_ragged.log 2>&1; rc=$?
tail -25 gpurun_out/pytest_ragged.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-600 &&
timeout -k 10 300 python bench/gemm_bench.py --mb 8192 > gpurun_out/gemm_mlp8192.jsonl 2>&1 && cat gpurun_out/gemm_mlp8192.jsonl | cut -c1-300 &&
timeout -k 10 300 python bench/gemm_bench.py --set ragged > gpurun_out/gemm_ragged_bf16.jsonl 2>&1 && cat gpurun_out/gemm_ragged_bf16.jsonl | cut -c1-300 &&
timeout -k 10 300 python bench/gemm_bench.py --set ragged --dtype f32 > gpurun_out/gemm_ragged_f32.jsonl 2>&1 && cat gpurun_out/gemm_ragged_f32.jsonl | cut -c1-300
