#!/bin/bash
# Pipelined 256x256 main loop (gemm_set_main_loop(2)): numerics on every layout / K-tile count, then GEMM timings
# of the one-role vs pipelined loops (same process, interleaved) and the flagship bench with each.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "256_tile" --timeout 120 --timeout-method thread > gpurun_out/pytest_pl.log 2>&1; rc=$?
tail -20 gpurun_out/pytest_pl.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/gemm_bench.py --mb 8192 --loops 0,2 --shapes fwd0,fwd1,fwd2,bwdd1,bwdd2,sq4k,sq8k > gpurun_out/gemm_pl_ab.jsonl 2>&1 && cut -c1-420 gpurun_out/gemm_pl_ab.jsonl &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_one.log 2>&1 && tail -1 gpurun_out/bench_one.log | cut -c1-300 &&
FAN_GEMM_PL=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_pl.log 2>&1 && tail -1 gpurun_out/bench_pl.log | cut -c1-300 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_one2.log 2>&1 && tail -1 gpurun_out/bench_one2.log | cut -c1-300
