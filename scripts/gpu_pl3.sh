#!/bin/bash
# Pipelined loop on every layout (incl. the bwd-weight colsum / wire epilogues): whole GPU suite, GEMM A/B vs the
# one-role loop with the fused epilogue arms, flagship bench A/B.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu_pl4.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu_pl4.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu_pl4.log | head; exit $rc; }
timeout -k 10 300 python bench/gemm_bench.py --mb 8192 --loops 0,2 --epi-arms > gpurun_out/gemm_pl4_ab.jsonl 2>&1 && cut -c1-520 gpurun_out/gemm_pl4_ab.jsonl &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_pl4.log 2>&1 && tail -1 gpurun_out/bench_pl4.log | cut -c1-300 &&
FAN_GEMM_PL=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_pl4_0.log 2>&1 && tail -1 gpurun_out/bench_pl4_0.log | cut -c1-300 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_pl4b.log 2>&1 && tail -1 gpurun_out/bench_pl4b.log | cut -c1-300 &&
FAN_GEMM_PL=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_pl4_0b.log 2>&1 && tail -1 gpurun_out/bench_pl4_0b.log | cut -c1-300
