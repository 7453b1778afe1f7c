#!/bin/bash
# Pipelined loop as default: GEMM tests, the MN-contiguous-A layouts on the pipelined loop (experiment flag), the
# fwd2 shape on 256x256 split-K 2 (pipelined) vs the planned 128x256, flagship bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_gemm_ragged.py tests/test_gpu_prepack.py -x -q --timeout 120 --timeout-method thread > gpurun_out/pytest_pl2.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_pl2.log
[ $rc -eq 0 ] || exit $rc
FAN_GEMM_PL_ALL=1 timeout -k 10 300 python bench/gemm_bench.py --mb 8192 --loops 0,2 --shapes bwdw2,bwdw1,bwdw0 > gpurun_out/gemm_pl_all.jsonl 2>&1 && cut -c1-420 gpurun_out/gemm_pl_all.jsonl &&
FAN_GEMM_PLAN="8192x1024x4096=256,256,2" timeout -k 10 300 python bench/gemm_bench.py --mb 8192 --loops 0,2 --shapes fwd2 > gpurun_out/gemm_fwd2_sk2.jsonl 2>&1 && cut -c1-420 gpurun_out/gemm_fwd2_sk2.jsonl &&
FAN_GEMM_PLAN="8192x1024x4096=256,256,1" timeout -k 10 300 python bench/gemm_bench.py --mb 8192 --loops 0,2 --shapes fwd2 > gpurun_out/gemm_fwd2_sk1.jsonl 2>&1 && cut -c1-420 gpurun_out/gemm_fwd2_sk1.jsonl &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_pl_default.log 2>&1 && tail -1 gpurun_out/bench_pl_default.log | cut -c1-300 &&
FAN_GEMM_PL=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_pl0.log 2>&1 && tail -1 gpurun_out/bench_pl0.log | cut -c1-300 &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_pl_default2.log 2>&1 && tail -1 gpurun_out/bench_pl_default2.log | cut -c1-300
