#!/bin/bash
# Pipelined loop + parallel ordered colsum reduce: GEMM/prepack/trainer tests, bwd-weight epilogue arms under a
# kernel trace, flagship bench A/B (pipelined vs one-role loop, alternated).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pl5
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pl5/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pl5/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/pl5/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/pl5/prof -o run --output-format csv -- python3 bench/gemm_bench.py --mb 8192 --shapes bwdw2,bwdw1,bwdw0 --epi-arms --rounds 3 > gpurun_out/pl5/gemm_epi.jsonl 2>&1 && grep shape gpurun_out/pl5/gemm_epi.jsonl | cut -c1-420 &&
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/pl5/bench_pl_$i.log 2>&1 && tail -1 gpurun_out/pl5/bench_pl_$i.log | cut -c1-250 &&
FAN_GEMM_PL=0 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/pl5/bench_0_$i.log 2>&1 && tail -1 gpurun_out/pl5/bench_0_$i.log | cut -c1-250 || exit 1
done
