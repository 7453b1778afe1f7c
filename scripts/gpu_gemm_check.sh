#!/bin/bash
# GEMM change check: kernel tests, GEMM bench at MB 2048 and 8192 (vs hipBLASLt), flagship bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -m pytest tests/test_gpu_kernels.py tests/test_gpu_prepack.py -x -q > gpurun_out/pytest_gemm.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gemm.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gemm.log; exit $rc; }
for mb in 2048 8192; do
  timeout -k 10 600 python bench/gemm_bench.py --mb $mb --rounds 5 --shapes fwd0,fwd1,fwd2,bwdw2,bwdw1,bwdw0,bwdd2,bwdd1 > gpurun_out/gemm_$mb.jsonl 2>&1 || { tail -20 gpurun_out/gemm_$mb.jsonl; exit 1; }
  python3 -c "
import json
tot_m=tot_r=0
for l in open('gpurun_out/gemm_$mb.jsonl'):
    if l.startswith('{'):
        d=json.loads(l); tot_m+=d['mine_us']; tot_r+=d['torch_matmul_only_us']
        print('$mb', d['shape'], d['plan'], d['mine_us'], d['torch_matmul_only_us'])
print('$mb total mine', round(tot_m,1), 'hipblaslt', round(tot_r,1))
"
done
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/bench_g.log 2>&1 && tail -1 gpurun_out/bench_g.log | cut -c1-200
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --mb-per-gpu 2048 > gpurun_out/bench_g2.log 2>&1 && tail -1 gpurun_out/bench_g2.log | cut -c1-200
