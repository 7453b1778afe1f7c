#!/bin/bash
# Tile / split-K sweep of the MLP's narrow GEMMs at MB 8192 (bwd-weight of fc0 / fc2 with K = 8192, fwd0 / fwd2,
# bwd-data of fc2), plus the bwd-weight epilogue arms (colsum, BFP wire) under the default plan.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sweep
export TMPDIR=/tmp
timeout -k 10 500 python bench/gemm_bench.py --mb 8192 --sweep --rounds 3 --shapes bwdw0,bwdw2,fwd0,fwd2,bwdd2 > gpurun_out/sweep/sweep.jsonl 2>&1 &&
timeout -k 10 300 python bench/gemm_bench.py --mb 8192 --epi-arms --rounds 5 --shapes bwdw0,bwdw2 > gpurun_out/sweep/arms.jsonl 2>&1 && echo ok
