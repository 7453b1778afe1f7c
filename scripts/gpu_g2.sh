#!/bin/bash
# MB-8192 GEMM tile/split-K sweep for the narrow shapes + PMC passes on the big ones.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench/gemm_bench.py --mb 8192 --shapes bwdw0,bwdw2,fwd2 --sweep --rounds 3 > gpurun_out/sweep8192.log 2>&1 &&
SHAPES=fwd1,bwdd1,bwdw1,bwdw0 bash scripts/gpu_pmc_gemm.sh
