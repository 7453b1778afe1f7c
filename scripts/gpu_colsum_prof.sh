#!/bin/bash
# Kernel-level split of the fused bias-gradient cost on the bwd-weight GEMMs (GEMM kernel vs colsum reduce).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/colsum_prof2
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/colsum_prof2 -o run --output-format csv -- python3 bench/gemm_bench.py --mb 8192 --shapes bwdw1,bwdw0 --epi-arms --rounds 3 > gpurun_out/colsum_prof2/bench.log 2>&1
rc=$?; cut -c1-400 gpurun_out/colsum_prof2/bench.log | grep shape; exit $rc
