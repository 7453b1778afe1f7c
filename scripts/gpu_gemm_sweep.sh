#!/bin/bash
# Tile / split-K sweep of the narrow bwd-weight shapes with each 256x256 main loop (FAN_GEMM_PP=0/1).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for pp in 0 1; do
  FAN_GEMM_PP=$pp timeout -k 10 300 python bench/gemm_bench.py --mb ${MB:-8192} --shapes ${SHAPES:-bwdw2,bwdw0} --sweep --rounds 3 \
    > gpurun_out/sweep_pp$pp.log 2>&1 || exit $?
done
grep -h sweep_us gpurun_out/sweep_pp0.log gpurun_out/sweep_pp1.log | cut -c1-600
