#!/bin/bash
# Flagship bench, main-loop selection A/B: default (auto) vs FAN_GEMM_PL=${ARM_B:-3}, alternated 3x.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/flagab
export TMPDIR=/tmp
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/flagab/a_$i.log 2>&1 && echo "default $(tail -1 gpurun_out/flagab/a_$i.log | cut -c150-230)" &&
FAN_GEMM_PL=${ARM_B:-3} timeout -k 10 300 python bench.py --steps 40 --warmup 5 > gpurun_out/flagab/b_$i.log 2>&1 && echo "PL=${ARM_B:-3} $(tail -1 gpurun_out/flagab/b_$i.log | cut -c150-230)" || exit 1
done
