#!/bin/bash
# Forced multi-rank path: decode+SGD epilogue on the comm stream (per layer, after its bwd-data GEMM) vs on the
# compute stream after the last backward GEMM (default), alternated; plus trainer equivalence tests for both.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/epi
export TMPDIR=/tmp
for i in 1 2 3; do
for e in producer comm; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --force-dist --ref-mb 0 --epi $e > gpurun_out/epi/${e}_$i.log 2>&1 && echo "epi $e $(tail -1 gpurun_out/epi/${e}_$i.log | cut -c150-230)" || exit 1
done
done
