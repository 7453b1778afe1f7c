#!/bin/bash
# Kernel-trace stats of the multi-rank path (forced 1-rank RCCL group) with both epilogue placements.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
for arm in producer comm; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fd_$arm -o p --output-format csv -- \
    python3 bench.py --steps 20 --warmup 5 --force-dist --epi $arm > gpurun_out/prof_fd_$arm.log 2>&1 || exit 1
  tail -1 gpurun_out/prof_fd_$arm.log | cut -c1-200
done
echo done
