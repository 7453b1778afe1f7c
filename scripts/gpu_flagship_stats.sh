#!/bin/bash
# Kernel statistics of the flagship bench step (world 1) under rocprofv3 --kernel-trace --stats.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/flag
export TMPDIR=/tmp
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/flag/bench.log 2>&1 && tail -1 gpurun_out/flag/bench.log | cut -c1-300 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/flag/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 > gpurun_out/flag/prof.log 2>&1 && echo prof-ok
