#!/bin/bash
# Kernel trace of the flagship step inline (world 1) vs through the multi-rank path (--force-dist: 1-rank RCCL
# group, side-stream engine), plus plain timings of both, for the per-kernel / overlap comparison.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 > gpurun_out/mr_inline.log 2>&1 &&
timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --force-dist > gpurun_out/mr_fd.log 2>&1 &&
timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 > gpurun_out/mr_inline2.log 2>&1 &&
timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --force-dist > gpurun_out/mr_fd2.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_inline -o p --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_inline.log 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_fd -o p --output-format csv -- python3 bench.py --steps 20 --warmup 5 --force-dist > gpurun_out/prof_fd.log 2>&1 &&
echo done
