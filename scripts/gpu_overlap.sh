#!/bin/bash
# Overlap evidence: kernel trace of the flagship bench through the full multi-rank path at world 1 (1-rank
# RCCL communicator, side comm stream), then the compute/comm overlap computed from the trace.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
export MASTER_ADDR=127.0.0.1 MASTER_PORT=29571 RANK=0 WORLD_SIZE=1 LOCAL_RANK=0
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_ovl -o run --output-format csv -- python3 bench.py --force-dist --steps 10 --warmup 3 --mb-per-gpu ${MB:-8192} > gpurun_out/prof_ovl.log 2>&1 || { tail -30 gpurun_out/prof_ovl.log; exit 1; }
tail -1 gpurun_out/prof_ovl.log | cut -c1-300
python3 tools/overlap_report.py $(find gpurun_out/prof_ovl -name "*kernel_trace.csv" | head -1) --json gpurun_out/overlap.json
