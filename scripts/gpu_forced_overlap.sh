#!/bin/bash
# Forced 1-rank RCCL path vs inline world 1 (alternated), then a kernel trace of the forced path -> overlap report.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fov
export TMPDIR=/tmp
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/fov/inline_$i.log 2>&1 && echo "inline $(tail -1 gpurun_out/fov/inline_$i.log | cut -c150-230)" &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --force-dist > gpurun_out/fov/forced_$i.log 2>&1 && echo "forced $(tail -1 gpurun_out/fov/forced_$i.log | cut -c150-230)" || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fov/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --force-dist --ref-mb 0 > gpurun_out/fov/prof.log 2>&1 &&
python3 tools/overlap_report.py gpurun_out/fov/prof/run_kernel_trace.csv --json gpurun_out/fov/overlap.json
