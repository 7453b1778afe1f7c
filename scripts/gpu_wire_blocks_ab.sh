#!/bin/bash
# Flagship bench vs the BFP kernels' grid cap (FAN_WIRE_MAX_BLOCKS: 2048 default, 8192, 1024), alternated twice,
# plus the SGD kernel time from a kernel trace at each cap.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/wblk
export TMPDIR=/tmp
for i in 1 2; do
for b in 2048 8192 1024; do
FAN_WIRE_MAX_BLOCKS=$b timeout -k 10 300 python bench.py --steps 40 --warmup 5 --ref-mb 0 > gpurun_out/wblk/b_${b}_$i.log 2>&1 && echo "blocks $b $(tail -1 gpurun_out/wblk/b_${b}_$i.log | cut -c150-230)" || exit 1
done
done
for b in 2048 8192; do
FAN_WIRE_MAX_BLOCKS=$b timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/wblk/prof_$b -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 --ref-mb 0 > gpurun_out/wblk/prof_$b.log 2>&1 || exit 1
grep wire_sgd gpurun_out/wblk/prof_$b/run_kernel_stats.csv | cut -d, -f1-6 | cut -c1-200
done
