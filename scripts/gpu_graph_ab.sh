#!/bin/bash
# Flagship bench: HIP-graph replay of the whole world-1 step vs eager launches, alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/graph
export TMPDIR=/tmp
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --graph > gpurun_out/graph/b_graph_$i.log 2>&1 && echo "graph $(tail -1 gpurun_out/graph/b_graph_$i.log | cut -c150-230) $(grep -o '"hip_graph": [a-z]*' gpurun_out/graph/b_graph_$i.log)" &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/graph/b_eager_$i.log 2>&1 && echo "eager $(tail -1 gpurun_out/graph/b_eager_$i.log | cut -c150-230)" || exit 1
done
grep -i "capture failed" gpurun_out/graph/*.log | head -3
