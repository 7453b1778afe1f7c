#!/bin/bash
# Forced multi-rank path: comm-stream priority high (-1, default) vs normal (0), alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/prio
export TMPDIR=/tmp
for i in 1 2 3; do
for p in -1 0; do
FAN_COMM_PRIORITY=$p timeout -k 10 300 python bench.py --steps 30 --warmup 5 --force-dist --ref-mb 0 > gpurun_out/prio/p${p}_$i.log 2>&1 && echo "prio $p $(tail -1 gpurun_out/prio/p${p}_$i.log | cut -c150-230)" || exit 1
done
done
