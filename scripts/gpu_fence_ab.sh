#!/bin/bash
# Release scope of the engine's cross-stream events (FAN_EVENT_FENCE unset = HIP default vs device): the flagship
# step shows a 5.5 us idle gap after every request's epilogue (three per step); same-box A/B, alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/fence
export TMPDIR=/tmp
for i in 1 2 3; do
for f in default device; do
if [ $f = default ]; then unset FAN_EVENT_FENCE; else export FAN_EVENT_FENCE=$f; fi
timeout -k 10 200 python bench.py --ref-mb 0 --steps 40 > gpurun_out/fence/bench_${f}_$i.jsonl 2>/dev/null || exit 1
echo "$f $(tail -1 gpurun_out/fence/bench_${f}_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
done
export FAN_EVENT_FENCE=device
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/fence/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --ref-mb 0 > gpurun_out/fence/prof.log 2>&1 && echo prof done
