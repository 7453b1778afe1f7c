#!/bin/bash
# Forced multi-rank path (1-rank RCCL group) vs inline on the last tree, alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/fdfinal
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --ref-mb 0 > $O/inline_$i.jsonl 2>/dev/null && echo "inline $(tail -1 $O/inline_$i.jsonl | python3 -c 'import json,sys; print(json.loads(sys.stdin.read())["ms_per_step"])')" &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 --ref-mb 0 --force-dist > $O/forced_$i.jsonl 2>/dev/null && echo "forced $(tail -1 $O/forced_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); a=d["extra"].get("allreduce") or {}; print(d["ms_per_step"], {k: a.get(k) for k in ("algo_bw_GBps", "comm_ms_per_step")})')" || exit 1
done
