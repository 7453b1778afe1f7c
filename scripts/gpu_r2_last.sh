#!/bin/bash
# Last check of the round on the final tree: whole GPU suite, smoke, flagship bench x3, kernel statistics.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/last
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?
tail -2 $O/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "Error|assert|FAIL" $O/pytest_gpu.log | head -8; exit $rc; }
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 && tail -1 $O/smoke.log || exit 1
for i in 1 2 3; do
timeout -k 10 300 python bench.py > $O/bench_$i.jsonl 2>$O/bench_$i.err || exit 1
tail -1 $O/bench_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print("bench", d["value"], d["ms_per_step"], "mb1792", d["extra"]["mb1792"]["samples_per_s"] if d["extra"].get("mb1792") else None)'
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --ref-mb 0 > $O/prof.log 2>&1 && echo prof done
