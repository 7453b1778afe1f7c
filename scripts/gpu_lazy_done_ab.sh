#!/bin/bash
# Inline requests' done event recorded lazily (default) vs at every commit (FAN_LAZY_DONE=0), and the HIP-graph
# replay of the step, alternated on one box; kernel trace of the default for the inter-kernel gaps. GPU engine tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/lazy
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_native_engine.py tests/test_gpu_p2p.py -x -q --timeout 120 --timeout-method thread > gpurun_out/lazy/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/lazy/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/lazy/pytest.log | head -8; exit $rc; }
for i in 1 2 3; do
for f in 1 0 g; do
if [ $f = g ]; then export FAN_LAZY_DONE=1; G=--graph; else export FAN_LAZY_DONE=$f; G=; fi
timeout -k 10 200 python bench.py --ref-mb 0 --steps 40 $G > gpurun_out/lazy/bench_${f}_$i.jsonl 2>/dev/null || exit 1
echo "lazy=$f $(tail -1 gpurun_out/lazy/bench_${f}_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"], d["config"]["hip_graph"])')"
done
done
export FAN_LAZY_DONE=1
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/lazy/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --ref-mb 0 > gpurun_out/lazy/prof.log 2>&1 && echo prof done
