#!/bin/bash
# Round-2 resume check: whole GPU suite on the rebuilt tree, smoke, flagship bench x2, kernel stats of the step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/resume
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/resume/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/resume/pytest_gpu.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 200 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/resume/smoke.log 2>&1 && tail -1 gpurun_out/resume/smoke.log || exit 1
for i in 1 2; do
timeout -k 10 300 python bench.py > gpurun_out/resume/bench_$i.jsonl 2>gpurun_out/resume/bench_$i.err && tail -1 gpurun_out/resume/bench_$i.jsonl | cut -c1-300 || exit 1
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/resume/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --ref-mb 0 > gpurun_out/resume/prof.log 2>&1 && echo prof done
