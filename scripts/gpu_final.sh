#!/bin/bash
# Round-end record on one box: GPU tests, smoke(), flagship bench (3 runs), kernel-trace stats of the flagship.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/final_pytest.log 2>&1 &&
tail -2 gpurun_out/final_pytest.log &&
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/final_smoke.log 2>&1 && tail -1 gpurun_out/final_smoke.log &&
for rep in 1 2 3; do
  timeout -k 10 200 python3 bench.py > gpurun_out/final_bench_$rep.log 2>&1 || exit 1
  tail -1 gpurun_out/final_bench_$rep.log
done &&
timeout -k 10 200 python3 bench.py --force-dist --steps 40 --warmup 10 > gpurun_out/final_fd.log 2>&1 && tail -1 gpurun_out/final_fd.log &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_final -o p --output-format csv -- python3 bench.py --steps 20 --warmup 5 > gpurun_out/prof_final.log 2>&1 &&
echo done
