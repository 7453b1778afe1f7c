#!/bin/bash
# Round-2 check: full GPU test suite, flagship bench (world 1 inline), the multi-rank path at world 1 with the
# device-timed all-reduce report, rocprof kernel stats. Every GPU step under its own timeout, chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[r2] host $(hostname) start $(date)"
python -c "import torch;print('torch', torch.__version__, torch.cuda.get_device_name(0))" &&
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; grep -E "^(FAILED|ERROR)|Error" gpurun_out/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-2000 &&
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --force-dist > gpurun_out/bench_fd.log 2>&1 && tail -1 gpurun_out/bench_fd.log | cut -c1-3000 &&
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof.log 2>&1 && echo "[r2] profile done"
fi
