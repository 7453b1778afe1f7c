#!/bin/bash
# One GPU verification round: kernel/engine tests, bench, rocprof kernel stats. Each GPU step is time-limited
# and steps are chained with && so that a failure stops the run.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
echo "[gpu_round] host $(hostname) start $(date)"
# refuse to run with a stale extension (sources newer than the .so)
if [ -n "$(find csrc -newer fpga_ai_nic_amd/_C.so -type f 2>/dev/null)" ] || [ ! -f fpga_ai_nic_amd/_C.so ]; then
  echo "[gpu_round] _C.so is stale or missing: rebuilding"; python tools/build_ext.py -j 16 || exit 1
fi
python -c "import torch;print('torch', torch.__version__, torch.cuda.get_device_name(0))" &&
timeout -k 10 900 python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit $rc; }
timeout -k 10 300 python bench.py --steps ${BENCH_STEPS:-20} --warmup 5 > gpurun_out/bench.log 2>&1 && tail -2 gpurun_out/bench.log &&
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- python3 bench.py --steps 10 --warmup 3 > gpurun_out/prof.log 2>&1 && echo "[gpu_round] profile done"
fi
