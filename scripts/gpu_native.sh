#!/bin/bash
# Native engine check: its GPU tests, then the bench with the Python- and C++-issued request paths
# (inline world 1 and the forced 1-rank RCCL path). Every GPU step is time-limited; chained with &&.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$(find csrc -newer fpga_ai_nic_amd/_C.so -type f 2>/dev/null)" ] || [ ! -f fpga_ai_nic_amd/_C.so ]; then
  echo "[gpu_native] _C.so is stale or missing: rebuilding"; python tools/build_ext.py -j 16 || exit 1
fi
R="python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531"
timeout -k 10 600 python -m pytest tests/test_gpu_native_engine.py ${PYTEST_ARGS:-} -x -q > gpurun_out/pytest_native.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_native.log
[ $rc -eq 0 ] || { echo "pytest failed rc=$rc"; exit $rc; }
for args in "--engine python" "--engine native" \
            "--engine python --force-dist" "--engine native --force-dist" \
            "--engine native --force-dist --algo ring"; do
  case "$args" in *force-dist*) L="$R";; *) L=python;; esac
  timeout -k 10 300 $L bench.py --steps 30 --warmup 5 $args > gpurun_out/bench_native.log 2>&1 ||
    { echo "bench failed: $args"; tail -20 gpurun_out/bench_native.log; exit 1; }
  echo "$args :: $(tail -1 gpurun_out/bench_native.log)"
done
