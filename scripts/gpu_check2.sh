#!/bin/bash
# Full GPU test suite, then bench with both request paths, then the reference f32 workload via mlp_mpi.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
if [ -n "$(find csrc -newer fpga_ai_nic_amd/_C.so -type f 2>/dev/null)" ] || [ ! -f fpga_ai_nic_amd/_C.so ]; then
  echo "[gpu_check2] _C.so is stale or missing: rebuilding"; python tools/build_ext.py -j 16 || exit 1
fi
timeout -k 10 900 python -m pytest tests -m gpu -x -q > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_gpu.log; exit $rc; }
for e in "--engine python" "--engine native" "--engine native --graph" "--engine python --graph" "--engine native"; do
  timeout -k 10 300 python bench.py --steps 50 --warmup 10 $e > gpurun_out/bench_x.log 2>&1 || { tail -20 gpurun_out/bench_x.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/bench_x.log').read().strip().splitlines()[-1]);print('$e', d['ms_per_step'], d['value'], d['config']['hip_graph'], d['extra']['host_enqueue_ms_per_step'], d['extra']['final_loss'])"
done
timeout -k 10 300 python -m fpga_ai_nic_amd.cli.mlp_mpi 20 5376 0 A 32 32 32 2048 2048 2048 2048 2048 2048 2048 2048 2048 2048 2048 --dtype f32 --warmup 3 > gpurun_out/mlp_ref_f32.log 2>&1 && grep -E "GFLOPS|fp time|SAMPLES" gpurun_out/mlp_ref_f32.log
