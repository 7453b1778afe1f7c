#!/bin/bash
# Two ranks sharing one MI355X over the direct P2P transport (control plane gloo): the flagship bench through the
# direct mesh path (device-timed comm phases in extra.allreduce) and a kernel trace showing the direct kernels.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
FAN_CTRL_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --transport p2p --steps 10 --warmup 3 \
  --mb-per-gpu 2048 > gpurun_out/bench_p2p2.log 2>&1 || { tail -30 gpurun_out/bench_p2p2.log; exit 1; }
grep metric gpurun_out/bench_p2p2.log | cut -c1-1500
FAN_CTRL_BACKEND=gloo timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_p2p -o run --output-format csv -- python3 -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29562 bench.py --gpus 2 --transport p2p --steps 5 --warmup 2 --ref-mb 0 \
  --mb-per-gpu 2048 > gpurun_out/prof_p2p.log 2>&1 || { tail -20 gpurun_out/prof_p2p.log; exit 1; }
find gpurun_out/prof_p2p -name "*kernel_stats.csv" | head -3
