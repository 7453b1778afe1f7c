#!/bin/bash
# Multi-rank GPU validation on ONE MI355X: P2P transport tests (2 processes), then the flagship bench with
# 2 ranks sharing the GPU (control plane over gloo, gradient plane over HIP-IPC P2P). Functional, not perf.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 400 python -m pytest tests/test_gpu_p2p.py -x -q > gpurun_out/pytest_p2p.log 2>&1; rc=$?
tail -5 gpurun_out/pytest_p2p.log
[ $rc -eq 0 ] || { tail -40 gpurun_out/pytest_p2p.log; exit $rc; }
FAN_CTRL_BACKEND=gloo timeout -k 10 300 python -m torch.distributed.run --nnodes 1 --nproc-per-node 2 \
  --master-addr 127.0.0.1 --master-port 29561 bench.py --gpus 2 --transport p2p --steps 10 --warmup 3 \
  --mb-per-gpu 2048 > gpurun_out/bench_p2p2.log 2>&1 || { tail -30 gpurun_out/bench_p2p2.log; exit 1; }
grep metric gpurun_out/bench_p2p2.log | cut -c1-400
