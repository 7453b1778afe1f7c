#!/bin/bash
# Throughput vs per-GPU minibatch for the flagship bench (1 GPU).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for mb in ${MBS:-1024 2048 4096 8192 16384}; do
  timeout -k 10 300 python bench.py --steps 30 --warmup 5 --mb-per-gpu $mb "$@" > gpurun_out/mb_$mb.log 2>&1 || { tail -20 gpurun_out/mb_$mb.log; exit 1; }
  python3 -c "import json;d=json.loads(open('gpurun_out/mb_$mb.log').read().strip().splitlines()[-1]);print('mb', $mb, d['ms_per_step'], d['value'], d['extra']['achieved_tflops'])"
done
