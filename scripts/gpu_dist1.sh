#!/bin/bash
# Exercise the multi-rank code path on one GPU: 1-rank RCCL process group, side-stream engine, real collectives.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
R="python -m torch.distributed.run --nnodes 1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29541"
timeout -k 10 240 python bench.py --steps 30 --warmup 5 > gpurun_out/d1_inline.log 2>&1 && tail -1 gpurun_out/d1_inline.log | cut -c1-160 &&
timeout -k 10 240 $R bench.py --steps 30 --warmup 5 --force-dist > gpurun_out/d1_torch.log 2>&1 && grep metric gpurun_out/d1_torch.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('torch-dist', d['ms_per_step'], d['extra'])" &&
timeout -k 10 240 $R bench.py --steps 30 --warmup 5 --force-dist --transport native > gpurun_out/d1_native.log 2>&1 && grep metric gpurun_out/d1_native.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('native', d['ms_per_step'], d['extra'])" &&
timeout -k 10 240 $R bench.py --steps 30 --warmup 5 --force-dist --compress rccl > gpurun_out/d1_rccl.log 2>&1 && grep metric gpurun_out/d1_rccl.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('rccl-baseline', d['ms_per_step'], d['extra'])" &&
timeout -k 10 240 $R bench.py --steps 30 --warmup 5 --force-dist --algo ring --rings 1 > gpurun_out/d1_ring.log 2>&1 && grep metric gpurun_out/d1_ring.log | python3 -c "import json,sys;d=json.loads(sys.stdin.read());print('ring', d['ms_per_step'], d['extra'])"
