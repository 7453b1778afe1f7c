#!/bin/bash
# 256x128 tiles on the 4-wave pipelined loop: numerics (all layouts, split-K, colsum) then shapes whose 256x256 grid
# would be half empty (fwd2, BERT ffn/qkv) with the 256x128 plan forced: pipelined (2) vs one-role (0).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/p128
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -q -k "256x128 or 256_tile" --timeout 120 --timeout-method thread > gpurun_out/p128/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/p128/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" gpurun_out/p128/pytest.log | head -5; exit $rc; }
FAN_GEMM_PLAN="8192x1024x4096=256,128,1;4096x4096x8192=256,128,2" timeout -k 10 300 python bench/gemm_bench.py --mb 8192 --loops 0 --shapes fwd2,bwdw1 > gpurun_out/p128/mlp.jsonl 2>&1 &&
FAN_GEMM_PLAN="4096x768x3072=256,128,1;4096x2304x768=256,128,1" timeout -k 10 300 python bench/gemm_bench.py --set bert --mb 4096 --loops 0 > gpurun_out/p128/bert.jsonl 2>&1 &&
python3 - <<'PY'
import json
for f in ("gpurun_out/p128/mlp.jsonl", "gpurun_out/p128/bert.jsonl"):
    for l in open(f):
        if l.startswith('{'):
            d = json.loads(l); print(d['shape'], d['plan'], 'mine', d['mine_us'], 'loops', d.get('loop_us'), 'torch', d['torch_matmul_only_us'])
PY
