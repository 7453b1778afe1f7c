#!/bin/bash
# 4-wave AGPR pipelined loop (gemm_set_main_loop(3)): numerics on every layout, then in-process timings vs the
# 8-wave pipelined loop (2) and hipBLASLt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pl4
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_kernels.py -x -v -k "256_tile" --timeout 120 --timeout-method thread > gpurun_out/pl4/pytest.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error|error" gpurun_out/pl4/pytest.log | tail -8
[ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python bench/gemm_bench.py --mb 8192 --loops 2,3,4 --shapes fwd0,fwd1,fwd2,bwdw2,bwdw1,bwdd2,bwdd1,sq8k > gpurun_out/pl4/gemm.jsonl 2>&1 && python3 - <<'PY'
import json
for l in open('gpurun_out/pl4/gemm.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print(d['shape'], d['plan'], 'default', d['mine_us'], 'loops', d.get('loop_us'), 'torch', d['torch_matmul_only_us'])
PY
