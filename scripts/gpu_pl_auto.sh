#!/bin/bash
# Pipelined loop with per-layout 4/8-wave selection: whole GPU suite, GEMM timings (auto vs forced 8-wave vs
# forced 4-wave), flagship bench alternated with the 8-wave-only loop.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/plauto
export TMPDIR=/tmp
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/plauto/pytest.log 2>&1; rc=$?
tail -2 gpurun_out/plauto/pytest.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/plauto/pytest.log | head; exit $rc; }
timeout -k 10 400 python bench/gemm_bench.py --mb 8192 --loops 5,3 --epi-arms > gpurun_out/plauto/gemm.jsonl 2>&1 && python3 - <<'PY'
import json
for l in open('gpurun_out/plauto/gemm.jsonl'):
    if l.startswith('{'):
        d = json.loads(l); print(d['shape'], d['plan'], 'auto', d['mine_us'], 'loops', d.get('loop_us'), 'torch', d['torch_matmul_only_us'], d.get('epi_arms_us', ''))
PY
for i in 1 2; do
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/plauto/b_auto_$i.log 2>&1 && echo "auto $(tail -1 gpurun_out/plauto/b_auto_$i.log | cut -c150-230)" &&
FAN_GEMM_PL=5 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/plauto/b_pl8_$i.log 2>&1 && echo "pl8 $(tail -1 gpurun_out/plauto/b_pl8_$i.log | cut -c150-230)" || exit 1
done
