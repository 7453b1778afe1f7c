#!/bin/bash
# Engine checks: new native verify/fault tests + P2P abort first (fast fail), the full GPU suite, the flagship bench,
# and the config-4 all-reduce sweep on the production engine (world 1 through the 1-rank RCCL path).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_faults_verify.py tests/test_gpu_p2p.py tests/test_gpu_native_engine.py -x -v --timeout 150 --timeout-method thread > gpurun_out/pytest_engine.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed" gpurun_out/pytest_engine.log | tail -40
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-400 &&
timeout -k 10 400 python bench/allreduce_bw.py --sizes-mb 4,16,64,256 --iters 5 --rounds 3 > gpurun_out/allreduce_bw_1gpu.jsonl 2>gpurun_out/allreduce_bw_1gpu.err && cat gpurun_out/allreduce_bw_1gpu.jsonl | cut -c1-420
