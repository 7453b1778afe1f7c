#!/bin/bash
# Engine debug snapshot + P2P device stall counters: the P2P and engine GPU tests, then the whole GPU suite.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/dbg
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_p2p.py tests/test_gpu_native_engine.py -x -v --timeout 200 --timeout-method thread > gpurun_out/dbg/pytest_dbg.log 2>&1; rc=$?
grep -E "PASS|FAIL|Error" gpurun_out/dbg/pytest_dbg.log | tail -12
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/dbg/pytest_gpu.log 2>&1; rc=$?
tail -2 gpurun_out/dbg/pytest_gpu.log; exit $rc
