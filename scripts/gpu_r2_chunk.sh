#!/bin/bash
# Chunked mesh pipeline: new tests first, then the full suite, flagship bench and the config-4 sweep (256 MB -> 8 chunks).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_native_loopback.py tests/test_gpu_native_engine.py -x -v --timeout 200 --timeout-method thread -k "chunk or one_gib or trains_like" > gpurun_out/pytest_chunk.log 2>&1; rc=$?
grep -E "PASS|FAIL|ERROR|passed|failed|Error" gpurun_out/pytest_chunk.log | tail -30
[ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1; rc=$?
tail -3 gpurun_out/pytest_gpu.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python bench.py --steps 20 --warmup 5 > gpurun_out/bench.log 2>&1 && tail -1 gpurun_out/bench.log | cut -c1-300 &&
FAN_CHUNK_ELEMS=8388608 timeout -k 10 400 python bench/allreduce_bw.py --sizes-mb 64,256 --variants bfp_mesh,raw_mesh --iters 5 --rounds 3 > gpurun_out/allreduce_bw_chunked.jsonl 2>gpurun_out/allreduce_bw_chunked.err && cat gpurun_out/allreduce_bw_chunked.jsonl | cut -c1-420
