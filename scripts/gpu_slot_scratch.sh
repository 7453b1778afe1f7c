#!/bin/bash
# Per-slot epilogue scratch (preallocated on first use): engine tests, flagship + multi-rank bench, the
# all-reduce bandwidth bench (256 MB payload) and the BERT overlap bench.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_native_loopback.py tests/test_gpu_native_engine.py > gpurun_out/ss_tests.log 2>&1 &&
tail -1 gpurun_out/ss_tests.log &&
timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 > gpurun_out/ss_inline.log 2>&1 && tail -1 gpurun_out/ss_inline.log | cut -c1-330 &&
timeout -k 10 200 python3 bench.py --steps 40 --warmup 3 --force-dist > gpurun_out/ss_fd.log 2>&1 && tail -1 gpurun_out/ss_fd.log | cut -c1-330 &&
timeout -k 10 300 python bench/allreduce_bw.py --variants bfp_mesh,bfp_ring,raw_mesh,rccl > gpurun_out/ss_allreduce_bw.log 2>&1 && grep bench gpurun_out/ss_allreduce_bw.log | cut -c1-300 &&
timeout -k 10 300 python bench/bert_overlap.py > gpurun_out/ss_bert.log 2>&1 && grep bench gpurun_out/ss_bert.log | cut -c1-300 &&
echo done
