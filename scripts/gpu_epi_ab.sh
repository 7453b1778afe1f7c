#!/bin/bash
# A/B of where the side-stream engine runs its decode+SGD epilogues (forced 1-rank RCCL path, one box, arms
# alternated): on the comm stream, overlapped with the rest of the backward (--epi comm), or on the compute
# stream after the last backward GEMM (--epi producer). Inline world-1 arm for reference. Then the new tests.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread \
  tests/test_gpu_native_loopback.py tests/test_gpu_native_engine.py > gpurun_out/epi_tests.log 2>&1 &&
tail -2 gpurun_out/epi_tests.log &&
for rep in 1 2 3; do
  for arm in comm producer; do
    timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --force-dist --epi $arm > gpurun_out/epi_${arm}_$rep.log 2>&1 || exit 1
    echo "$arm $rep $(tail -1 gpurun_out/epi_${arm}_$rep.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  done
done &&
timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 > gpurun_out/epi_inline.log 2>&1 &&
echo "inline $(tail -1 gpurun_out/epi_inline.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')" &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_epi_prod -o p --output-format csv -- python3 bench.py --steps 20 --warmup 5 --force-dist --epi producer > gpurun_out/prof_epi_prod.log 2>&1 &&
echo done
