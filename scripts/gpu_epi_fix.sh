#!/bin/bash
# Null-stream commit fix check: the engine treated torch's default stream (handle 0) as "no producer", so
# a committed epilogue was NOT ordered after the producer's work. After the fix: race/determinism probes,
# the engine tests (the comm-stream test should now pass), and the epilogue-placement A/B on the forced
# 1-rank RCCL path (arms alternated on one box).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest -x -q -rxX --timeout 120 --timeout-method thread \
  tests/test_gpu_native_loopback.py tests/test_gpu_native_engine.py > gpurun_out/fix_tests.log 2>&1 &&
tail -4 gpurun_out/fix_tests.log &&
timeout -k 10 200 python3 -u tools/probes/race_probe.py 1 producer,comm > gpurun_out/fix_race.log 2>&1 && cat gpurun_out/fix_race.log &&
timeout -k 10 300 python3 -u tools/probes/determinism_probe.py > gpurun_out/fix_det.log 2>&1 && cat gpurun_out/fix_det.log &&
for rep in 1 2 3; do
  for arm in comm producer; do
    timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 --force-dist --epi $arm > gpurun_out/fix_${arm}_$rep.log 2>&1 || exit 1
    echo "$arm $rep $(tail -1 gpurun_out/fix_${arm}_$rep.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')"
  done
done &&
timeout -k 10 200 python3 bench.py --steps 40 --warmup 10 > gpurun_out/fix_inline.log 2>&1 &&
echo "inline $(tail -1 gpurun_out/fix_inline.log | python3 -c 'import json,sys; r=json.loads(sys.stdin.read()); print(r["value"], r["ms_per_step"])')" &&
echo done
