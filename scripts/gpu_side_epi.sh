#!/bin/bash
# World-1 side-stream epilogue (FAN_SIDE_EPI=1): engine / trainer GPU tests with it on, then the flagship bench
# A/B against the in-order epilogue, alternated.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/sepi
export TMPDIR=/tmp
FAN_SIDE_EPI=1 timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/sepi/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/sepi/pytest.log
[ $rc -eq 0 ] || { grep -E "^(FAILED|ERROR)" gpurun_out/sepi/pytest.log | head; exit $rc; }
for i in 1 2 3; do
FAN_SIDE_EPI=1 timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/sepi/b_side_$i.log 2>&1 && echo "side $(tail -1 gpurun_out/sepi/b_side_$i.log | cut -c1-200)" &&
timeout -k 10 300 python bench.py --steps 30 --warmup 5 > gpurun_out/sepi/b_inorder_$i.log 2>&1 && echo "inorder $(tail -1 gpurun_out/sepi/b_inorder_$i.log | cut -c1-200)" || exit 1
done
