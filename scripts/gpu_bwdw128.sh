#!/bin/bash
# bwd-weight 4096^2 (K 8192, BFP wire + bias-gradient epilogue) on 3-stage 256x128 tiles of the 4-wave kernel vs the
# default 256x256 8-wave pipelined kernel: wire numerics, then the flagship alternated (FAN_GEMM_PLAN).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/bwdw128
mkdir -p $O
export TMPDIR=/tmp
timeout -k 10 300 python -u -m pytest tests/test_gpu_prepack.py tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread > $O/pytest.log 2>&1; rc=$?
tail -2 $O/pytest.log
[ $rc -eq 0 ] || { grep -E "Error|assert" $O/pytest.log | head -8; exit $rc; }
for i in 1 2 3; do
for arm in default w128; do
if [ $arm = default ]; then unset FAN_GEMM_PLAN; else export FAN_GEMM_PLAN="4096x4096x8192=256,128,1"; fi
timeout -k 10 200 python bench.py --ref-mb 0 --steps 40 > $O/b_${arm}_$i.jsonl 2>/dev/null || exit 1
echo "$arm $(tail -1 $O/b_${arm}_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
done
