#!/bin/bash
# In-step plan A/B after the 3-stage 256x128 kernel: default vs narrow bwd-weight on 256x128 split 2, vs the K-1024
# 8192x4096 GEMMs (forward of fc0, bwd-data of fc2) on 256x128 tiles. Alternated, same box.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/planab3
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
for arm in default bwdw128 k1024_128; do
case $arm in
default) unset FAN_GEMM_PLAN;;
bwdw128) export FAN_GEMM_PLAN="1024x4096x8192=256,128,2;4096x1024x8192=256,128,2";;
k1024_128) export FAN_GEMM_PLAN="8192x4096x1024=256,128,1";;
esac
timeout -k 10 200 python bench.py --ref-mb 0 --steps 40 > $O/b_${arm}_$i.jsonl 2>/dev/null || exit 1
echo "$arm $(tail -1 $O/b_${arm}_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
done
