#!/bin/bash
# Persistent GEMM beside concurrent comm kernels: the forced multi-rank path (1-rank RCCL group, side-stream engine)
# with FAN_GEMM_PERSIST=256 vs 0, alternated; plus the bwd-weight epilogue arms at MB 8192.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
O=gpurun_out/persistfd
mkdir -p $O
export TMPDIR=/tmp
for i in 1 2 3; do
for c in 256 0; do
FAN_GEMM_PERSIST=$c timeout -k 10 200 python bench.py --ref-mb 0 --steps 30 --force-dist > $O/fd_${c}_$i.jsonl 2>/dev/null || exit 1
echo "forced persist=$c $(tail -1 $O/fd_${c}_$i.jsonl | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); print(d["ms_per_step"])')"
done
done
timeout -k 10 300 python bench/gemm_bench.py --mb 8192 --epi-arms --rounds 5 --shapes bwdw1 > $O/arms.jsonl 2>&1 && grep '^{' $O/arms.jsonl | cut -c1-600
