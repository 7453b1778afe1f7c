#!/bin/bash
# A/B helper: bench.py from the working tree vs a copy of it that loads gpurun_ab/_C_prev.so (a previous build:
# copy fpga_ai_nic_amd/_C.so there before rebuilding; delete it afterwards, every gpurun call uploads it).
# usage (on the GPU box): bash scripts/ab_prev.sh OUTDIR ROUNDS bench-args...
set -u
out=$1; rounds=$2; shift 2
mkdir -p "$out"
prev=$(mktemp -d)
cp -r fpga_ai_nic_amd bench.py "$prev"/ && cp gpurun_ab/_C_prev.so "$prev"/fpga_ai_nic_amd/_C.so || exit 1
for r in $(seq 1 "$rounds"); do
  for arm in new prev; do
    dir=.; [ "$arm" = prev ] && dir=$prev
    ( cd "$dir" && timeout -k 10 300 python bench.py "$@" ) > "$out/ab_${arm}_$r.jsonl" 2> "$out/ab_${arm}_$r.err"
    rc=$?; echo "[ab] $arm $r rc=$rc $(grep -h '^{' "$out/ab_${arm}_$r.jsonl" | python3 -c 'import sys,json; [print(json.loads(l)["ms_per_step"]) for l in sys.stdin]')"
    [ $rc -eq 0 ] || exit $rc
  done
done
