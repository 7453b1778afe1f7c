#!/bin/bash
# Same-box A/B of two builds of the extension: alternates abso/_C_<a>.so and abso/_C_<b>.so into place and runs
# the flagship bench with each (separate processes, interleaved rounds). Usage: scripts/gpu_so_ab.sh a b [rounds]
set -e
A=$1; B=$2; R=${3:-3}
mkdir -p gpurun_out
cp fpga_ai_nic_amd/_C.so /tmp/_C_orig.so
for r in $(seq 1 $R); do
  for v in $A $B; do
    cp abso/_C_$v.so fpga_ai_nic_amd/_C.so
    echo -n "$v round $r: " | tee -a gpurun_out/so_ab.log
    timeout -k 10 300 python bench.py --steps 40 --warmup 10 | tee -a gpurun_out/so_ab.log
  done
done
cp /tmp/_C_orig.so fpga_ai_nic_amd/_C.so
