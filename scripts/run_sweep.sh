#!/bin/bash
# The reference's commented sweep (sw/run.sh:17-36): MB per node in {1792, 448}, 21 feature sizes of 2048,
# BFP on/off, logged per config under ./log/<ngpus>_<mode>_<mb>.log
cd "$(dirname "$0")/.."
mkdir -p log
NGPUS=${NGPUS:-$(python -c "import torch;print(max(1,torch.cuda.device_count()))")}
C=$(python -c "print(' '.join(['2048']*21))")
for mb in 1792 448; do
  for mode in bfp rccl; do
    python -m torch.distributed.run --nnodes 1 --nproc-per-node "$NGPUS" --master-addr 127.0.0.1 \
      --master-port "${MASTER_PORT:-29532}" -m fpga_ai_nic_amd.cli.mlp_mpi \
      20 $((mb * NGPUS)) 0 A 32 32 32 $C --dtype f32 --compress $mode > "log/${NGPUS}_${mode}_${mb}.log" 2>&1
    grep PERFDUMP "log/${NGPUS}_${mode}_${mb}.log"
  done
done
