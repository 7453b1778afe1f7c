#!/bin/bash
# MI355X equivalent of the reference sw/run.sh workload: 10 FC layers of 2048, f32, global MB 5376, 20 iterations,
# one process per GPU (NGPUS defaults to all visible GPUs). Extra args are passed through (e.g. --compress rccl).
NGPUS=${NGPUS:-$(python -c "import torch;print(max(1,torch.cuda.device_count()))")}
cd "$(dirname "$0")/.."
python -m torch.distributed.run --nnodes 1 --nproc-per-node "$NGPUS" --master-addr 127.0.0.1 \
  --master-port "${MASTER_PORT:-29531}" -m fpga_ai_nic_amd.cli.mlp_mpi \
  20 5376 0 A 32 32 32 2048 2048 2048 2048 2048 2048 2048 2048 2048 2048 2048 --dtype f32 --profile "$@"
