#!/bin/bash
# Component benches on one GPU: all-reduce codec throughput, BERT overlap, GEMMs vs hipBLASLt.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 300 python bench/allreduce_bw.py --variants bfp_mesh,bfp_ring,raw_mesh,rccl > gpurun_out/allreduce_bw.log 2>&1 && cat gpurun_out/allreduce_bw.log | grep bench &&
timeout -k 10 300 python bench/bert_overlap.py > gpurun_out/bert_overlap.log 2>&1 && grep bench gpurun_out/bert_overlap.log &&
timeout -k 10 300 python -m fpga_ai_nic_amd.cli.mlp_mpi 20 5376 0 A 32 32 32 2048 2048 2048 2048 2048 2048 2048 2048 2048 2048 2048 --dtype f32 --profile > gpurun_out/mlp_ref_f32.log 2>&1 && grep -E "GFLOP|fp time|PERFDUMP|SAMPLES|LOSS|Bwdupd|FC time" gpurun_out/mlp_ref_f32.log
