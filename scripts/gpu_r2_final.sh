#!/bin/bash
# Round-2 measurement set for the docs: flagship bench (3 runs), its kernel statistics, GEMMs vs hipBLASLt at
# MB 8192 (MLP shapes, default main-loop selection), PMC pass over the flagship step.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/final
export TMPDIR=/tmp
for i in 1 2 3; do
timeout -k 10 300 python bench.py > gpurun_out/final/bench_$i.jsonl 2>gpurun_out/final/bench_$i.err && tail -1 gpurun_out/final/bench_$i.jsonl | cut -c1-260 || exit 1
done
timeout -k 10 400 python bench/gemm_bench.py --mb 8192 > gpurun_out/final/gemm_mlp8192.jsonl 2>&1 &&
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/final/prof -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --ref-mb 0 > gpurun_out/final/prof.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/final/pmc1 -o p --output-format csv -- python3 bench.py --steps 5 --warmup 2 --ref-mb 0 > gpurun_out/final/pmc1.log 2>&1 &&
python3 tools/pmc_summary.py gpurun_out/final/pmc1/p_counter_collection.csv --filter gemm > gpurun_out/final/pmc_summary.txt && echo done
