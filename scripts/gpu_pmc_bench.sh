#!/bin/bash
# PMC counters over the flagship bench step (3 passes, each within the per-block counter-slot limits).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
B="python3 bench.py --steps 5 --warmup 2 ${BENCH_ARGS:-}"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmcb1 -o p --output-format csv -- $B > gpurun_out/pmcb1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE FETCH_SIZE -d gpurun_out/pmcb2 -o p --output-format csv -- $B > gpurun_out/pmcb2.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE WRITE_SIZE TCC_HIT_sum -d gpurun_out/pmcb3 -o p --output-format csv -- $B > gpurun_out/pmcb3.log 2>&1 &&
python3 tools/pmc_summary.py gpurun_out/pmcb1/p_counter_collection.csv gpurun_out/pmcb2/p_counter_collection.csv gpurun_out/pmcb3/p_counter_collection.csv > gpurun_out/pmc_bench_summary.txt && echo pmc-done
