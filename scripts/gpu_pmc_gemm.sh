#!/bin/bash
# PMC counters (two passes, each within the per-block slot limits) for the MLP GEMM shapes at MB ${MB:-8192}.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
S=${SHAPES:-fwd1}
MB=${MB:-8192}
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmc1 -o p --output-format csv -- python3 bench/gemm_bench.py --mb $MB --shapes $S --rounds 1 --iters 3 > gpurun_out/pmc1.log 2>&1 &&
timeout -k 10 300 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_ACTIVE_INST_LDS SQ_INSTS_MFMA SQ_ACTIVE_INST_ANY -d gpurun_out/pmc2 -o p --output-format csv -- python3 bench/gemm_bench.py --mb $MB --shapes $S --rounds 1 --iters 3 > gpurun_out/pmc2.log 2>&1 && echo pmc-done
