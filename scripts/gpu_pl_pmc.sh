#!/bin/bash
# Colsum rework check (GEMM tests), then PMC counters of the pipelined GEMM kernel on fwd1 / bwdd1 / bwdw1 shapes
# (two passes; each within the per-block counter limits).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/plpmc
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py tests/test_gpu_gemm_ragged.py tests/test_gpu_prepack.py tests/test_gpu_native_engine.py -x -q --timeout 120 --timeout-method thread > gpurun_out/plpmc/pytest.log 2>&1; rc=$?
tail -3 gpurun_out/plpmc/pytest.log
[ $rc -eq 0 ] || exit $rc
B="python3 bench/gemm_bench.py --mb 8192 --shapes fwd1,bwdd1,bwdw1 --rounds 1 --iters 3"
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS -d gpurun_out/plpmc/p1 -o p --output-format csv -- $B > gpurun_out/plpmc/p1.log 2>&1 &&
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE TCC_HIT_sum TCC_MISS_sum TA_BUSY_avr TA_TA_BUSY_sum SQ_WAIT_ANY SQ_INSTS_VMEM SQ_ACTIVE_INST_ANY -d gpurun_out/plpmc/p2 -o p --output-format csv -- $B > gpurun_out/plpmc/p2.log 2>&1 &&
python3 tools/pmc_summary.py gpurun_out/plpmc/p1/p_counter_collection.csv gpurun_out/plpmc/p2/p_counter_collection.csv --filter gemm_pl > gpurun_out/plpmc/summary.txt && cat gpurun_out/plpmc/summary.txt
