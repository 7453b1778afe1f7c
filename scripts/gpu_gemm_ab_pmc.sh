#!/bin/bash
# GEMM kernel tests, the one-role vs staggered main-loop A/B, then one PMC pass over both loops on two shapes.
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
export TMPDIR=/tmp
timeout -k 10 400 python -u -m pytest tests/test_gpu_kernels.py -x -q --timeout 120 --timeout-method thread \
  > gpurun_out/pytest_kernels.log 2>&1; rc=$?; tail -3 gpurun_out/pytest_kernels.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench/gemm_bench.py --mb ${MB:-8192} --ab --rounds 5 --shapes ${AB_SHAPES:-fwd0,fwd1,bwdw1,bwdd2,bwdd1,sq8k} \
  > gpurun_out/gemm_ab.log 2>&1; rc=$?
python - <<'PY'
import json
for l in open("gpurun_out/gemm_ab.log"):
    if l.startswith("{"):
        r = json.loads(l); print(r["shape"], "staggered", r["mine_us"], "oneloop", r.get("oneloop_us"), "hipblaslt", r["torch_matmul_only_us"])
PY
[ $rc -eq 0 ] || exit $rc
timeout -s KILL 120 rocprofv3 --pmc GRBM_GUI_ACTIVE SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_VALU_MFMA_BUSY_CYCLES SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT -d gpurun_out/pmcab -o p --output-format csv -- python3 bench/gemm_bench.py --mb ${MB:-8192} --ab --shapes bwdd1,fwd1 --rounds 1 --iters 3 > gpurun_out/pmcab.log 2>&1 &&
python tools/pmc_summary.py gpurun_out/pmcab/p_counter_collection.csv --filter gemm > gpurun_out/pmcab_summary.txt && echo pmc-done
