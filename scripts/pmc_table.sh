# MFMA utilisation table of the final tree: one rocprofv3 --pmc pass per counter group over a short world-1 run
# (flagship and the MB 1792 cell), summarised by tools/pmc_summary.py --table
set -e
mkdir -p gpurun_out/r6q
export TMPDIR=/tmp
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_MFMA GRBM_GUI_ACTIVE -d gpurun_out/r6q/p1 -o p1 --output-format csv -- python3 bench.py --steps 5 --warmup 2 --extra-budget 0 > gpurun_out/r6q/p1.log 2>&1
timeout -s KILL 120 rocprofv3 --pmc SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES -d gpurun_out/r6q/p2 -o p2 --output-format csv -- python3 bench.py --steps 5 --warmup 2 --extra-budget 0 > gpurun_out/r6q/p2.log 2>&1
ls gpurun_out/r6q/p1 gpurun_out/r6q/p2
