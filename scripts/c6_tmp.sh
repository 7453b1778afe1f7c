set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/c6; mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_e2e_numerics.py -q -s --timeout 280 --timeout-method thread > $O/e2e.log 2>&1; echo e2e_rc=$?; grep -E "passed|failed|per step|trajectory" $O/e2e.log
for k in compute comm overlap; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_$k -o run --output-format csv -- python3 bench/bert_overlap.py --only $k --rounds 3 > $O/bert_$k.log 2>&1 || { echo prof_$k failed; exit 1; }
done
python tools/overlap_attrib.py $(find $O/prof_compute -name '*kernel_trace.csv' | head -1) $(find $O/prof_comm -name '*kernel_trace.csv' | head -1) $(find $O/prof_overlap -name '*kernel_trace.csv' | head -1) > $O/overlap_attrib.txt 2>&1; head -40 $O/overlap_attrib.txt
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc1 -o p --output-format csv -- python3 bench.py --steps 5 --warmup 2 --ref-mb 0 --extra-budget 0 > $O/pmc1.log 2>&1; echo pmc_rc=$?
f=$(find $O/pmc1 -name '*counter_collection.csv' | head -1); [ -n "$f" ] && python tools/pmc_summary.py "$f" --table > $O/mfma_table.txt 2>&1; head -30 $O/mfma_table.txt
echo done
