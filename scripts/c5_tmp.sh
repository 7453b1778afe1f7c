set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/c5; mkdir -p $O
timeout -k 10 60 rocprofv3 -L > $O/counters.txt 2>&1; echo L_rc=$?
timeout -k 10 700 python -u -m pytest tests -m gpu -q --timeout 240 --timeout-method thread -rf -s > $O/test.log 2>&1; echo test_rc=$?; tail -4 $O/test.log
timeout -k 10 400 python bench.py --gpus 2 --steps 10 --warmup 3 --ref-mb 0 --timeout 200 > $O/b2.jsonl 2> $O/b2.err; echo b2_rc=$?
GPU_MAX_HW_QUEUES=32 timeout -k 10 300 python -u tools/probes/ring_hops_local.py --world 8 --size-mb 64 --arms ring:1,ring:7,ring:7:3,mesh:1 > $O/ring_hops8.jsonl 2> $O/ring_hops8.err; echo hops_rc=$?
timeout -k 10 200 python bench/bert_overlap.py > $O/bert.jsonl 2> $O/bert.err; echo bert_rc=$?
for k in compute comm overlap; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_$k -o run --output-format csv -- python3 bench/bert_overlap.py --only $k --rounds 3 > $O/bert_$k.log 2>&1 || { echo prof_$k failed; exit 1; }
done
timeout -s KILL 120 rocprofv3 --kernel-trace --pmc SQ_INSTS_MFMA SQ_INSTS_VALU_MFMA_MOPS_BF16 SQ_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc1 -o p --output-format csv -- python3 bench.py --steps 5 --warmup 2 --ref-mb 0 --extra-budget 0 > $O/pmc1.log 2>&1; echo pmc_rc=$?
f=$(find $O/pmc1 -name '*counter_collection.csv' | head -1); [ -n "$f" ] && python tools/pmc_summary.py "$f" --table > $O/mfma_table.txt 2>&1; head -30 $O/mfma_table.txt
python tools/overlap_attrib.py $(find $O/prof_compute -name '*kernel_trace.csv' | head -1) $(find $O/prof_comm -name '*kernel_trace.csv' | head -1) $(find $O/prof_overlap -name '*kernel_trace.csv' | head -1) > $O/overlap_attrib.txt 2>&1; head -40 $O/overlap_attrib.txt
echo done
