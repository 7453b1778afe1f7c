set -o pipefail
cd "${GRAFT_REPO_ROOT:-.}"
export TMPDIR=/tmp
O=gpurun_out/c7; mkdir -p $O
for k in compute comm overlap; do
  timeout -k 10 200 rocprofv3 --kernel-trace -d $O/prof_$k -o run --output-format csv -- python3 bench/bert_overlap.py --only $k --rounds 3 > $O/bert_$k.log 2>&1 || { echo prof_$k failed; exit 1; }
done
python tools/overlap_attrib.py $(find $O/prof_compute -name '*kernel_trace.csv' | head -1) $(find $O/prof_comm -name '*kernel_trace.csv' | head -1) $(find $O/prof_overlap -name '*kernel_trace.csv' | head -1) > $O/overlap_attrib.txt 2>&1; cat $O/overlap_attrib.txt
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_flag -o run --output-format csv -- python3 bench.py --steps 20 --warmup 3 --ref-mb 0 --extra-budget 0 > $O/prof_flag.log 2>&1; echo prof_rc=$?
python tools/step_breakdown.py $(find $O/prof_flag -name '*kernel_trace.csv' | head -1) --steps 20 > $O/step_breakdown.txt 2>&1; head -30 $O/step_breakdown.txt
for i in 1 2; do timeout -k 10 200 python bench.py > $O/b1_$i.jsonl 2> $O/b1_$i.err; echo b1_rc=$?; done
FAN_VERIFY=1 timeout -k 10 400 python bench.py --gpus 2 --steps 5 --warmup 2 --ref-mb 0 --extra-budget 0 --mb-per-gpu 2048 --timeout 200 > $O/b2_verify.jsonl 2> $O/b2_verify.err; echo b2v_rc=$?
echo done
