# A/B: HIP-graph replay of the world-1 step (bench.py --graph: the step captured once after warmup, with the plans
# tuned in the eager steps before it) vs eager launches, MB 8192 and the reference batch MB 1792
set -e
mkdir -p gpurun_out/r6i
for r in 1 2 3; do
  for g in eager graph; do
    fl=""; [ $g = graph ] && fl="--graph"
    timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --extra-budget 0 --ref-mb 0 $fl > gpurun_out/r6i/b8192_${g}_r${r}.log 2>&1
    timeout -k 10 200 python3 bench.py --mb-per-gpu 1792 --ref-mb 0 --steps 100 --warmup 20 --extra-budget 0 $fl > gpurun_out/r6i/b1792_${g}_r${r}.log 2>&1
  done
done
for f in gpurun_out/r6i/*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1) $(grep -o '"hip_graph": [a-z]*' $f | head -1)"; done
