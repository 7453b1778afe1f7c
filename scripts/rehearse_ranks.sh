# one-GPU rehearsals of the driver's multi-rank command (N ranks time-share one GPU; not scaling data): the late
# round-6 tree end to end through the schedule A/B, gates and extras
set -e
mkdir -p gpurun_out/r6k
timeout -k 10 500 python3 bench.py --gpus 2 --steps 10 --warmup 3 > gpurun_out/r6k/g2.log 2>&1
timeout -k 10 600 python3 bench.py --gpus ${N4:-4} --steps 10 --warmup 3 > gpurun_out/r6k/g4.log 2>&1
for f in gpurun_out/r6k/g2.log gpurun_out/r6k/g4.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1) $(grep -o '"gates_failed": [^]]*]' $f | head -1)"; done
