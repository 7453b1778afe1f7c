# one-GPU rehearsal of the driver's command at the reference's own world size (3 ranks, sw/run.sh: mpirun -n 3)
set -e
mkdir -p gpurun_out/r6o
timeout -k 10 600 python3 bench.py --gpus 3 --steps 10 --warmup 3 > gpurun_out/r6o/g3.log 2>&1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6o/g3.log | head -1; grep -o '"gates_failed": [^]]*]' gpurun_out/r6o/g3.log | head -1
