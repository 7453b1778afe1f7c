# kernel traces of the world-1 step: plain (fused update) and through the multi-rank path with the sharded update
set -e
mkdir -p gpurun_out/r6j
export TMPDIR=/tmp
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r6j/plain -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --extra-budget 0 --ref-mb 0 --no-trace > gpurun_out/r6j/plain.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace -d gpurun_out/r6j/forced -o run --output-format csv -- python3 bench.py --force-dist --shard-update 1 --schedule fixed --steps 20 --warmup 5 --extra-budget 0 --ref-mb 0 --no-trace > gpurun_out/r6j/forced.log 2>&1
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6j/plain.log gpurun_out/r6j/forced.log
