# Round-6 late check of the current tree on one box: GPU suite, smoke, the driver's N=1 command, and a kernel trace of
# the flagship and the MB 1792 step (per-kernel breakdown with tools/step_breakdown.py)
set -e
mkdir -p gpurun_out/r6g
export TMPDIR=/tmp
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/r6g/suite.log 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/r6g/smoke.log 2>&1
timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/r6g/bench_driver.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6g/prof8192 -o run --output-format csv -- python3 bench.py --steps 20 --warmup 5 --extra-budget 0 > gpurun_out/r6g/prof8192.log 2>&1
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/r6g/prof1792 -o run --output-format csv -- python3 bench.py --mb-per-gpu 1792 --ref-mb 0 --steps 20 --warmup 5 --extra-budget 0 > gpurun_out/r6g/prof1792.log 2>&1
tail -n 2 gpurun_out/r6g/suite.log; tail -n 1 gpurun_out/r6g/smoke.log
grep -o '"ms_per_step": [0-9.]*' gpurun_out/r6g/bench_driver.log | head -1
