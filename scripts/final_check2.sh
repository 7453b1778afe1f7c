# End-of-round check of the final tree on one box: GPU suite, smoke, the driver's N=1 command three times
set -e
mkdir -p gpurun_out/${OUT_DIR:-r6n}
timeout -k 10 600 python3 -u -m pytest tests -m gpu -x -q --timeout 120 --timeout-method thread > gpurun_out/${OUT_DIR:-r6n}/suite.log 2>&1
timeout -k 10 200 python3 -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/${OUT_DIR:-r6n}/smoke.log 2>&1
for r in 1 2 3; do
  timeout -k 10 400 python3 bench.py --steps 20 --warmup 5 > gpurun_out/${OUT_DIR:-r6n}/bench_driver_r$r.log 2>&1
done
tail -n 1 gpurun_out/${OUT_DIR:-r6n}/suite.log; tail -n 1 gpurun_out/${OUT_DIR:-r6n}/smoke.log
for r in 1 2 3; do grep -o '"ms_per_step": [0-9.]*' gpurun_out/${OUT_DIR:-r6n}/bench_driver_r$r.log | head -2 | tr '\n' ' '; echo; done
