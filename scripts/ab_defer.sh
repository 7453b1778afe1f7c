# A/B: deferred bias-gradient reduces (FAN_DEFER_COLSUM) on the flagship (MB 8192) and the reference batch (MB 1792)
set -e
mkdir -p gpurun_out/r6d
timeout -k 10 240 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_defer_colsum.py tests/test_gpu_fused_update.py > gpurun_out/r6d/tests.log 2>&1
for r in 1 2; do
  for d in 1 0; do
    FAN_DEFER_COLSUM=$d timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --extra-budget 0 > gpurun_out/r6d/b8192_d${d}_r${r}.log 2>&1
    FAN_DEFER_COLSUM=$d timeout -k 10 200 python3 bench.py --mb-per-gpu 1792 --ref-mb 0 --steps 100 --warmup 20 --extra-budget 0 > gpurun_out/r6d/b1792_d${d}_r${r}.log 2>&1
  done
done
for f in gpurun_out/r6d/b*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1)"; done
