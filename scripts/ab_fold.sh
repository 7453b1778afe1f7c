# A/B: split-K classifier GEMM folded into the softmax-xent kernel (FAN_FOLD_LOGITS) at MB 1792 / 8192, after its
# bit-identity tests
set -e
mkdir -p gpurun_out/r6f${AB_TAG}
timeout -k 10 240 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fold_logits.py tests/test_gpu_defer_colsum.py tests/test_gpu_fused_update.py > gpurun_out/r6f${AB_TAG}/tests.log 2>&1
for r in 1 2 3; do
  for d in 1 0; do
    FAN_FOLD_LOGITS=$d timeout -k 10 200 python3 bench.py --mb-per-gpu 1792 --ref-mb 0 --steps 100 --warmup 20 --extra-budget 0 > gpurun_out/r6f${AB_TAG}/b1792_f${d}_r${r}.log 2>&1
  done
done
FAN_FOLD_LOGITS=1 timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --extra-budget 0 > gpurun_out/r6f${AB_TAG}/b8192_f1.log 2>&1
for f in gpurun_out/r6f${AB_TAG}/b*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1)"; done
