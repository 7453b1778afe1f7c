# A/B: the MB 8192 classifier GEMM (8192x1024x4096, f32 logits + bias) on 256x128 unsplit tiles (default) vs
# 256x256 tiles split 2 / 4 now that the softmax folds the split-K slabs (FAN_FOLD_LOGITS default on)
set -e
mkdir -p gpurun_out/r6h
for r in 1 2 3; do
  timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --extra-budget 0 > gpurun_out/r6h/def_r${r}.log 2>&1
  FAN_GEMM_PLAN="8192x1024x4096=256,256,2" timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --extra-budget 0 > gpurun_out/r6h/s2_r${r}.log 2>&1
  FAN_GEMM_PLAN="8192x1024x4096=256,256,4" timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --extra-budget 0 > gpurun_out/r6h/s4_r${r}.log 2>&1
done
for f in gpurun_out/r6h/*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1)"; done
