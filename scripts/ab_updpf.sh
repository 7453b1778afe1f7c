# A/B: fused-update epilogue master prefetch depth (FAN_GEMM_UPD_PF = 1 / 2 / 3 row blocks ahead), three builds of
# the extension swapped in between runs (so_ab/_C_pf*.so); numerics: the fused-update tests on each build
set -e
mkdir -p gpurun_out/r6e
cp fpga_ai_nic_amd/_C.so so_ab/_C_orig.so
for v in ${AB_TEST_VARIANTS:-1 2 3}; do
  cp so_ab/_C_pf$v.so fpga_ai_nic_amd/_C.so
  timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_fused_update.py tests/test_gpu_defer_colsum.py > gpurun_out/r6e/tests_pf$v.log 2>&1
done
for r in 3 4 5; do
  for v in 1 2 3; do
    cp so_ab/_C_pf$v.so fpga_ai_nic_amd/_C.so
    timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --extra-budget 0 > gpurun_out/r6e/b8192_pf${v}_r${r}.log 2>&1
    timeout -k 10 200 python3 bench.py --mb-per-gpu 1792 --ref-mb 0 --steps 100 --warmup 20 --extra-budget 0 > gpurun_out/r6e/b1792_pf${v}_r${r}.log 2>&1
  done
done
cp so_ab/_C_orig.so fpga_ai_nic_amd/_C.so
rm -f so_ab/_C_orig.so
for f in gpurun_out/r6e/tests_*.log; do echo "$f $(tail -n 1 $f)"; done
for f in gpurun_out/r6e/b*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1)"; done
