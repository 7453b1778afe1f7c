# A/B: fragment reads bunched at the start of each k-step and the operand DMA after them (diagnostic builds
# -DFAN_GEMM_RSP_Q4 / -DFAN_GEMM_DMA_Q0 / -DFAN_GEMM_DMA_SP, variants r1..r3) vs the default interleaving
set -e
mkdir -p gpurun_out/r6s
for v in r1 r2; do
  cp so_ab/_C_$v.so fpga_ai_nic_amd/_C.so
  timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_gemm_ovl.py > gpurun_out/r6s/tests_$v.log 2>&1
done
for r in 1 2; do
  for v in base r1 r2; do
    cp so_ab/_C_$v.so fpga_ai_nic_amd/_C.so
    timeout -k 10 120 python3 tools/probes/hipblaslt_nt_probe.py > gpurun_out/r6s/p_${v}_r${r}.log 2>&1
    timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --extra-budget 0 --ref-mb 0 > gpurun_out/r6s/b_${v}_r${r}.log 2>&1
  done
done
for f in gpurun_out/r6s/tests_*.log; do echo "$f $(tail -n 1 $f)"; done
for f in gpurun_out/r6s/p_*.log; do echo "$f $(tail -n 1 $f)"; done
for f in gpurun_out/r6s/b_*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1)"; done
