# A/B: the GEMM LDS-DMA pieces as MUBUF buffer_load_dwordx4 ... lds (diagnostic build -DFAN_GEMM_BUFLDS) vs
# global_load_lds_dwordx4 (default): GEMM numerics on the variant, the library-comparison probe and the step
set -e
mkdir -p gpurun_out/r6l
cp so_ab/_C_buf.so fpga_ai_nic_amd/_C.so
timeout -k 10 300 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_gemm_ovl.py tests/test_gpu_fused_update.py > gpurun_out/r6l/tests_buf.log 2>&1
for r in 1 2 3; do
  for v in base buf; do
    cp so_ab/_C_$v.so fpga_ai_nic_amd/_C.so
    timeout -k 10 120 python3 tools/probes/hipblaslt_nt_probe.py > gpurun_out/r6l/probe_${v}_r${r}.log 2>&1
    timeout -k 10 200 python3 bench.py --steps 50 --warmup 10 --extra-budget 0 --ref-mb 0 > gpurun_out/r6l/b8192_${v}_r${r}.log 2>&1
  done
done
tail -n 1 gpurun_out/r6l/tests_buf.log
for f in gpurun_out/r6l/probe_*.log; do echo "$f $(tail -n 1 $f)"; done
for f in gpurun_out/r6l/b*.log; do echo "$f $(grep -o '"ms_per_step": [0-9.]*' $f | head -1)"; done
