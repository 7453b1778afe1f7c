# Parameter sweep of the two-barrier K-tile schedule (diagnostic -DFAN_GEMM_EDMA builds e1..e5, see pl4_run ktile)
# against the default one-barrier loop: GEMM numerics on each variant, then tools/probes/hipblaslt_nt_probe.py
set -e
mkdir -p gpurun_out/r6r
for v in e1 e2 e3 e4 e5; do
  cp so_ab/_C_$v.so fpga_ai_nic_amd/_C.so
  timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py tests/test_gpu_gemm_ovl.py > gpurun_out/r6r/tests_$v.log 2>&1
done
for r in 1 2; do
  for v in base e1 e2 e3 e4 e5; do
    cp so_ab/_C_$v.so fpga_ai_nic_amd/_C.so
    timeout -k 10 120 python3 tools/probes/hipblaslt_nt_probe.py > gpurun_out/r6r/p_${v}_r${r}.log 2>&1
  done
done
for f in gpurun_out/r6r/tests_*.log; do echo "$f $(tail -n 1 $f)"; done
for f in gpurun_out/r6r/p_*.log; do echo "$f $(tail -n 1 $f)"; done
