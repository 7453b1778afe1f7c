# Decomposition of the 256x256 4-wave loop (diagnostic builds, wrong results, timing only): full / without the
# operand LDS-DMA (-DFAN_GEMM_NODMA) / without the MFMAs (-DFAN_GEMM_NOMFMA, fragments still read) / neither;
# tools/probes/hipblaslt_nt_probe.py (M=8192 N=4096 K=4096; lib_nt = the library's NT kernel for reference)
set -e
mkdir -p gpurun_out/r6p
for r in 1 2; do
  for v in base nodma nomfma none; do
    cp so_ab/_C_$v.so fpga_ai_nic_amd/_C.so
    timeout -k 10 120 python3 tools/probes/hipblaslt_nt_probe.py > gpurun_out/r6p/p_${v}_r${r}.log 2>&1
  done
done
for f in gpurun_out/r6p/p_*.log; do echo "$f $(tail -n 1 $f)"; done
