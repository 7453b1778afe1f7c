# A/B: softmax-xent with the label's logit taken from registers (new) vs reloaded from memory (base)
set -e
mkdir -p gpurun_out/r6m
cp so_ab/_C_new.so fpga_ai_nic_amd/_C.so
timeout -k 10 200 python3 -u -m pytest -x -q --timeout 120 --timeout-method thread tests/test_gpu_kernels.py -k softmax tests/test_gpu_gemm_ragged.py tests/test_gpu_fold_logits.py > gpurun_out/r6m/tests.log 2>&1
for r in 1 2 3; do
  for v in base new; do
    cp so_ab/_C_$v.so fpga_ai_nic_amd/_C.so
    timeout -k 10 100 python3 tools/probes/softmax_probe.py > gpurun_out/r6m/p_${v}_r${r}.log 2>&1
  done
done
tail -n 1 gpurun_out/r6m/tests.log
for f in gpurun_out/r6m/p_*.log; do echo "$f $(tail -n 1 $f)"; done
