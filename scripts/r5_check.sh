mkdir -p gpurun_out/r5d
for i in 1 2; do
  (cd old_r4 && timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extra-budget 0 > ../gpurun_out/r5d/old_$i.json 2> ../gpurun_out/r5d/old_$i.err) || exit 1
  timeout -k 10 200 python bench.py --steps 20 --warmup 5 --extra-budget 0 > gpurun_out/r5d/new_$i.json 2> gpurun_out/r5d/new_$i.err || exit 1
done
timeout -k 10 400 python -u -m pytest -x -v --timeout 150 --timeout-method thread tests/test_gpu_shard_update.py tests/test_gpu_gemm_group.py > gpurun_out/r5d/pytest_new.log 2>&1
echo "pytest rc=$?" >> gpurun_out/r5d/pytest_new.log
