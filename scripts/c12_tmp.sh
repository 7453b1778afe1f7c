set -o pipefail
O=gpurun_out/c16; mkdir -p $O
timeout -k 10 300 python -u -m pytest -x -v --timeout 240 --timeout-method thread tests/test_gpu_p2p.py -k "four_processes or two_processes_one_gpu" > $O/t.log 2>&1; rc=$?; echo t_rc=$rc
case $rc in 0|1) ;; *) exit $rc;; esac
timeout -k 10 500 python -u bench.py --gpus 4 --steps 4 --warmup 2 --ab-steps 2 --ref-mb 0 --mb-per-gpu 1024 --timeout 100 --extra-budget 90 > $O/b4.jsonl 2> $O/b4.err; echo b4_rc=$?
