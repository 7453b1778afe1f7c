#!/bin/bash
# Same-box, in-step A/B of run-time knobs: each line of ARMS_FILE is "name|VAR=value VAR2=value" (empty env =
# baseline); the flagship bench runs once per arm per round, arms interleaved, separate processes.
# Usage: scripts/gpu_env_ab.sh ARMS_FILE [rounds] [extra bench args]
set -e
ARMS=$1; R=${2:-3}; shift 2 || true
mkdir -p gpurun_out
for r in $(seq 1 $R); do
  while IFS='|' read -r name envs; do
    [ -z "$name" ] && continue
    echo -n "$name round $r: " | tee -a gpurun_out/env_ab.log
    env $envs timeout -k 10 300 python bench.py --steps 40 --warmup 10 "$@" | tee -a gpurun_out/env_ab.log
  done < "$ARMS"
done
