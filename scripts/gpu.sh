#!/bin/bash
# One parametrized runner for every GPU-box job (replaces the per-experiment gpu_*.sh launchers):
#
#   gpurun -- 'bash scripts/gpu.sh [OUT=<dir>] <step> [<step> ...]'
#
# Steps run in order; each runs under its own `timeout -k 10 <s>` and the script stops at the first step that
# fails (a fault, an abort, a time limit: nothing more touches the GPU in that call). Outputs go to
# gpurun_out/<OUT> (default gpurun_out/run); every step's log is <step-index>_<name>.log there.
#
#   test[=<pytest args>]      pytest -m gpu (default: the whole GPU suite) with a per-test thread timeout
#   smoke                     __graft_entry__.smoke()
#   bench[=<bench.py args>]   one flagship bench run (JSON line -> bench.jsonl)
#   prof[=<bench.py args>]    rocprofv3 --kernel-trace --stats of a bench run; per-kernel summary -> prof_stats.csv
#   pmc=<c1,c2,...>[:<args>]  ONE rocprofv3 --pmc pass (counters within the per-block slot limits) over a bench run
#   py=<script> [args]        any python tool / probe in the tree (e.g. py=bench/gemm_bench.py --shapes mlp)
#   sh=<command>              a shell command (non-GPU post-processing, listings)
#   env=<NAME>=<value>        export a variable for the following steps (unenv=<NAME> removes it): in-call A/B
#
# Knobs: T_TEST, T_BENCH, T_PROF, T_PY (seconds; defaults 600 / 300 / 300 / 300).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/run
if [[ "$1" == OUT=* ]]; then OUT=gpurun_out/${1#OUT=}; shift; fi
mkdir -p "$OUT"
i=0
for step in "$@"; do
  i=$((i + 1))
  name=${step%%=*}
  arg=""
  [[ "$step" == *=* ]] && arg=${step#*=}
  log="$OUT/$(printf %02d $i)_$name.log"
  echo "[gpu.sh] step $i: $step" | cut -c1-300
  case "$name" in
    test)
      timeout -k 10 "${T_TEST:-600}" python -u -m pytest ${arg:-tests} -m gpu -x -q --timeout 240 --timeout-method thread > "$log" 2>&1
      rc=$?; tail -3 "$log"
      [ $rc -eq 0 ] || { grep -E "Error|assert|FAIL|Timeout" "$log" | head -20; exit $rc; } ;;
    smoke)
      timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$log" 2>&1; rc=$?; tail -2 "$log"
      [ $rc -eq 0 ] || exit $rc ;;
    bench)
      timeout -k 10 "${T_BENCH:-300}" python bench.py $arg > "$OUT/bench_$i.jsonl" 2> "$log"; rc=$?
      tail -1 "$OUT/bench_$i.jsonl" | python3 -c 'import json,sys; d=json.loads(sys.stdin.read()); e=d["extra"]; print("bench", d["n_gpus"], d["value"], d["ms_per_step"], {k: e[k]["ms_per_step"] for k in e if k.startswith("mb") and e[k]}, "allreduce", e.get("allreduce"))' 2>/dev/null
      cat "$OUT/bench_$i.jsonl" >> "$OUT/bench.jsonl"
      [ $rc -eq 0 ] || { tail -20 "$log"; exit $rc; } ;;
    prof)
      timeout -k 10 "${T_PROF:-300}" rocprofv3 --kernel-trace --stats -d "$OUT/prof_$i" -o run --output-format csv -- python3 bench.py ${arg:---steps 20 --warmup 3 --ref-mb 0} > "$log" 2>&1; rc=$?
      [ $rc -eq 0 ] || { tail -20 "$log"; exit $rc; }
      f=$(find "$OUT/prof_$i" -name '*kernel_stats.csv' | head -1)
      [ -n "$f" ] && cp "$f" "$OUT/prof_stats_$i.csv" && head -25 "$f" | cut -d, -f1-6 | cut -c1-160 ;;
    pmc)
      ctr=${arg%%:*}; bargs=""; [[ "$arg" == *:* ]] && bargs=${arg#*:}
      timeout -s KILL 120 rocprofv3 --pmc ${ctr//,/ } -d "$OUT/pmc_$i" -o p --output-format csv -- python3 bench.py ${bargs:---steps 5 --warmup 2 --ref-mb 0} > "$log" 2>&1; rc=$?
      [ $rc -eq 0 ] || { tail -20 "$log"; exit $rc; }
      find "$OUT/pmc_$i" -name '*counter_collection.csv' -exec cp {} "$OUT/pmc_$i.csv" \; ;;
    py)
      timeout -k 10 "${T_PY:-300}" python -u $arg > "$log" 2>&1; rc=$?; tail -25 "$log" | cut -c1-400
      [ $rc -eq 0 ] || exit $rc ;;
    sh)
      bash -c "$arg" > "$log" 2>&1; rc=$?; tail -25 "$log" | cut -c1-400
      [ $rc -eq 0 ] || exit $rc ;;
    env)
      export "$arg"; echo "  export $arg" ;;
    unenv)
      unset "$arg"; echo "  unset $arg" ;;
    *)
      echo "[gpu.sh] unknown step '$name'"; exit 2 ;;
  esac
done
echo "[gpu.sh] all $i steps ok"
