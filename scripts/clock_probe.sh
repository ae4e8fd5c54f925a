#!/bin/bash
# GPU clock and power while cfg2 runs, per arithmetic / ablation mode: is the
# fused front end clock-limited (power) or not?  Each mode runs a long bench
# (~2-3 s of timed steps) and rocm-smi is sampled while it is in its timed
# region.   TAG=clk bash scripts/clock_probe.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
. scripts/timing_lib.sh  # SDR_ABLATE etc. need the timing build
OUT=gpurun_out/${TAG:-clk}
mkdir -p "$OUT"
STEPS=${STEPS:-60000}
for mode in exact fma ablate2 ablate1 exact; do
  envs=""
  case $mode in
    fma) envs="SDR_ARITH_FMA=1" ;;
    ablate2) envs="SDR_ABLATE=2" ;;
    ablate1) envs="SDR_ABLATE=1" ;;
  esac
  env $envs timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps $STEPS --warmup 3 --no-cpu-baseline \
      --no-fma-variant > "$OUT/bench_$mode.json" 2> "$OUT/bench_$mode.err" &
  pid=$!
  sleep ${SETTLE:-9}
  for i in 1 2 3 4 5 6; do
    timeout -k 5 20 rocm-smi --showclocks --showpower --showtemp >> "$OUT/smi_$mode.txt" 2>&1
    sleep 0.2
  done
  wait $pid; rc=$?
  echo "$mode rc=$rc $(python3 -c "import json;d=json.load(open('$OUT/bench_$mode.json'));print(d['ms_per_step'], d['roofline']['frac'])" 2>/dev/null)"
  grep -E 'sclk|fclk|mclk|Power|Socket' "$OUT/smi_$mode.txt" | sort | uniq -c | head -12
  [ $rc -eq 0 ] || exit $rc
done
