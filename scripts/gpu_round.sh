#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a fault / abort / timeout stops the
# script (exit codes other than 0 = pass and 1 = test failures).
#   TAG=r02b [TESTS=0] [EXTRA_CFGS="cfg3 cfg4"] [PROF_CFGS="cfg3"] [PMC=1] bash scripts/gpu_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r02}
mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }
STEPS=${STEPS:-100}

echo "== host: $(nproc) cpus"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -rf --timeout 300 \
      --timeout-method thread > "$OUT/pytest_gpu.log" 2>&1
  rc=$?; tail -25 "$OUT/pytest_gpu.log"; ok $rc || { echo "pytest rc=$rc, stopping"; exit $rc; }
  timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
  rc=$?; tail -5 "$OUT/smoke.log"; [ $rc -eq 0 ] || { echo "smoke rc=$rc"; ok $rc || exit $rc; }
fi

timeout -k 10 600 python bench.py --steps $STEPS --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"; [ $rc -eq 0 ] || exit $rc

for cfg in ${EXTRA_CFGS:-}; do
  timeout -k 10 600 python bench.py --config "$cfg" --steps $STEPS --warmup 3 --no-cpu-baseline > "$OUT/bench_$cfg.json" 2>> "$OUT/bench.err"
  rc=$?; cat "$OUT/bench_$cfg.json"; [ $rc -eq 0 ] || exit $rc
done

export TMPDIR=/tmp
# kernel trace of the default bench command (exact run only: the timed
# region is the kernel's last $STEPS dispatches -> scripts/prof_timed.py)
for cfg in cfg2 ${PROF_CFGS:-}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof_$cfg" -o bench \
    -- python3 bench.py --config $cfg --steps $STEPS --warmup 5 --no-cpu-baseline --no-fma-variant \
    > "$OUT/prof_bench_$cfg.json" 2>> "$OUT/prof.err"
  rc=$?; echo "rocprof $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python scripts/prof_timed.py "$(find $OUT/prof_$cfg -name '*kernel_trace.csv' | head -1)" $STEPS \
    "$OUT/prof_timed_$cfg.json" "$OUT/prof_bench_$cfg.json"
done

# HBM traffic: one counter per pass (FETCH_SIZE, then WRITE_SIZE)
if [ -n "${PMC:-}" ]; then
  for cfg in cfg2 ${PMC_CFGS:-}; do
    for ctr in FETCH_SIZE WRITE_SIZE; do
      timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/pmc_${cfg}_$ctr" -o pmc \
        -- python3 bench.py --config $cfg --steps 3 --warmup 1 --warm-seconds 0 --no-cpu-baseline --no-fma-variant --no-graph --sustain-seconds 0 \
        > /dev/null 2>> "$OUT/prof.err"
      rc=$?; echo "pmc $cfg $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
    done
    k=fir_tile; [ $cfg = cfg3 ] && k=resample_lp
    python scripts/pmc_traffic.py "$(find $OUT/pmc_${cfg}_FETCH_SIZE -name '*counter_collection.csv' | head -1)" \
      "$(find $OUT/pmc_${cfg}_WRITE_SIZE -name '*counter_collection.csv' | head -1)" $k "$OUT/traffic_$cfg.json"
  done
fi
# the per-dispatch traces run to tens of MB: keep the stats and the timed summaries only
[ "${TRIM:-1}" = 1 ] && find "$OUT" -name '*kernel_trace.csv' -delete
exit 0
