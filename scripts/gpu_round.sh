#!/bin/bash
# One GPU-box session: parity tests, smoke, bench, rocprofv3 kernel trace.
# Every GPU step has its own time limit; a fault / abort / timeout stops the
# script (exit codes other than 0 = pass and 1 = test failures).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r01}
mkdir -p "$OUT"
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }

echo "== host: $(nproc) cpus"; rocm-smi --showproductname 2>/dev/null | grep -i -E 'card|series' | head -3
timeout -k 10 900 python -m pytest tests -m gpu -q -p no:cacheprovider -rf > "$OUT/pytest_gpu.log" 2>&1
rc=$?; tail -25 "$OUT/pytest_gpu.log"; ok $rc || { echo "pytest rc=$rc, stopping"; exit $rc; }

timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; cat "$OUT/smoke.log" | tail -5; [ $rc -eq 0 ] || { echo "smoke rc=$rc"; ok $rc || exit $rc; }

timeout -k 10 600 python bench.py --steps 20 --warmup 5 > "$OUT/bench.json" 2> "$OUT/bench.err"
rc=$?; cat "$OUT/bench.json"; tail -5 "$OUT/bench.err"; [ $rc -eq 0 ] || exit $rc

for cfg in ${EXTRA_CFGS:-}; do
  timeout -k 10 600 python bench.py --config "$cfg" --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/bench_$cfg.json" 2>> "$OUT/bench.err"
  rc=$?; cat "$OUT/bench_$cfg.json"; [ $rc -eq 0 ] || exit $rc
done

export TMPDIR=/tmp
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o bench \
  -- python3 bench.py --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/prof_bench.json" 2> "$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"; find "$OUT/prof" -name '*stats*' | head
[ $rc -eq 0 ] || exit $rc

# per-config kernel statistics (the other configs' dominant kernels)
for cfg in ${PROF_CFGS:-}; do
  timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof_$cfg" -o bench \
    -- python3 bench.py --config "$cfg" --steps 10 --warmup 3 --no-cpu-baseline > "$OUT/prof_bench_$cfg.json" 2>> "$OUT/prof.err"
  rc=$?; echo "rocprof $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
done

# HBM traffic: one counter per pass (FETCH_SIZE, then WRITE_SIZE)
if [ -n "${PMC:-}" ]; then
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/pmc_$ctr" -o pmc \
      -- python3 bench.py --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> "$OUT/prof.err"
    rc=$?; echo "pmc $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python scripts/pmc_traffic.py "$(find $OUT/pmc_FETCH_SIZE -name '*counter_collection.csv' | head -1)" \
    "$(find $OUT/pmc_WRITE_SIZE -name '*counter_collection.csv' | head -1)" fir_tile "$OUT/traffic_cfg2.json"
  # the resampler's traffic (cfg3)
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 600 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/pmc3_$ctr" -o pmc \
      -- python3 bench.py --config cfg3 --steps 3 --warmup 1 --no-cpu-baseline > /dev/null 2>> "$OUT/prof.err"
    rc=$?; echo "pmc cfg3 $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  python scripts/pmc_traffic.py "$(find $OUT/pmc3_FETCH_SIZE -name '*counter_collection.csv' | head -1)" \
    "$(find $OUT/pmc3_WRITE_SIZE -name '*counter_collection.csv' | head -1)" resample_lp "$OUT/traffic_cfg3.json"
fi
exit 0
