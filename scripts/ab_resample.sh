#!/bin/bash
# Resampler iteration: resampler parity tests, then cfg3 on each kernel
# (same box), then a kernel trace of the default kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-rs}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -rf --timeout 120 \
  --timeout-method thread -k "${TESTK:-resample}" > "$OUT/pytest.log" 2>&1
rc=$?; tail -15 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
for kv in "lp:" "rs:SDR_RESAMPLE_LP=0"; do
  name=${kv%%:*}; env=${kv#*:}
  env $env timeout -k 10 300 python bench.py --config cfg3 --steps 100 --warmup 3 --no-cpu-baseline \
    > "$OUT/bench_cfg3_$name.json" 2>> "$OUT/bench.err"
  rc=$?; echo "$name: $(cat $OUT/bench_cfg3_$name.json)"; [ $rc -eq 0 ] || exit $rc
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof_cfg3" -o bench \
  -- python3 bench.py --config cfg3 --steps 100 --warmup 3 --no-cpu-baseline > "$OUT/prof_bench_cfg3.json" 2>> "$OUT/prof.err"
rc=$?; echo "rocprof rc=$rc"; [ $rc -eq 0 ] || exit $rc
cat $(find $OUT/prof_cfg3 -name '*kernel_stats.csv' | head -1) | head -8
exit 0
