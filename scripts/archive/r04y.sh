#!/bin/bash
# r04y: fir_long_mfma with 8 waves (two per SIMD, one tile each; SDR_F16_W8=1) -- f16 parity
# under it, then the cfg5h A/B + kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SDR_F16_W8=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16 or cfg5" > gpurun_out/r04y_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04y_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04y_pytest.log | head; exit $rc; }
ARMS="SDR_F16_W8=0 SDR_F16_W8=1" CFGS="cfg5h" REPS=3 bash scripts/sweep_env.sh || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r04y; mkdir -p $OUT
for w in 0 1; do
  SDR_F16_W8=$w timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/w8_$w" -o k \
    -- python3 bench.py --config cfg5h --steps 100 --warmup 3 --no-cpu-baseline --no-fma-variant --sustain-seconds 0 \
    > $OUT/bench_w8_$w.json 2>>$OUT/err.log || exit 1
  f=$(find $OUT/w8_$w -name '*kernel_stats.csv' | head -1)
  echo "w8 $w: $(grep fir_long_mfma $f | cut -d, -f1-5)"
done
find $OUT -name '*kernel_trace.csv' -delete
