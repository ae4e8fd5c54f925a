#!/bin/bash
# r04x: fir_long_mfma tap copies written from registers before the first barrier
# (SDR_F16_TAPS=1; 0 = the LDS row + copy pass + second barrier) -- f16 parity, cfg5h A/B + trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16 or cfg5" > gpurun_out/r04x_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04x_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04x_pytest.log | head; exit $rc; }
ARMS="SDR_F16_TAPS=0 SDR_F16_TAPS=1" CFGS="cfg5h" REPS=3 bash scripts/sweep_env.sh || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r04x; mkdir -p $OUT
for tp in 0 1; do
  SDR_F16_TAPS=$tp timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/taps$tp" -o k \
    -- python3 bench.py --config cfg5h --steps 100 --warmup 3 --no-cpu-baseline --no-fma-variant --sustain-seconds 0 \
    > $OUT/bench_taps$tp.json 2>>$OUT/err.log || exit 1
  f=$(find $OUT/taps$tp -name '*kernel_stats.csv' | head -1)
  echo "taps $tp: $(grep fir_long_mfma $f | cut -d, -f1-5)"
done
find $OUT -name '*kernel_trace.csv' -delete
