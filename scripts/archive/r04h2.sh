#!/bin/bash
# r04h2: fir_long_mfma as 4,096-output workgroups of 4 one-tile waves (two per CU, SDR_F16_HALF=1)
# -- f16 parity under it, then the cfg5h A/B + kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SDR_F16_HALF=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16 or cfg5" > gpurun_out/r04h2_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04h2_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04h2_pytest.log | head; exit $rc; }
ARMS="SDR_F16_HALF=0 SDR_F16_HALF=1" CFGS="cfg5h" REPS=3 bash scripts/sweep_env.sh || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r04h2; mkdir -p $OUT
for w in 0 1; do
  SDR_F16_HALF=$w timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/half_$w" -o k \
    -- python3 bench.py --config cfg5h --steps 100 --warmup 3 --no-cpu-baseline --no-fma-variant --sustain-seconds 0 \
    > $OUT/bench_half_$w.json 2>>$OUT/err.log || exit 1
  f=$(find $OUT/half_$w -name '*kernel_stats.csv' | head -1)
  echo "half $w: $(grep fir_long_mfma $f | cut -d, -f1-5)"
done
find $OUT -name '*kernel_trace.csv' -delete
