#!/bin/bash
# r04w: fir_long_mfma with scheduling barriers pinning the fragment reads ahead of the
# previous group's MFMAs (SDR_F16_SB=1) -- f16 parity, then the cfg5h A/B + kernel trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16 or cfg5" > gpurun_out/r04w_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04w_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04w_pytest.log | head; exit $rc; }
ARMS="SDR_F16_SB=0 SDR_F16_SB=1" CFGS="cfg5h" REPS=3 bash scripts/sweep_env.sh || exit 1
export TMPDIR=/tmp
OUT=gpurun_out/r04w; mkdir -p $OUT
for sb in 0 1; do
  SDR_F16_SB=$sb timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/sb$sb" -o k \
    -- python3 bench.py --config cfg5h --steps 100 --warmup 3 --no-cpu-baseline --no-fma-variant --sustain-seconds 0 \
    > $OUT/bench_sb$sb.json 2>>$OUT/err.log || exit 1
  f=$(find $OUT/sb$sb -name '*kernel_stats.csv' | head -1)
  echo "sb $sb: $(grep fir_long_mfma $f | cut -d, -f1-5)"
done
