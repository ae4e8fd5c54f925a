#!/bin/bash
# r05i: fir_long_mfma fragment-group size (SDR_F16_G 2/4/6 vs 3) and the
# 4-wave shape under conflict-free A reads; f16 parity under each build.
# Mono pipeline fused (delay line in the front end's row, PCM from the audio
# FIR): parity + same-box A/B against the unfused library + kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05i; mkdir -p $OUT
for l in g2 g4 g6; do
  SDRHIP_LIB=$PWD/ab/$l.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16 or cfg5h" > $OUT/pytest_$l.log 2>&1; rc=$?
  echo "$l: $(tail -1 $OUT/pytest_$l.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_$l.log | head; exit $rc; }
done
ARMS="ab/base.so ab/g2.so ab/g4.so ab/g6.so ab/base.so:SDR_F16_W8=0" CFGS="cfg5h" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_g.txt 2>&1; rc=$?; cat $OUT/ab_g.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u -m pytest tests/test_dropin.py tests/test_gpu_scale.py -m gpu -x -q -p no:cacheprovider \
  --timeout 200 --timeout-method thread -k "mono" > $OUT/pytest_mono.log 2>&1; rc=$?
echo "mono: $(tail -1 $OUT/pytest_mono.log)"; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_mono.log | head; exit $rc; }
ARMS="tree ab/base.so" CFGS="mono0" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_mono.txt 2>&1; rc=$?; cat $OUT/ab_mono.txt; [ $rc -eq 0 ] || exit $rc
TAG=r05i CFGS="mono0" bash scripts/prof_cfg.sh || exit 1
find $OUT -name '*kernel_trace.csv' -delete
exit 0
