#!/bin/bash
# r05q: fir_long_mfma head workgroup's state loads issued before the image
# loads -- f16 parity, phase trace (default / no head loads / head as
# interior), same-box A/B against the previous tree (ab/pre.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05q; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16 or cfg5h" > $OUT/pytest_f16.log 2>&1; rc=$?
tail -1 $OUT/pytest_f16.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_f16.log | head -20; exit $rc; }
for v in "SDR_F16_HEAD=1" "SDR_ABLATE=8" "SDR_ABLATE=7"; do
  echo "== $v" >> $OUT/f16_trace.txt
  env $v SDRHIP_LIB=$PWD/ab/timing.so SDR_F16_TRACE=1 REPS=2 timeout -k 10 200 python -u scripts/f16_trace.py 2>&1 | grep -E "span|staging|barrier \(|MFMA done" >> $OUT/f16_trace.txt; rc=$?
  [ $rc -eq 0 ] || exit $rc
done
cat $OUT/f16_trace.txt
ARMS="tree ab/pre.so" CFGS="cfg5h" REPS=4 bash scripts/ab_libs.sh > $OUT/ab_head.txt 2>&1; rc=$?; cat $OUT/ab_head.txt; [ $rc -eq 0 ] || exit $rc
TAG=r05q CFGS="cfg5h" bash scripts/prof_cfg.sh || exit 1
find $OUT -name '*kernel_trace.csv' -delete
exit 0
