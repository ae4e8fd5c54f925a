#!/bin/bash
# r05v: fir_long_mfma head workgroup: state halves in 16-bit holders (no
# packing wait), loads after the image's; timing stamps kept in registers
# (the per-stamp store was an outstanding vector-memory op every later
# vmcnt(0) waited for).  f16 parity, trace, same-box A/B vs 60eba7f.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05v; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16 or cfg5h" > $OUT/pytest_f16.log 2>&1; rc=$?
tail -1 $OUT/pytest_f16.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_f16.log | head -20; exit $rc; }
for v in "SDR_F16_HEAD=1" "SDR_ABLATE=7"; do
  echo "== $v" >> $OUT/f16_trace.txt
  env $v SDRHIP_LIB=$PWD/ab/timing.so SDR_F16_TRACE=1 REPS=3 timeout -k 10 200 python -u scripts/f16_trace.py >> $OUT/f16_trace.txt 2>&1; rc=$?
  [ $rc -eq 0 ] || exit $rc
done
cat $OUT/f16_trace.txt
ARMS="tree ab/f16base.so" CFGS="cfg5h" REPS=4 bash scripts/ab_libs.sh > $OUT/ab_head.txt 2>&1; rc=$?; cat $OUT/ab_head.txt; [ $rc -eq 0 ] || exit $rc
TAG=r05v CFGS="cfg5h" bash scripts/prof_cfg.sh || exit 1
find $OUT -name '*kernel_trace.csv' -delete
exit 0
