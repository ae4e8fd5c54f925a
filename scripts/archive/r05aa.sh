#!/bin/bash
# r05aa: fir_long_mfma head workgroup loops only over rows that hold state
# elements (no EXEC=0 loads); resample_lp loader's state commit loads batched.
# f16 + resampler parity, head trace, same-box A/B against HEAD (ab/lpbase.so).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05aa; mkdir -p $OUT
timeout -k 10 500 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread -k "f16 or cfg5h or resample or cfg3" > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
for v in "SDR_F16_HEAD=1" "SDR_ABLATE=7"; do
  echo "== $v" >> $OUT/f16_trace.txt
  env $v SDRHIP_LIB=$PWD/ab/timing.so SDR_F16_TRACE=1 REPS=2 timeout -k 10 200 python -u scripts/f16_trace.py 2>&1 | grep -E "span|staging|MFMA done" >> $OUT/f16_trace.txt; rc=$?
  [ $rc -eq 0 ] || exit $rc
done
cat $OUT/f16_trace.txt
ARMS="tree ab/lpbase.so" CFGS="cfg5h cfg3" REPS=3 bash scripts/ab_libs.sh > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
TAG=r05aa CFGS="cfg5h" bash scripts/prof_cfg.sh || exit 1
find $OUT -name '*kernel_trace.csv' -delete
exit 0
