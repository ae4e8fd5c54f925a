#!/bin/bash
# r05aj: the whole GPU suite with each kernel-selection switch flipped from
# the environment (every test's default path becomes the fallback), one run
# per switch; stops at the first failing run.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05aj; mkdir -p $OUT
for sw in SDR_FIR_SC=0 SDR_FIR_SC_U8=0 SDR_RESAMPLE_LP=0 SDR_RESAMPLE_LOADER=0 SDR_LONG_VTAP=0 SDR_F16_MFMA=0 SDR_F16_HEAD=0 SDR_F16_W8=0 SDR_PLL_FAST=0 SDR_PLL_GUARD=0 SDR_STEREO_FORK=1; do
  env $sw timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > $OUT/pytest_$sw.log 2>&1; rc=$?
  echo "$sw: $(tail -1 $OUT/pytest_$sw.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_$sw.log | head -20; exit $rc; }
done
exit 0
