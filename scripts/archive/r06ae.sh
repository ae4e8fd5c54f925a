#!/bin/bash
# r06ae: stereo with the recurrences alone on the second stream (--stereo-pipeline 2: block b's
# post stage after block b+1's front stage on the first): pipeline parity, then A/B vs two stages
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06ae; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_scale.py tests/test_dropin.py -m gpu -x -q -p no:cacheprovider \
  --timeout 300 --timeout-method thread -k "stereo" > $OUT/pytest_stereo.log 2>&1; rc=$?
tail -2 $OUT/pytest_stereo.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_stereo.log | head -20; exit $rc; }
ARMS="tree:SDR_BENCH_STEREO_PIPE=1 tree:SDR_BENCH_STEREO_PIPE=2" CFGS="stereo0 stereo0w" REPS=3 STEPS=30 \
  bash scripts/ab_libs.sh > $OUT/ab.txt 2>&1; rc=$?
cat $OUT/ab.txt; exit $rc
