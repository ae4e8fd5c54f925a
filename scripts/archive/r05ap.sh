#!/bin/bash
# r05ap: fir_long_mfma walks its A / B fragments from pointers bumped once
# per pair of groups (every read an immediate offset; before, ~4 VALU of
# mf_pad arithmetic per B read): f16 parity, same-box A/B vs HEAD
# (ab/head.so) with the sustained column, timed rocprof of cfg5h.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ap; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread -k "f16 or cfg5h" > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
ARMS="tree ab/head.so" CFGS="cfg5h" REPS=4 bash scripts/ab_libs.sh > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
TAG=r05ap CFGS="cfg5h" bash scripts/prof_cfg.sh || exit 1
find $OUT -name '*kernel_trace.csv' -delete
exit 0
