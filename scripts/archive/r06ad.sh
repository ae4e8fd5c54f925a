#!/bin/bash
# r06ad: the PLL guard pre-pass moved into the two-stage stereo front stage (off the back stage's
# critical path): PLL / stereo / program parity, then stereo0 / stereo0w A/B against the guard
# in the back stage (ab/guard_vec.so: streaming kernel; ab/guard_old.so: the round-5 kernel)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06ad; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_scale.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread -k "pll or stereo or project" > $OUT/pytest_pll.log 2>&1; rc=$?
tail -2 $OUT/pytest_pll.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_pll.log | head -20; exit $rc; }
ARMS="tree ab/guard_vec.so ab/guard_old.so" CFGS="stereo0 stereo0w" REPS=3 STEPS=30 bash scripts/ab_libs.sh > $OUT/ab.txt 2>&1; rc=$?
cat $OUT/ab.txt; exit $rc
