#!/bin/bash
# r06ac: the PLL guard pre-pass as a streaming kernel (16-B lane loads, lane-pair combine):
# PLL / stereo parity on the tree, then stereo0 / stereo0w A/B against ab/guard_old.so
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06ac; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_scale.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread -k "pll or stereo" > $OUT/pytest_pll.log 2>&1; rc=$?
tail -2 $OUT/pytest_pll.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_pll.log | head -20; exit $rc; }
ARMS="tree ab/guard_old.so" CFGS="stereo0 stereo0w" REPS=3 STEPS=30 bash scripts/ab_libs.sh > $OUT/ab.txt 2>&1; rc=$?
cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
TAG=r06ac CFGS="stereo0" STEPS=30 bash scripts/prof_cfg.sh > /dev/null || exit 1
python3 -c "
import json; d=json.load(open('$OUT/prof_timed_stereo0.json'))
for k in d['kernels'][:9]: print(k['kernel'][:60], k['calls'], k.get('avg_us_timed'))"
find $OUT -name '*kernel_trace.csv' -delete
exit 0
