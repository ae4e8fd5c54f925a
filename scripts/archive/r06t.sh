#!/bin/bash
# r06t: PLL certified path vs exact-library path at receiver scale: the suite's short
# screen, then a long one (16,384 streams x 400 blocks x 5,120 samples = 3.4e10 PLL steps)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06t; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_scale.py -m gpu -x -q -p no:cacheprovider --timeout 240 \
  --timeout-method thread -k screen > $OUT/pytest_screen.log 2>&1; rc=$?
tail -2 $OUT/pytest_screen.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_screen.log | head; exit $rc; }
timeout -k 10 900 python -u tests/pll_screen.py --streams 16384 --blocks 400 --seed 1 > $OUT/screen_400.json 2> $OUT/screen.err; rc=$?
tail -3 $OUT/screen.err; cat $OUT/screen_400.json; exit $rc
