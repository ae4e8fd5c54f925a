#!/bin/bash
# r05y: fir_tile_grp one-channel tile 0 loading its extra inputs before the
# span's wait (SDR_GRP_T0PRE) vs not (ab/grp0.so): FIR / mono / stereo parity
# and same-box A/B on mono0 / stereo0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05y; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_scale.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread -k "fir or mono or stereo or decim or block or nonfinite" > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
ARMS="tree ab/grp0.so" CFGS="mono0 stereo0" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_grp.txt 2>&1; rc=$?; cat $OUT/ab_grp.txt; [ $rc -eq 0 ] || exit $rc
TAG=r05y CFGS="mono0 cfg5h" bash scripts/prof_cfg.sh || exit 1
find $OUT -name '*kernel_trace.csv' -delete
exit 0
