#!/bin/bash
# r05k: fir_tile_grp one span per channel (one-channel FIRs: 16 waves per CU,
# one round of tiles) vs two (ab/slice2.so); FIR / mono / stereo parity.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05k; mkdir -p $OUT
timeout -k 10 60 ./tools/ubench_ldsmask > $OUT/ubench_ldsmask.txt 2>&1; rc=$?; cat $OUT/ubench_ldsmask.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_scale.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread -k "fir or mono or stereo or decim or block or resample" > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head; exit $rc; }
ARMS="tree ab/slice2.so ab/fused1.so" CFGS="mono0 stereo0" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_slice.txt 2>&1; rc=$?; cat $OUT/ab_slice.txt; [ $rc -eq 0 ] || exit $rc
TAG=r05k CFGS="mono0" bash scripts/prof_cfg.sh || exit 1
find $OUT -name '*kernel_trace.csv' -delete
exit 0
