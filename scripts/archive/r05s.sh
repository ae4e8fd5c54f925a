#!/bin/bash
# r05s: fir_tile_sc tile 0 with its extra loads in the span's batch
# (SDR_SC_T0PRE) -- front-end / mono / stereo parity, same-box A/B against
# the build without it (ab/t0off.so) on cfg2 / cfg2u8 / mono0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05s; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_dropin.py tests/test_gpu_scale.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread -k "frontend or u8 or cfg2 or cfg4 or nonfinite or mono or stereo or golden or demod" > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
ARMS="tree ab/t0off.so" CFGS="cfg2 cfg2u8 mono0" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_t0pre.txt 2>&1; rc=$?; cat $OUT/ab_t0pre.txt; [ $rc -eq 0 ] || exit $rc
exit 0
