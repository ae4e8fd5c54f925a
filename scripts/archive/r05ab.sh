#!/bin/bash
# r05ab: dead rows of the edge / block-tail loops not issued (EXEC=0 loads
# cost the address path): parity of every tile kernel, same-box A/B vs HEAD.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ab; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_dropin.py tests/test_gpu_scale.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread -k "frontend or u8 or cfg2 or cfg4 or nonfinite or mono or stereo or golden or demod or fir or decim or block" > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
ARMS="tree ab/ee.so" CFGS="cfg2u8 mono0 cfg2" REPS=3 bash scripts/ab_libs.sh > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
exit 0
