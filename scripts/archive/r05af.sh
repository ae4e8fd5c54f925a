#!/bin/bash
# r05af: fir_long_mfma with its LDS request raised past half a CU's LDS (one
# workgroup per CU; ab/lds1.so = SDR_F16_LDS_MIN=81936) vs the tree (79 KB:
# two can share a CU): f16 parity under the A/B build, same-box A/B on cfg5h.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05af; mkdir -p $OUT
SDRHIP_LIB=$PWD/ab/lds1.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread -k "f16 or cfg5h" > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
ARMS="tree ab/lds1.so" CFGS="cfg5h" REPS=4 bash scripts/ab_libs.sh > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
exit 0
