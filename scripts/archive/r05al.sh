#!/bin/bash
# r05al: fir_long_mfma SIMD partners de-synchronised (MI355X_MICROARCH items 4
# and 9): ab/p4.so = waves 4-7 at s_setprio 1 for the loop; ab/st2.so /
# st4.so = waves 4-7 s_sleep 2 / 4 before it (a stagger); ab/p4st2.so = both.
# Outputs bitwise unchanged (same operations and order); f16 parity on the
# combined build; same-box A/B on cfg5h (4th column: the 3 s sustained frac).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05al; mkdir -p $OUT
SDRHIP_LIB=$PWD/ab/p4st2.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread -k "f16 or cfg5h" > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
ARMS="tree ab/st2.so ab/st4.so ab/p4st2.so" CFGS="cfg5h" REPS=${REPS:-4} bash scripts/ab_libs.sh > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
exit 0
