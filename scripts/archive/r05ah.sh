#!/bin/bash
# r05ah: fir_long_mfma with one wave of each SIMD pair at a higher issue
# priority during the MFMA loop (it finishes first and stores while its
# partner computes): ab/prio.so = waves 0-3, ab/prio2.so = even waves;
# f16 parity under both, same-box A/B on cfg5h.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ah; mkdir -p $OUT
: > $OUT/pytest.log
for L in ab/prio.so ab/prio2.so; do
  SDRHIP_LIB=$PWD/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread -k "f16 or cfg5h" >> $OUT/pytest.log 2>&1; rc=$?
  tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
done
ARMS="tree ab/prio.so ab/prio2.so" CFGS="cfg5h" REPS=4 bash scripts/ab_libs.sh > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
exit 0
