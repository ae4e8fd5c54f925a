#!/bin/bash
# r05ac: fir_long_mfma A fragments two steps per LDS read (DPP row_shr / row_ror
# of the Toeplitz rows): f16 parity for each group size, same-box A/B vs the
# unpaired loop (ab/pair0.so = SDR_F16_PAIR=0); ab/pg2.so, ab/pg4.so = paired
# with 2 / 4 steps per group (tree: 6).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ac; mkdir -p $OUT
: > $OUT/pytest.log
for L in tree ab/pg2.so ab/pg4.so; do
  if [ $L = tree ]; then unset SDRHIP_LIB; else export SDRHIP_LIB=$PWD/$L; fi
  echo "== $L" >> $OUT/pytest.log
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
    -p no:cacheprovider --timeout 200 --timeout-method thread -k "f16 or cfg5h" >> $OUT/pytest.log 2>&1; rc=$?
  tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
done
unset SDRHIP_LIB
ARMS="tree ab/pg2.so ab/pg4.so ab/pair0.so" CFGS="cfg5h" REPS=3 bash scripts/ab_libs.sh > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
exit 0
