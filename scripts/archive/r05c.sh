#!/bin/bash
# r05c: interior span loads as raw buffer loads (ab/buf.so) -- parity + same-box
# A/B on cfg2 / cfg2u8 / mono0; fp16 non-temporal output stores (ab/f16nt.so);
# resample_lp's per-wave stall breakdown (SQ counters) for the cfg3 record.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05c; mkdir -p $OUT
SDRHIP_LIB=$PWD/ab/buf.so timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread -k "frontend or u8 or cfg2 or cfg4 or nonfinite or fir_decim" > $OUT/pytest_buf.log 2>&1; rc=$?
tail -1 $OUT/pytest_buf.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_buf.log | head; exit $rc; }
SDRHIP_LIB=$PWD/ab/f16nt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16 or cfg5" > $OUT/pytest_f16nt.log 2>&1; rc=$?
tail -1 $OUT/pytest_f16nt.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_f16nt.log | head; exit $rc; }
ARMS="tree ab/buf.so" CFGS="cfg2 cfg2u8 mono0" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_buf.txt 2>&1; rc=$?; cat $OUT/ab_buf.txt; [ $rc -eq 0 ] || exit $rc
ARMS="tree ab/f16nt.so" CFGS="cfg5h" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_f16nt.txt 2>&1; rc=$?; cat $OUT/ab_f16nt.txt; [ $rc -eq 0 ] || exit $rc
TAG=r05c/sq_cfg3 CFG=cfg3 KERNEL=resample_lp bash scripts/pmc_sq.sh || exit 1
exit 0
