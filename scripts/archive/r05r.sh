#!/bin/bash
# r05r: fir_long_mfma head workgroup anatomy (timing ablations 10: no
# new-state stores, 11: no state LDS writes); fir_tile_sc without its tile-0
# extra work (ablation 9) on cfg2 / cfg2u8 -- what the streams' first tiles cost
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05r; mkdir -p $OUT
for v in "SDR_ABLATE=10" "SDR_ABLATE=11" "SDR_F16_HEAD=1"; do
  echo "== $v" >> $OUT/f16_trace.txt
  env $v SDRHIP_LIB=$PWD/ab/timing9.so SDR_F16_TRACE=1 REPS=2 timeout -k 10 200 python -u scripts/f16_trace.py 2>&1 | grep -E "span|staging|barrier \(" >> $OUT/f16_trace.txt; rc=$?
  [ $rc -eq 0 ] || exit $rc
done
cat $OUT/f16_trace.txt
ARMS="ab/timing9.so ab/timing9.so:SDR_ABLATE=9" CFGS="cfg2 cfg2u8" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_t0.txt 2>&1; rc=$?; cat $OUT/ab_t0.txt; [ $rc -eq 0 ] || exit $rc
exit 0
