#!/bin/bash
# r05an: waves per group of the persistent fir_tile_grp (mono0's audio FIR
# ↓5; the front end is fir_tile_sc and unaffected): the timing build's
# SDR_FIR_WPG cap (default 16) at 4 / 8 / 12, same box, sustained column.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05an; mkdir -p $OUT
ARMS="ab/timing.so ab/timing.so:SDR_FIR_WPG=4 ab/timing.so:SDR_FIR_WPG=8 ab/timing.so:SDR_FIR_WPG=12" CFGS="mono0" REPS=3 \
  bash scripts/ab_libs.sh > $OUT/ab.txt 2>&1; rc=$?; cat $OUT/ab.txt; [ $rc -eq 0 ] || exit $rc
exit 0
