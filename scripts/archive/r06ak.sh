#!/bin/bash
# r06ak: stereo0w with the one-channel FIR groups (band-pass filters, resamplers) capped at
# 8 / 12 waves (timing build's SDR_FIR_WPG) against the default 16
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06ak; mkdir -p $OUT
L=3dy4-real-time-software-defined-radio-_amd/libsdrhip_timing.so
ARMS="$L $L:SDR_FIR_WPG=8 $L:SDR_FIR_WPG=12" CFGS="stereo0w" REPS=3 STEPS=30 bash scripts/ab_libs.sh > $OUT/ab.txt 2>&1; rc=$?
cat $OUT/ab.txt; exit $rc
