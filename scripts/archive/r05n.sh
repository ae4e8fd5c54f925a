#!/bin/bash
# r05n: which fir_long_mfma workgroups stage slowest (8-wave default shape)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05n; mkdir -p $OUT
SDRHIP_LIB=$PWD/ab/timing.so SDR_F16_TRACE=1 REPS=3 timeout -k 10 200 python -u scripts/f16_trace.py > $OUT/f16_trace.txt 2>&1; rc=$?
cat $OUT/f16_trace.txt; [ $rc -eq 0 ] || exit $rc
exit 0
