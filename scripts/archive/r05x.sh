#!/bin/bash
# r05x: per-wave entry / barrier stamps of fir_long_mfma's head workgroup
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05x; mkdir -p $OUT
for v in "SDR_F16_HEAD=1" "SDR_ABLATE=13" "SDR_ABLATE=7"; do
  echo "== $v" >> $OUT/f16_trace.txt
  env $v SDRHIP_LIB=$PWD/ab/timing.so SDR_F16_TRACE=1 REPS=2 timeout -k 10 200 python -u scripts/f16_trace.py 2>&1 | grep -E "span|staging|workgroup [0-9]+:" >> $OUT/f16_trace.txt; rc=$?
  [ $rc -eq 0 ] || exit $rc
done
cat $OUT/f16_trace.txt
exit 0
