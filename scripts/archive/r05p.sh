#!/bin/bash
# r05p (ablation 7: head as interior) and r05o: why the streams' first fir_long_mfma workgroups stage twice as long:
# head-state order A/B and ablations of the head's state / new-state loads
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05p; mkdir -p $OUT
for v in "SDR_ABLATE=7" "SDR_F16_HEAD=1"; do
  echo "== $v" >> $OUT/f16_trace.txt
  env $v SDRHIP_LIB=$PWD/ab/timing.so SDR_F16_TRACE=1 REPS=2 timeout -k 10 200 python -u scripts/f16_trace.py 2>&1 | grep -E "span|staging|barrier \(" >> $OUT/f16_trace.txt; rc=$?
  [ $rc -eq 0 ] || exit $rc
done
cat $OUT/f16_trace.txt
exit 0
