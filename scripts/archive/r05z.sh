#!/bin/bash
# r05z: fp16 head workgroup -- ablation 15 (head, every chunk written, no
# state ops) and 16 (head, its load block not issued, no state ops)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05z; mkdir -p $OUT
for v in "SDR_ABLATE=15" "SDR_ABLATE=16" "SDR_ABLATE=13"; do
  echo "== $v" >> $OUT/f16_trace.txt
  env $v SDRHIP_LIB=$PWD/ab/timing.so SDR_F16_TRACE=1 REPS=2 timeout -k 10 200 python -u scripts/f16_trace.py 2>&1 | grep -E "span|staging" >> $OUT/f16_trace.txt; rc=$?
  [ $rc -eq 0 ] || exit $rc
done
cat $OUT/f16_trace.txt
exit 0
