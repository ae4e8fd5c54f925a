#!/bin/bash
# r05ar: after the fp16 fragment walk, the whole GPU suite under each fp16
# switch flipped (4-wave shape, head order, dot2 kernel).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ar; mkdir -p $OUT
for sw in SDR_F16_W8=0 SDR_F16_HEAD=0 SDR_F16_MFMA=0; do
  env $sw timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
    > $OUT/pytest_$sw.log 2>&1; rc=$?
  echo "$sw: $(tail -1 $OUT/pytest_$sw.log)"
  [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_$sw.log | head -20; exit $rc; }
done
exit 0
