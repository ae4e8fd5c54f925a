#!/bin/bash
# r05l: fp16 MFMA as 4 waves of 64-row tiles (SDR_F16_R64: the second row
# block reuses the first's A fragments from two steps back, one A + one B
# read per two MFMAs): f16 parity under every shape, same-box A/B, phase trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05l; mkdir -p $OUT
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16 or cfg5h" > $OUT/pytest_f16.log 2>&1; rc=$?
tail -1 $OUT/pytest_f16.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_f16.log | head -20; exit $rc; }
ARMS="tree tree:SDR_F16_R64=1" CFGS="cfg5h" REPS=4 bash scripts/ab_libs.sh > $OUT/ab_r64.txt 2>&1; rc=$?; cat $OUT/ab_r64.txt; [ $rc -eq 0 ] || exit $rc
SDRHIP_LIB=$PWD/ab/timing.so SDR_F16_TRACE=1 SDR_F16_R64=1 REPS=2 timeout -k 10 200 python -u scripts/f16_trace.py > $OUT/f16_trace_r64.txt 2>&1; rc=$?
cat $OUT/f16_trace_r64.txt; [ $rc -eq 0 ] || exit $rc
exit 0
