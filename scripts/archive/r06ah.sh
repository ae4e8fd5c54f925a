#!/bin/bash
# r06ah: sdr_project with the recurrences alone on the second stream (SDR_PROJECT_SPLIT=2):
# the program's parity tests (every mode, mono / stereo schedules), then wall-clock of the
# program on 1,000 blocks beside the reference binary (modes 0 and 2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06ah; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 200 \
  --timeout-method thread -k "sdr_project" > $OUT/pytest_project.log 2>&1; rc=$?
tail -2 $OUT/pytest_project.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_project.log | head; exit $rc; }
NBLK=1000 timeout -k 10 900 bash scripts/time_project.sh > $OUT/time_project.txt 2>&1; rc=$?
cat $OUT/time_project.txt; exit $rc
