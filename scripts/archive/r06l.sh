#!/bin/bash
# r06l: whole GPU suite + smoke on the round-6 tree so far
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06l; mkdir -p $OUT
timeout -k 10 1000 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread \
  --durations=15 > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -22 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 ./tools/ubench_valu > $OUT/ubench_valu.txt 2>&1; rc=$?; grep -E "mix|mul\\(s\\)\\+add" $OUT/ubench_valu.txt | head -20
tail -2 $OUT/smoke.log; exit $rc
