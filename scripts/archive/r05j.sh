#!/bin/bash
# r05j: the whole GPU suite + smoke on the current tree; mono pipeline side
# copies batched with the state-carry loads (tree) vs unbatched (ab/fused1.so)
# vs unfused (ab/base.so); mono0 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05j; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -3 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
ARMS="tree ab/fused1.so ab/base.so" CFGS="mono0" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_mono.txt 2>&1; rc=$?; cat $OUT/ab_mono.txt; [ $rc -eq 0 ] || exit $rc
TAG=r05j CFGS="mono0" bash scripts/prof_cfg.sh || exit 1
find $OUT -name '*kernel_trace.csv' -delete
exit 0
