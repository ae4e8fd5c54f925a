#!/bin/bash
# r05d: the tree with the u8 buffer-load default -- the whole GPU suite and
# smoke; fp16 outputs transposed through LDS (ab/tstore.so): parity + A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05d; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1; tail -1 $OUT/smoke.log
SDRHIP_LIB=$PWD/ab/tstore.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16 or cfg5" > $OUT/pytest_tstore.log 2>&1; rc=$?
tail -1 $OUT/pytest_tstore.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_tstore.log | head; exit $rc; }
ARMS="tree ab/tstore.so" CFGS="cfg5h" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_tstore.txt 2>&1; rc=$?; cat $OUT/ab_tstore.txt; [ $rc -eq 0 ] || exit $rc
exit 0
