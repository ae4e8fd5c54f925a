#!/bin/bash
# r06aa: fir_tile_sc's f32 span by LDS-DMA (ab/sc_dma.so: -DSDR_SC_DMA=1, nt; ab/sc_dma_t.so: the
# same without the nt policy) -- front-end parity on the DMA build, then cfg2 / cfg4 A/B against the tree
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06aa; mkdir -p $OUT
SDRHIP_LIB=$PWD/ab/sc_dma.so timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread -k "frontend or golden or cfg2 or cfg4 or nonfinite or random" \
  > $OUT/pytest_dma.log 2>&1; rc=$?
tail -2 $OUT/pytest_dma.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_dma.log | head; exit $rc; }
ARMS="tree ab/sc_dma.so ab/sc_dma_t.so" CFGS="cfg2 cfg4" REPS=3 bash scripts/ab_libs.sh > $OUT/ab.txt 2>&1; rc=$?
cat $OUT/ab.txt; exit $rc
