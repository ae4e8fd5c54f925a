#!/bin/bash
# fir_tile_sc (two waves per tile, one channel each) vs fir_tile on the fused f32 front end:
# front-end parity under both, then same-box bench arms.   TAG=sc bash scripts/ab_sc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-sc}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider -rf \
  --timeout 120 --timeout-method thread -k "${TESTK:-frontend or cfg2_full}" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
ARMS="${ARMS:-tree:SDR_FIR_SC=0 tree:SDR_FIR_SC=1}" CFGS="${CFGS:-cfg2}" REPS=${REPS:-3} bash scripts/ab_libs.sh
