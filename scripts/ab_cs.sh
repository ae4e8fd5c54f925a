#!/bin/bash
# fir_tile_cs (channel-sequential LDS) vs fir_tile on the fused f32 front end:
# its parity tests first, then same-box bench arms.   TAG=cs bash scripts/ab_cs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-cs}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider -rf \
  --timeout 120 --timeout-method thread -k "${TESTK:-frontend or cfg2_full}" > "$OUT/pytest.log" 2>&1
rc=$?; tail -4 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
ARMS="${ARMS:-tree:SDR_FIR_CS=0 tree:SDR_FIR_CS=1}" CFGS="${CFGS:-cfg2}" REPS=${REPS:-3} bash scripts/ab_libs.sh
