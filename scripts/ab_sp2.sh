#!/bin/bash
# resample_sp2 (split tap rows, SDR_RESAMPLE_SP2=1) vs resample_lp: resampler parity first, then same-box cfg3 arms
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-sp2}; mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider -rf \
  --timeout 120 --timeout-method thread -k "${TESTK:-resample}" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
ARMS="${ARMS:-tree:SDR_RESAMPLE_SP2=0 tree:SDR_RESAMPLE_SP2=1}" CFGS="${CFGS:-cfg3}" REPS=${REPS:-2} bash scripts/sweep_lib_env.sh
