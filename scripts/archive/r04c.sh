#!/bin/bash
# r04c: VGPR-tap front end (parity + A/B on cfg2u8/cfg2/mono0) and the
# resampler's ablations (no staging, no math, no scan LDS reads).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04c; mkdir -p $OUT
timeout -k 10 120 ./tools/ubench_ldsmix > "$OUT/ubench_ldsmix.txt" 2>&1; rc=$?; cat "$OUT/ubench_ldsmix.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider \
  -rf --timeout 300 --timeout-method thread -k "frontend or cfg2" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
ARMS="SDR_FIR_VTAP_U8=0 SDR_FIR_VTAP_U8=1" CFGS="cfg2u8 mono0" REPS=2 bash scripts/sweep_env.sh || exit 1
ARMS="SDR_FIR_VTAP=0 SDR_FIR_VTAP=1" CFGS="cfg2" REPS=2 bash scripts/sweep_env.sh || exit 1
ARMS="SDR_ABLATE=0 SDR_ABLATE=1 SDR_ABLATE=2 SDR_ABLATE=4" CFGS="cfg3" REPS=2 bash scripts/sweep_env.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider \
  -rf --timeout 300 --timeout-method thread -k "f16" > "$OUT/pytest_f16.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_f16.log"; [ $rc -eq 0 ] || { echo "pytest f16 rc=$rc"; exit $rc; }
ARMS="SDR_F16_MFMA=1 SDR_F16_MFMA=0" CFGS="cfg5h" REPS=2 bash scripts/sweep_env.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_dropin.py -m gpu -x -q -p no:cacheprovider \
  -rf --timeout 300 --timeout-method thread -k "stereo or sdr_project" > "$OUT/pytest_stereo.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_stereo.log"; [ $rc -eq 0 ] || { echo "pytest stereo rc=$rc"; exit $rc; }
NBLK=3000 REPS=2 timeout -k 10 600 bash scripts/time_project.sh || exit 1
