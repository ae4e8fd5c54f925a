#!/bin/bash
# r04d: resample_pk2 (packed phase pairs) parity first, then cfg3 A/B against
# resample_lp, then the rest of r04c (VTAP front end, ablations, fp16 MFMA,
# stereo split).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04d; mkdir -p $OUT
timeout -k 10 120 ./tools/ubench_ldsmix > "$OUT/ubench_ldsmix.txt" 2>&1; rc=$?; cat "$OUT/ubench_ldsmix.txt"; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider \
  -rf --timeout 300 --timeout-method thread -k "resample or cfg3" > "$OUT/pytest_resample.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_resample.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "Error|assert" "$OUT/pytest_resample.log" | head -20; exit $rc; }
ARMS="SDR_RESAMPLE_PK2=1 SDR_RESAMPLE_PK2=0" CFGS="cfg3" REPS=3 bash scripts/sweep_env.sh || exit 1
ARMS="SDR_ABLATE=1 SDR_ABLATE=2 SDR_ABLATE=4" CFGS="cfg3" REPS=1 bash scripts/sweep_env.sh || exit 1
ARMS="SDR_RESAMPLE_PK2=1,SDR_ABLATE=1 SDR_RESAMPLE_PK2=1,SDR_ABLATE=2" CFGS="cfg3" REPS=1 bash scripts/sweep_env.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider \
  -rf --timeout 300 --timeout-method thread -k "frontend or cfg2 or f16" > "$OUT/pytest_fe.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_fe.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
ARMS="SDR_FIR_VTAP_U8=0 SDR_FIR_VTAP_U8=1" CFGS="cfg2u8 mono0" REPS=2 bash scripts/sweep_env.sh || exit 1
ARMS="SDR_FIR_VTAP=0 SDR_FIR_VTAP=1" CFGS="cfg2" REPS=2 bash scripts/sweep_env.sh || exit 1
ARMS="SDR_F16_MFMA=1 SDR_F16_MFMA=0" CFGS="cfg5h" REPS=2 bash scripts/sweep_env.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_dropin.py -m gpu -x -q -p no:cacheprovider \
  -rf --timeout 300 --timeout-method thread -k "stereo or sdr_project" > "$OUT/pytest_stereo.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_stereo.log"; [ $rc -eq 0 ] || { echo "pytest stereo rc=$rc"; exit $rc; }
NBLK=3000 REPS=2 MODES=0 timeout -k 10 600 bash scripts/time_project.sh || exit 1
