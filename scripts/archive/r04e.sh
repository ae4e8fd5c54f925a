#!/bin/bash
# r04e: front-end VGPR taps, fp16 MFMA and the two-stage stereo schedule: parity, then A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04e; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider \
  -rf --timeout 300 --timeout-method thread -k "frontend or cfg2 or f16" > "$OUT/pytest_fe.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_fe.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAILED|Error" "$OUT/pytest_fe.log" | head; exit $rc; }
ARMS="SDR_F16_MFMA=1 SDR_F16_MFMA=0" CFGS="cfg5h" REPS=2 bash scripts/sweep_env.sh || exit 1
ARMS="SDR_FIR_VTAP_U8=0 SDR_FIR_VTAP_U8=1" CFGS="cfg2u8 mono0" REPS=2 bash scripts/sweep_env.sh || exit 1
ARMS="SDR_FIR_VTAP=0 SDR_FIR_VTAP=1" CFGS="cfg2" REPS=2 bash scripts/sweep_env.sh || exit 1
timeout -k 10 600 python -u -m pytest tests/test_dropin.py tests/test_gpu_scale.py -m gpu -x -q -p no:cacheprovider \
  -rf --timeout 300 --timeout-method thread -k "stereo or sdr_project" > "$OUT/pytest_stereo.log" 2>&1
rc=$?; tail -3 "$OUT/pytest_stereo.log"; [ $rc -eq 0 ] || { echo "pytest stereo rc=$rc"; grep -E "FAILED|Error" "$OUT/pytest_stereo.log" | head; exit $rc; }
ARMS="SDR_BENCH_STEREO_PIPE=0 SDR_BENCH_STEREO_PIPE=1" CFGS="stereo0" REPS=2 bash scripts/sweep_env.sh || exit 1
NBLK=3000 REPS=2 MODES=0 timeout -k 10 600 bash scripts/time_project.sh || exit 1
