#!/bin/bash
# r04f: u8 front end on fir_tile_grp with VGPR taps (TM 2): parity, then same-box A/B.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-r04f}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_dropin.py -m gpu -x -q -p no:cacheprovider \
  -rf --timeout 300 --timeout-method thread -k "u8 or odd_shapes or batched or mono or stereo or sdr_project" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; grep -E "FAILED|Error" "$OUT/pytest.log" | head; exit $rc; }
ARMS="SDR_FIR_VT_U8=0 SDR_FIR_VT_U8=1" CFGS="cfg2u8 mono0 stereo0" REPS=2 bash scripts/sweep_env.sh || exit 1
