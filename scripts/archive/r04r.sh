#!/bin/bash
# r04r: three-stage stereo pipeline (front | PLL | post): parity, then stereo0 / stereo0w A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_scale.py tests/test_dropin.py tests/test_capi.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "stereo or sdr_project or symbols" > gpurun_out/r04r_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04r_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04r_pytest.log | head; exit $rc; }
ARMS="SDR_BENCH_STEREO_PIPE=1 SDR_BENCH_STEREO_PIPE=2" CFGS="stereo0 stereo0w" REPS=2 bash scripts/sweep_env.sh
