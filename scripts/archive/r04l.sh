#!/bin/bash
# r04l: loader-ring f32 front end (SDR_FIR_RING=1): parity, then cfg2 A/B against fir_tile_sc
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "ring" > gpurun_out/r04l_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04l_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04l_pytest.log | head; exit $rc; }
ARMS="SDR_FIR_RING=0 SDR_FIR_RING=1 SDR_FIR_RING=1,SDR_ABLATE=2 SDR_FIR_RING=1,SDR_RING_WALK=0,SDR_ABLATE=2" CFGS="cfg2" REPS=2 bash scripts/sweep_env.sh
