#!/bin/bash
# r04s: fir_tile_sc with R = 4 (SDR_FIR_SC_R4=1): parity under it, then cfg2u8 / cfg2 / mono0 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SDR_FIR_SC_R4=1 timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "frontend or cfg2 or u8 or mono" > gpurun_out/r04s_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04s_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04s_pytest.log | head; exit $rc; }
ARMS="SDR_FIR_SC_R4=0 SDR_FIR_SC_R4=1" CFGS="cfg2u8 cfg2 mono0" REPS=2 bash scripts/sweep_env.sh
