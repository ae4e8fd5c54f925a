#!/bin/bash
# r04t: fir_long_mfma with one 1,024-output tile per wave (SDR_F16_NT=1: 4,096 outputs per
# workgroup, twice the workgroups) -- f16 parity under it, then the cfg5h A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SDR_F16_NT=1 timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16" > gpurun_out/r04t_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04t_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04t_pytest.log | head; exit $rc; }
ARMS="SDR_F16_NT=2 SDR_F16_NT=1" CFGS="cfg5h" REPS=3 bash scripts/sweep_env.sh
