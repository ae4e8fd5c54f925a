#!/bin/bash
# r04u: fir_long_mfma with the first workgroup's state loads in the first load batch
# (SDR_F16_HEAD=1) -- f16 parity, then the cfg5h A/B against the old order
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16" > gpurun_out/r04u_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04u_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04u_pytest.log | head; exit $rc; }
ARMS="SDR_F16_HEAD=0 SDR_F16_HEAD=1" CFGS="cfg5h" REPS=3 bash scripts/sweep_env.sh
