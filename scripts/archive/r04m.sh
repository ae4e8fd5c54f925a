#!/bin/bash
# r04m: fp16 MFMA FIR with in-kernel state commit and LDS-built tap copies: parity, timing, trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16" > gpurun_out/r04m_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04m_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04m_pytest.log | head; exit $rc; }
ARMS="default" CFGS="cfg5h" REPS=3 bash scripts/sweep_env.sh || exit 1
TAG=r04m_prof CFGS="cfg5h" bash scripts/prof_cfg.sh
