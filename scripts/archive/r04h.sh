#!/bin/bash
# r04h: VGPR-tap u8 kernel, LDS read-ahead depth 1 / 2 (tree) / 3, full and scan-only (ABLATE=1)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "u8_golden or batched" > gpurun_out/r04h_pytest.log 2>&1 || { tail -5 gpurun_out/r04h_pytest.log; exit 1; }
tail -1 gpurun_out/r04h_pytest.log
ARMS="tree:SDR_FIR_VT_U8=1 ab/pf1.so:SDR_FIR_VT_U8=1 ab/pf3.so:SDR_FIR_VT_U8=1 tree:SDR_FIR_VT_U8=1,SDR_ABLATE=1 ab/pf1.so:SDR_FIR_VT_U8=1,SDR_ABLATE=1 ab/pf3.so:SDR_FIR_VT_U8=1,SDR_ABLATE=1 tree:SDR_FIR_VT_U8=0" CFGS="cfg2u8" REPS=2 bash scripts/ab_libs.sh
