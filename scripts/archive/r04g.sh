#!/bin/bash
# r04g: u8 front-end ablations per kernel (same box): no global loads (1), no scan (2)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ARMS="SDR_FIR_VT_U8=1 SDR_FIR_VT_U8=1,SDR_ABLATE=1 SDR_FIR_VT_U8=1,SDR_ABLATE=2 SDR_FIR_VT_U8=0,SDR_FIR_SC_U8=0 SDR_FIR_VT_U8=0,SDR_FIR_SC_U8=0,SDR_ABLATE=1 SDR_FIR_VT_U8=0,SDR_FIR_SC_U8=0,SDR_ABLATE=2 SDR_FIR_VT_U8=0 SDR_FIR_VT_U8=0,SDR_ABLATE=1 SDR_FIR_VT_U8=0,SDR_ABLATE=2" CFGS="cfg2u8" REPS=1 bash scripts/sweep_env.sh || exit 1
