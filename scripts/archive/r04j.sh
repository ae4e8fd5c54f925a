#!/bin/bash
# r04j: resample_lp with the ordered scan (K products, then K sums; -DSDR_LP_ORD=1): parity on that build, then cfg3 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SDRHIP_LIB=$PWD/ab/ord.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "resample or cfg3" > gpurun_out/r04j_pytest.log 2>&1 || { tail -5 gpurun_out/r04j_pytest.log; exit 1; }
tail -1 gpurun_out/r04j_pytest.log
ARMS="tree ab/ord.so tree:SDR_ABLATE=1 ab/ord.so:SDR_ABLATE=1" CFGS="cfg3" REPS=3 bash scripts/ab_libs.sh
