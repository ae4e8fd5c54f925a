#!/bin/bash
# r04k: resample_lp loader: DMAs before edge loads and state copy (-DSDR_LP_EARLY=1), with/without the ordered scan
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for l in early ordearly; do
SDRHIP_LIB=$PWD/ab/$l.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "resample or cfg3" > gpurun_out/r04k_pytest_$l.log 2>&1 || { tail -5 gpurun_out/r04k_pytest_$l.log; exit 1; }
tail -1 gpurun_out/r04k_pytest_$l.log
done
ARMS="tree ab/early.so ab/ord.so ab/ordearly.so" CFGS="cfg3" REPS=3 bash scripts/ab_libs.sh
