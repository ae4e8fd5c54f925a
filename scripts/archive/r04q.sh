#!/bin/bash
# r04q: resample_lp item DMA with the non-temporal policy: parity on that build, cfg3 A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
SDRHIP_LIB=$PWD/ab/lpnt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 200 --timeout-method thread -k "resample or cfg3" > gpurun_out/r04q_pytest.log 2>&1 || { tail -5 gpurun_out/r04q_pytest.log; exit 1; }
tail -1 gpurun_out/r04q_pytest.log
ARMS="tree ab/lpnt.so" CFGS="cfg3" REPS=4 bash scripts/ab_libs.sh
