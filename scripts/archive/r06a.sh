#!/bin/bash
# r06a: the full-output bench-launch tests (cfg2 every stream x both kernels, cfg4x8, cfg5 every output)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06a; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_fullsize.py -m gpu -x -v -p no:cacheprovider --timeout 300 --timeout-method thread \
  -k "cfg2_full_f32 or cfg4x8 or cfg5_full_windows" > $OUT/pytest.log 2>&1; rc=$?
tail -8 $OUT/pytest.log; exit $rc
