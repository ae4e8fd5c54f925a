#!/bin/bash
# r04o: split discriminator in fir_tile_sc (parity + same-box A/B), then the PLL saturation run (r04n)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "frontend or cfg2 or u8 or smoke" > gpurun_out/r04o_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04o_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04o_pytest.log | head; exit $rc; }
ARMS="tree ab/nosplit.so" CFGS="cfg2 cfg2u8" REPS=3 bash scripts/ab_libs.sh || exit 1
bash scripts/r04n.sh
