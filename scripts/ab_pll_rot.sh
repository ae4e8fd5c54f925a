#!/bin/bash
# Same-box check of the rotation phase detector (pll_fast.hpp atan2_rot):
# PLL / stereo parity tests, PLL kernel timing per mode against ab/head.so,
# and the stereo bench A/B (first: bash scripts/build_ab.sh <rev> head).
set -o pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out/pll_rot
timeout -k 10 400 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/ -k "pll or stereo" \
  > gpurun_out/pll_rot/pytest.log 2>&1 || { tail -n 40 gpurun_out/pll_rot/pytest.log; exit 1; }
tail -n 1 gpurun_out/pll_rot/pytest.log
for t in 0 1.6e7; do
  echo "== new, trig0 $t"; timeout -k 10 120 python -u scripts/pll_modes.py $t || exit 1
  echo "== head, trig0 $t"; SDRHIP_LIB=$PWD/ab/head.so timeout -k 10 120 python -u scripts/pll_modes.py $t || exit 1
done 2>&1 | tee gpurun_out/pll_rot/pll_modes.txt
LIBS="ab/head.so" CFGS="stereo0 stereo0w" REPS=2 STEPS=30 timeout -k 10 500 bash scripts/ab.sh 2>&1 | tee gpurun_out/pll_rot/ab.txt
