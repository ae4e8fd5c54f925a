#!/bin/bash
# r06u: long PLL screens, certified path vs exact-library path: 6 seeds x 16,384 streams
# x 3,000 blocks x 5,120 samples (2.5e11 PLL steps per seed)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06u; mkdir -p $OUT
for seed in 2 3 4 5 6 7; do
  timeout -k 10 400 python -u tests/pll_screen.py --streams 16384 --blocks 3000 --seed $seed >> $OUT/screens.jsonl 2>> $OUT/screen.err || exit 1
  tail -1 $OUT/screens.jsonl
done
exit 0
