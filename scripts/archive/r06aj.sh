#!/bin/bash
# r06aj: more PLL screens (certified step vs exact-library step), seeds 8..27,
# 16,384 streams x 3,000 blocks x 5,120 samples each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06aj; mkdir -p $OUT
for seed in $(seq 8 27); do
  timeout -k 10 200 python -u tests/pll_screen.py --streams 16384 --blocks 3000 --seed $seed >> $OUT/screens.jsonl 2>> $OUT/screen.err || exit 1
  tail -1 $OUT/screens.jsonl | cut -c1-200
done
exit 0
