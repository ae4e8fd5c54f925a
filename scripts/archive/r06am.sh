#!/bin/bash
# r06am: PLL screens at the other modes' IF rates (mode 1: 288 kHz, mode 3: 384 kHz; the
# reference's fmPLL runs at the IF rate, src/project.cpp:123), 16,384 streams x 3,000 blocks
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06am; mkdir -p $OUT
for fs in 288e3 384e3; do
  for seed in 101 102; do
    timeout -k 10 200 python -u tests/pll_screen.py --streams 16384 --blocks 3000 --seed $seed --fs $fs >> $OUT/screens.jsonl 2>> $OUT/screen.err || exit 1
    tail -1 $OUT/screens.jsonl | cut -c1-220
  done
done
exit 0
