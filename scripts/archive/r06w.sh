#!/bin/bash
# r06w: the timed window with and without a 2 ms spin kernel ahead of its start event
# (--head-start-ms), same box, alternating: timed vs sustained ms per step
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06w; mkdir -p $OUT
for rep in 1 2 3; do
  for cfg in cfg5h cfg2 cfg5 mono0; do
    for hs in 0 2; do
      timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 5 --no-cpu-baseline --head-start-ms $hs \
        > $OUT/b_${cfg}_h${hs}_$rep.json 2>>$OUT/bench.err || exit 1
      python3 -c "import json;d=json.load(open('$OUT/b_${cfg}_h${hs}_$rep.json'));print('rep $rep $cfg head=$hs', d['ms_per_step'], d['roofline']['frac'], d['sustained']['ms_per_step'])" | tee -a $OUT/summary.txt
    done
  done
done
timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline > $OUT/b_driver_shape.json 2>>$OUT/bench.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/b_driver_shape.json'));print('driver shape (20 steps)', d['ms_per_step'], d['roofline']['frac'], d['config']['launch'])" | tee -a $OUT/summary.txt
exit 0
