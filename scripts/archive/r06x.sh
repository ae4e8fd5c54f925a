#!/bin/bash
# r06x: stereo0 / stereo0w / mono0 under more HIP hardware queues per process
# (GPU_MAX_HW_QUEUES 4 = the default, 8, 16), same box, alternating
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06x; mkdir -p $OUT
for rep in 1 2; do
  for cfg in stereo0 stereo0w; do
    for q in 4 8 16; do
      GPU_MAX_HW_QUEUES=$q timeout -k 10 300 python bench.py --config $cfg --steps 30 --warmup 3 --no-cpu-baseline \
        > $OUT/b_${cfg}_q${q}_$rep.json 2>>$OUT/bench.err || exit 1
      python3 -c "import json;d=json.load(open('$OUT/b_${cfg}_q${q}_$rep.json'));print('rep $rep $cfg queues=$q', d['ms_per_step'], d['sustained']['ms_per_step'])" | tee -a $OUT/summary.txt
    done
  done
done
exit 0
