#!/bin/bash
# Effect of the clock-ramp warmup on the cfg2 line (same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_warm; mkdir -p "$OUT"
for rep in 1 2; do
  for w in 0 0.25 1.0; do
    r=$(timeout -k 10 120 python bench.py --steps 20 --warmup 5 --warm-seconds $w --no-cpu-baseline 2>>"$OUT/err.log" |
        python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'], d['fma_variant']['ms_per_step'])") || exit 1
    echo "warm $w rep$rep: $r" | tee -a "$OUT/results.txt"
  done
done
for c in cfg2u8 cfg3 stereo0; do
  timeout -k 10 120 python bench.py --config $c --no-cpu-baseline > "$OUT/$c.json" 2>>"$OUT/err.log" || exit 1
  python -c "import json;d=json.load(open('$OUT/$c.json'));print('$c', d['ms_per_step'], d['roofline']['frac'], d['value'])"
done
