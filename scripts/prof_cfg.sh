#!/bin/bash
# Kernel trace (rocprofv3 --kernel-trace --stats) of one bench config; the
# timed region's per-kernel averages via scripts/prof_timed.py.
#   TAG=r04g CFGS="cfg5h cfg3" bash scripts/prof_cfg.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-prof}; mkdir -p "$OUT"
export TMPDIR=/tmp
STEPS=${STEPS:-100}
for cfg in ${CFGS:-cfg2}; do
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof_$cfg" -o bench \
    -- python3 bench.py --config $cfg --steps $STEPS --warmup 5 --no-cpu-baseline --no-fma-variant --sustain-seconds 0 \
    > "$OUT/prof_bench_$cfg.json" 2>> "$OUT/prof.err"
  rc=$?; echo "rocprof $cfg rc=$rc"; [ $rc -eq 0 ] || exit $rc
  python scripts/prof_timed.py "$(find $OUT/prof_$cfg -name '*kernel_trace.csv' | head -1)" $STEPS \
    "$OUT/prof_timed_$cfg.json" "$OUT/prof_bench_$cfg.json"
  python3 -c "
import json; d=json.load(open('$OUT/prof_timed_$cfg.json'))
for k in d['kernels'][:6]: print('$cfg', k['kernel'][:70], k['calls'], k.get('avg_us_timed'))
"
done
