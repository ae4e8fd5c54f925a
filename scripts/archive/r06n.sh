#!/bin/bash
# r06n: closing record, part 1 -- the whole GPU suite and smoke, then every
# bench config with its CPU baseline (cfg5b / cfg5hb included).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r06n}; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_cfg2.json 2> $OUT/bench.err || exit 1
for c in cfg2u8 cfg3 cfg4 cfg4x8 cfg5 cfg5b cfg5h cfg5hb mono0 stereo0 stereo0w; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 3 > $OUT/bench_$c.json 2>>$OUT/bench.err || exit 1
done
for f in $OUT/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));c=d['cpu_baseline'] or {};print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('sustained',{}).get('ms_per_step'), c.get('value'), c.get('kind'))"; done
exit 0
