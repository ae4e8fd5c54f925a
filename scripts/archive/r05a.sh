#!/bin/bash
# r05a: the round-5 parity additions (non-finite fixtures on every f32 FIR /
# demod kernel, cfg4's full single-call launch, fir_long at 8192 taps, destroy
# while another context's work is queued), then the whole GPU suite, smoke and
# this box's default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05a; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider --timeout 120 --timeout-method thread \
  -k "nonfinite or 8192 or cfg4_full or destroy_waits or two_stage" > $OUT/pytest_new.log 2>&1; rc=$?
tail -3 $OUT/pytest_new.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_new.log | head -20; exit $rc; }
timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -3 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_gpu.log | head -20; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1; tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2>$OUT/bench.err || exit 1
for c in cfg2u8 cfg3 cfg5h; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 3 --no-cpu-baseline > $OUT/bench_$c.json 2>>$OUT/bench.err || exit 1
done
for f in $OUT/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('sustained',{}).get('ms_per_step'))"; done
