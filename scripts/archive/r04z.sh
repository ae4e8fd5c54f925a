#!/bin/bash
# r04z: the 8-wave fp16 default -- f16 / cfg5 tests (both shapes), smoke, default bench, cfg5h bench + trace
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r04z; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16 or cfg5" > $OUT/pytest.log 2>&1; rc=$?
tail -3 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1; tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2>$OUT/bench.err || exit 1
timeout -k 10 300 python bench.py --config cfg5h --steps 100 --warmup 3 --no-cpu-baseline > $OUT/bench_cfg5h.json 2>>$OUT/bench.err || exit 1
export TMPDIR=/tmp
timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof_cfg5h" -o k \
  -- python3 bench.py --config cfg5h --steps 100 --warmup 3 --no-cpu-baseline --no-fma-variant --sustain-seconds 0 \
  > $OUT/prof_bench_cfg5h.json 2>>$OUT/bench.err || exit 1
python scripts/prof_timed.py "$(find $OUT/prof_cfg5h -name '*kernel_trace.csv' | head -1)" 100 $OUT/prof_timed_cfg5h.json $OUT/prof_bench_cfg5h.json
find $OUT -name '*kernel_trace.csv' -delete
for f in $OUT/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));print('$f'.split('/')[-1], d['ms_per_step'], d['roofline']['frac'], d['sustained']['frac'])"; done
