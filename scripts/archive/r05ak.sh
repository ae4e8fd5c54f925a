#!/bin/bash
# r05ak: the round-end check on the committed tree -- what the driver runs:
# the GPU suite, smoke(), the default bench line.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ak; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -1 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -1 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench.json 2> $OUT/bench.err || exit 1
python3 -c "import json;d=json.load(open('$OUT/bench.json'));print(d['value'], d['ms_per_step'], d['roofline']['frac'], d['roofline']['traffic'], d['sustained']['ms_per_step'], d['cpu_baseline']['value'])"
exit 0
