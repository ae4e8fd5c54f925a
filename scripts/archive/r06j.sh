#!/bin/bash
# r06j: two-stage mono: parity (pipelined over two contexts), then mono0 one-call vs pipelined, same box
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06j; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "mono" > $OUT/pytest_mono.log 2>&1; rc=$?
tail -3 $OUT/pytest_mono.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_mono.log | head -20; exit $rc; }
for r in 1 2; do for mp in 0 1; do
  timeout -k 10 300 python bench.py --config mono0 --steps 100 --warmup 3 --no-cpu-baseline --mono-pipeline $mp \
    > $OUT/b_mp${mp}_$r.json 2>>$OUT/bench.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/b_mp${mp}_$r.json'));print('$r mono-pipeline=$mp', d['ms_per_step'], d.get('sustained',{}).get('ms_per_step'), d['roofline']['frac'])"
done; done
