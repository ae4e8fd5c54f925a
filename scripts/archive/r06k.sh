#!/bin/bash
# r06k: pipelined mono0 with the back stage's audio FIR in small groups (SDR_MONO_BACK_WPG) vs one call
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06k; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 300 \
  --timeout-method thread -k "mono_two_stage" > $OUT/pytest_mono.log 2>&1; rc=$?
tail -1 $OUT/pytest_mono.log; [ $rc -eq 0 ] || exit $rc
for r in 1 2; do
  timeout -k 10 300 python bench.py --config mono0 --steps 100 --warmup 3 --no-cpu-baseline --mono-pipeline 0 \
    > $OUT/b_mp0_$r.json 2>>$OUT/bench.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/b_mp0_$r.json'));print('$r one-call', d['ms_per_step'], d.get('sustained',{}).get('ms_per_step'))"
  for wpg in 1 2 4 16; do
    SDR_MONO_BACK_WPG=$wpg timeout -k 10 300 python bench.py --config mono0 --steps 100 --warmup 3 --no-cpu-baseline \
      --mono-pipeline 1 > $OUT/b_w${wpg}_$r.json 2>>$OUT/bench.err || exit 1
    python3 -c "import json;d=json.load(open('$OUT/b_w${wpg}_$r.json'));print('$r pipelined wpg=$wpg', d['ms_per_step'], d.get('sustained',{}).get('ms_per_step'))"
  done
done
