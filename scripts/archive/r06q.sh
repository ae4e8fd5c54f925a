#!/bin/bash
# r06q: fir_long's in-kernel state commit (SDR_LONG_COMMIT): long-FIR parity
# under both paths, then cfg5 / cfg5b same-box A/B (commit in-kernel vs long_commit launch)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06q; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider \
  --timeout 120 --timeout-method thread -k "long or fir_block or fir_decim or cfg5 or nonfinite" > $OUT/pytest_long.log 2>&1; rc=$?
tail -2 $OUT/pytest_long.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_long.log | head -20; exit $rc; }
for rep in 1 2 3; do
  for c in 1 0; do
    for cfg in cfg5 cfg5b; do
      SDR_LONG_COMMIT=$c timeout -k 10 300 python bench.py --config $cfg --steps 100 --warmup 3 --no-cpu-baseline \
        > $OUT/b_${cfg}_c${c}_$rep.json 2>>$OUT/bench.err || exit 1
      python3 -c "import json;d=json.load(open('$OUT/b_${cfg}_c${c}_$rep.json'));print('rep $rep $cfg commit=$c', d['ms_per_step'], d['roofline']['frac'], d['sustained']['ms_per_step'])" | tee -a $OUT/summary.txt
    done
  done
done
exit 0
