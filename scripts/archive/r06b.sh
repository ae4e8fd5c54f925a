#!/bin/bash
# r06b: libm_exact on the device (every-float sin/cos hash, ROCm diff, fixtures, atan2 screen), the PLL /
# stereo / mono parity tests on the new routines, cfg5b / cfg5hb / stereo bench lines
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06b; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_libm.py -m gpu -x -v -s -p no:cacheprovider --timeout 300 \
  --timeout-method thread > $OUT/pytest_libm.log 2>&1; rc=$?
tail -12 $OUT/pytest_libm.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_scale.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread -k "pll or stereo or mono or project" > $OUT/pytest_pll.log 2>&1; rc=$?
tail -4 $OUT/pytest_pll.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_pll.log | head -20; exit $rc; }
for c in stereo0 stereo0w cfg5b cfg5hb cfg5h; do
  timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 3 --no-cpu-baseline > $OUT/bench_$c.json 2>>$OUT/bench.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/bench_$c.json'));print('$c', d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('sustained',{}).get('ms_per_step'))"
done
exit 0
