#!/bin/bash
# r06m: PLL with the 32-ulp sine/cosine window: parity, then old (OCML) / chunk (r06 libm, one window) / win A/B
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06m; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_scale.py tests/test_gpu_libm.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread -k "pll or stereo or libm" > $OUT/pytest_pll.log 2>&1; rc=$?
tail -2 $OUT/pytest_pll.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_pll.log | head -20; exit $rc; }
TAG=r06m LIBS="old_stereo new_chunk new_win old_stereo new_win" bash scripts/archive/r06d.sh || exit 1
for r in 1 2; do for lib in old_stereo new_chunk new_win; do for c in stereo0 stereo0w; do
  SDRHIP_LIB=$PWD/ab/$lib.so timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 3 --no-cpu-baseline \
    --sustain-seconds 1 > $OUT/bb_${lib}_${c}_$r.json 2>>$OUT/bench.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/bb_${lib}_${c}_$r.json'));print('$r $lib $c', d['ms_per_step'], d.get('sustained',{}).get('ms_per_step'))"
done; done; done
