#!/bin/bash
# r06i: certificate-only PLL re-run: PLL/stereo parity, then old / chunk / cert A/B (profiler + bench)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06i; mkdir -p $OUT
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_scale.py tests/test_gpu_libm.py -m gpu -x -q \
  -p no:cacheprovider --timeout 300 --timeout-method thread -k "pll or stereo or libm" > $OUT/pytest_pll.log 2>&1; rc=$?
tail -3 $OUT/pytest_pll.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_pll.log | head -20; exit $rc; }
TAG=r06i LIBS="old_stereo new_chunk new_cert old_stereo new_cert" bash scripts/archive/r06d.sh || exit 1
for r in 1 2; do for lib in old_stereo new_cert; do
  SDRHIP_LIB=$PWD/ab/$lib.so timeout -k 10 300 python bench.py --config stereo0 --steps 50 --warmup 3 --no-cpu-baseline \
    --sustain-seconds 1 > $OUT/bb_${lib}_$r.json 2>>$OUT/bench.err || exit 1
  python3 -c "import json;d=json.load(open('$OUT/bb_${lib}_$r.json'));print('$r $lib stereo0', d['ms_per_step'], d.get('sustained',{}).get('ms_per_step'))"
done; done
