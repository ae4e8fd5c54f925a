#!/bin/bash
# r05t (r05s + no store drain in tile 0's carry, parallel prev products):
# fir_tile_sc tile 0 with its extra loads in the span's batch
# (SDR_SC_T0PRE) -- front-end / mono / stereo parity, same-box A/B against
# the build without it (ab/t0off.so) on cfg2 / cfg2u8 / mono0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05t; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_dropin.py tests/test_gpu_scale.py -m gpu -x -q \
  -p no:cacheprovider --timeout 200 --timeout-method thread -k "frontend or u8 or cfg2 or cfg4 or nonfinite or mono or stereo or golden or demod" > $OUT/pytest.log 2>&1; rc=$?
tail -1 $OUT/pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest.log | head -20; exit $rc; }
ARMS="tree ab/t0off.so ab/pre3.so" CFGS="cfg2 cfg2u8 mono0" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_t0pre.txt 2>&1; rc=$?; cat $OUT/ab_t0pre.txt; [ $rc -eq 0 ] || exit $rc
for v in "SDR_ABLATE=12" "SDR_ABLATE=13"; do
  echo "== $v" >> $OUT/f16_trace.txt
  env $v SDRHIP_LIB=$PWD/ab/timing.so SDR_F16_TRACE=1 REPS=2 timeout -k 10 200 python -u scripts/f16_trace.py 2>&1 | grep -E "span|staging|barrier \(" >> $OUT/f16_trace.txt; rc=$?
  [ $rc -eq 0 ] || exit $rc
done
cat $OUT/f16_trace.txt
exit 0
