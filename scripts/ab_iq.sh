#!/bin/bash
# fir_tile_iq (I/Q-paired packed arithmetic) vs the planar fir_tile: the
# front-end parity tests, then a same-box A/B of SDR_FIR_IQ on cfg2/cfg2u8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab_iq}
mkdir -p "$OUT"
timeout -k 10 900 python -u -m pytest tests -m gpu -x -v -p no:cacheprovider -rf --timeout 180 --timeout-method thread \
  --durations=15 > "$OUT/pytest.log" 2>&1
rc=$?; tail -4 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
timeout -k 10 120 python -c "import __graft_entry__ as g; g.smoke()" > "$OUT/smoke.log" 2>&1
rc=$?; tail -2 "$OUT/smoke.log"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2 3; do
  for cfg in ${CFGS:-cfg2 cfg2u8}; do
    for v in 1 0; do
      r=$(SDR_FIR_IQ=$v timeout -k 10 120 python bench.py --config $cfg --steps 100 --warmup 3 --no-cpu-baseline 2>>"$OUT/bench.err" |
          python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'], d.get('fma_variant',{}).get('ms_per_step'))")
      rc=$?; echo "rep $rep $cfg SDR_FIR_IQ=$v: $r"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
