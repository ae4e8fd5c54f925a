#!/bin/bash
# GPU tests, then same-box A/B of the working tree against ab/*.so builds,
# then (optional) the fir_tile timeline trace.
#   TAG=x LIBS="ab/prev.so" CFGS="cfg2 cfg2u8" REPS=3 [TRACE=1] bash scripts/gpu_ab_round.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-abr}
mkdir -p "$OUT"
if [ "${TESTS:-1}" = 1 ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider -rf --timeout 180 --timeout-method thread \
    > "$OUT/pytest.log" 2>&1
  rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
for rep in $(seq ${REPS:-3}); do
  for cfg in ${CFGS:-cfg2}; do
    for l in tree ${LIBS:-}; do
      if [ "$l" = tree ]; then unset SDRHIP_LIB; else export SDRHIP_LIB=$PWD/$l; fi
      r=$(timeout -k 10 120 python bench.py --config $cfg --steps ${STEPS:-100} --warmup 3 --no-cpu-baseline 2>>"$OUT/bench.err" |
          python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'], (d.get('fma_variant') or {}).get('ms_per_step'))")
      rc=$?; echo "rep $rep $cfg $l: $r"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
unset SDRHIP_LIB
if [ -n "${TRACE:-}" ]; then
  TAG=${TAG:-abr}/trace ARMS="${TRACE_ARMS:-default}" bash scripts/trace_fir.sh || exit $?
fi
