#!/bin/bash
# Full GPU parity, then tile exact vs fma on cfg2 / cfg2u8 (same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_r1b; mkdir -p "$OUT"
RES=$OUT/results.txt
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 30 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r" | tee -a "$RES"; return $rc; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
   > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
for rep in 1 2; do
  b "cfg2 exact rep$rep" || exit 1
  b "cfg2 fma rep$rep" SDR_BENCH_ARITH=fma || exit 1
  b "cfg2 stream rep$rep" SDR_FIR_STREAM=1 || exit 1
  CFG=cfg2u8 b "cfg2u8 exact rep$rep" || exit 1
  CFG=cfg2u8 b "cfg2u8 fma rep$rep" SDR_BENCH_ARITH=fma || exit 1
done
exit 0
