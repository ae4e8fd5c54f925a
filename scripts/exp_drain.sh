#!/bin/bash
# GPU parity, then same-box A/B: previous commit's build vs the working tree (exact, fma).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=$ROOT/gpurun_out/exp_drain; mkdir -p "$OUT"
RES=$OUT/results.txt
b() { local label=$1 dir=$2; shift 2
  r=$(cd "$dir" && env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 40 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r" | tee -a "$RES"; return $rc; }
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
   > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
for rep in 1 2 3; do
  b "head rep$rep" ab/head || exit 1
  b "tree exact rep$rep" . || exit 1
  b "tree pf1 rep$rep" . SDR_FIR_VARIANT=2x1r || exit 1
  b "tree fma rep$rep" . SDR_BENCH_ARITH=fma || exit 1
  CFG=cfg2u8 b "head u8 rep$rep" ab/head || exit 1
  CFG=cfg2u8 b "tree u8 rep$rep" . || exit 1
done
exit 0
