#!/bin/bash
# PLL input prefetch: full GPU parity, then stereo0 A/B against the previous library (warm, same box).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=$ROOT/gpurun_out/exp_pll; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
   > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-stereo0} --steps 30 --warmup 3 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r" | tee -a "$OUT/results.txt"; return $rc; }
for rep in 1 2; do
  b "stereo0 prev rep$rep" SDRHIP_LIB=$ROOT/ab/prev.so || exit 1
  b "stereo0 tree rep$rep" || exit 1
done
