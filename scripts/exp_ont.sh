#!/bin/bash
# Non-temporal demod output stores (ab/ont.so) vs tree, warm same box; parity of ont first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=$ROOT/gpurun_out/exp_ont; mkdir -p "$OUT"
SDRHIP_LIB=$ROOT/ab/ont.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k frontend -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$OUT/pytest_ont.log" 2>&1
rc=$?; echo "parity ont: $(tail -1 $OUT/pytest_ont.log)"; [ $rc -eq 0 ] || exit $rc
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 100 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'], d.get('fma_variant',{}).get('ms_per_step'))")
  rc=$?; echo "$label: $r" | tee -a "$OUT/results.txt"; return $rc; }
for rep in 1 2 3; do
  b "cfg2 tree rep$rep" || exit 1
  b "cfg2 ont rep$rep" SDRHIP_LIB=$ROOT/ab/ont.so || exit 1
  CFG=cfg2u8 b "u8 tree rep$rep" || exit 1
  CFG=cfg2u8 b "u8 ont rep$rep" SDRHIP_LIB=$ROOT/ab/ont.so || exit 1
done
