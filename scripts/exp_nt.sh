#!/bin/bash
# Warm same-box A/B: non-temporal span loads (ab/nt.so) and grid sizes, cfg2 / cfg2u8.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=$ROOT/gpurun_out/exp_nt; mkdir -p "$OUT"
SDRHIP_LIB=$ROOT/ab/nt.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k frontend -p no:cacheprovider \
  --timeout 120 --timeout-method thread > "$OUT/pytest_nt.log" 2>&1
rc=$?; echo "parity nt: $(tail -1 $OUT/pytest_nt.log)"; [ $rc -eq 0 ] || exit $rc
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 100 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'], d.get('fma_variant',{}).get('ms_per_step'))")
  rc=$?; echo "$label: $r" | tee -a "$OUT/results.txt"; return $rc; }
for rep in 1 2; do
  b "cfg2 tree rep$rep" || exit 1
  b "cfg2 nt rep$rep" SDRHIP_LIB=$ROOT/ab/nt.so || exit 1
  for w in 40 96 128; do b "cfg2 tree wpc$w rep$rep" SDR_WG_PER_CU=$w || exit 1; done
  CFG=cfg2u8 b "u8 tree rep$rep" || exit 1
  CFG=cfg2u8 b "u8 nt rep$rep" SDRHIP_LIB=$ROOT/ab/nt.so || exit 1
  for w in 16 24 48 64; do CFG=cfg2u8 b "u8 tree wpc$w rep$rep" SDR_WG_PER_CU=$w || exit 1; done
done
