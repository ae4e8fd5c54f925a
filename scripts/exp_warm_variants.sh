#!/bin/bash
# cfg2 exact with the clock-ramp warmup: fir_tile variants / grid sizes / stream kernel, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_wv; mkdir -p "$OUT"
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 100 --warmup 5 --no-cpu-baseline --no-fma-variant 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r" | tee -a "$OUT/results.txt"; return $rc; }
for rep in 1 2; do
  b "default rep$rep" || exit 1
  b "2x1r(pf1) rep$rep" SDR_FIR_VARIANT=2x1r || exit 1
  b "2x1(lds taps) rep$rep" SDR_FIR_VARIANT=2x1 || exit 1
  b "4x1r rep$rep" SDR_FIR_VARIANT=4x1r || exit 1
  b "2x4 rep$rep" SDR_FIR_VARIANT=2x4 || exit 1
  b "stream rep$rep" SDR_FIR_STREAM=1 || exit 1
  b "wpc16 rep$rep" SDR_WG_PER_CU=16 || exit 1
  b "wpc32 rep$rep" SDR_WG_PER_CU=32 || exit 1
  b "wpc48 rep$rep" SDR_WG_PER_CU=48 || exit 1
  b "walk0 rep$rep" SDR_TILE_WALK=0 || exit 1
done
