#!/bin/bash
# cfg2 / cfg2u8 with the clock-ramp warmup: prefetch-1 tile (2x1r) grid sizes, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_pf1; mkdir -p "$OUT"
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 100 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'], d.get('fma_variant',{}).get('ms_per_step'))")
  rc=$?; echo "$label: $r" | tee -a "$OUT/results.txt"; return $rc; }
for rep in 1 2; do
  b "default rep$rep" || exit 1
  for w in 24 32 48 64 96; do b "2x1r wpc$w rep$rep" SDR_FIR_VARIANT=2x1r SDR_WG_PER_CU=$w || exit 1; done
  CFG=cfg2u8 b "u8 default rep$rep" || exit 1
  for w in 48 64; do CFG=cfg2u8 b "u8 wpc$w rep$rep" SDR_WG_PER_CU=$w || exit 1; done
done
