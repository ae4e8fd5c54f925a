#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_var; mkdir -p "$OUT"
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 30 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r"; return $rc; }
export SDR_FIR_STREAM=0
for v in 2x1p 2x1r 4x1r; do
  for a in 0 1 2; do
    b "$v ablate=$a" SDR_FIR_VARIANT=$v SDR_ABLATE=$a || exit 1
    b "$v ablate=$a nt" SDR_FIR_VARIANT=$v SDR_ABLATE=$a SDRHIP_LIB=$PWD/ab/nt.so || exit 1
  done
done
for w in 12 16 32; do b "4x1r wpc=$w nt" SDR_FIR_VARIANT=4x1r SDR_WG_PER_CU=$w SDRHIP_LIB=$PWD/ab/nt.so || exit 1; done
exit 0
