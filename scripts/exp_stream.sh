#!/bin/bash
# Streaming experiments for the headline kernel (round 1, session 2):
# read ceilings by cache policy, nt A/B, persistence sweep, ablations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_stream
mkdir -p "$OUT"
b() {  # label, env...
  local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 30 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r"; return $rc
}
timeout -k 10 300 ./tools/ubench_stream > "$OUT/ubench.txt" 2>&1; rc=$?; cat "$OUT/ubench.txt"; [ $rc -eq 0 ] || exit $rc
for rep in 1 2; do
  b "tree" X=1 || exit 1
  b "nt" SDRHIP_LIB=$PWD/ab/nt.so || exit 1
done
for w in 3 6 12 24 48; do b "wpc=$w" SDR_WG_PER_CU=$w || exit 1; b "nt wpc=$w" SDR_WG_PER_CU=$w SDRHIP_LIB=$PWD/ab/nt.so || exit 1; done
for a in 1 2 3 4; do b "ablate=$a" SDR_ABLATE=$a || exit 1; b "nt ablate=$a" SDR_ABLATE=$a SDRHIP_LIB=$PWD/ab/nt.so || exit 1; done
exit 0
