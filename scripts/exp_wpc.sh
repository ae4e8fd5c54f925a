#!/bin/bash
# cfg2 exact: sweep of the fir_tile grid size (SDR_WG_PER_CU) and tile walk (SDR_TILE_WALK).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_wpc; mkdir -p "$OUT"
RES=$OUT/results.txt
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 40 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r" | tee -a "$RES"; return $rc; }
for rep in 1 2; do
  b "default rep$rep" || exit 1
  for w in 3 4 6 8 12 16 32 64; do
    b "wpc$w walk1 rep$rep" SDR_WG_PER_CU=$w || exit 1
    b "wpc$w walk0 rep$rep" SDR_WG_PER_CU=$w SDR_TILE_WALK=0 || exit 1
  done
done
exit 0
