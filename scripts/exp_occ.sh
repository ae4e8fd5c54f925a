#!/bin/bash
# Occupancy sensitivity of fir_tile (cfg2, cfg2u8; warm): pad the dynamic LDS so fewer waves fit per CU.
# LDS per one-wave workgroup is 10,976 B (14 per CU); +1,000 -> 13, +2,000 -> 12, +4,000 -> 10, +12,000 -> 7.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_occ; mkdir -p "$OUT"
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 100 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'], d.get('fma_variant',{}).get('ms_per_step'))")
  rc=$?; echo "$label: $r" | tee -a "$OUT/results.txt"; return $rc; }
for rep in 1 2; do
  for pad in 0 1000 2000 4000 12000; do b "cfg2 pad$pad rep$rep" SDR_LDS_PAD=$pad || exit 1; done
  for pad in 0 1000 2000 4000; do CFG=cfg2u8 b "u8 pad$pad rep$rep" SDR_LDS_PAD=$pad || exit 1; done
done
