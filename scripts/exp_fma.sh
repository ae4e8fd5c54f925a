#!/bin/bash
# Same-box A/B: exact (mul + add) vs fused multiply-add FIR arithmetic, plus
# the write-cost ubench.  Results appended to gpurun_out/exp_fma/results.txt.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_fma; mkdir -p "$OUT"
RES=$OUT/results.txt
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 30 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r" | tee -a "$RES"; return $rc; }
timeout -k 10 120 ./tools/ubench_rw > "$OUT/ubench_rw.txt" 2>&1 || { echo "ubench rc=$?"; exit 1; }
cat "$OUT/ubench_rw.txt"
F=$PWD/ab/fma.so
for rep in 1 2; do
  b "tile exact rep$rep" SDR_FIR_STREAM=0 || exit 1
  b "tile fma rep$rep" SDR_FIR_STREAM=0 SDRHIP_LIB=$F || exit 1
  b "tile fma 4x1r rep$rep" SDR_FIR_STREAM=0 SDRHIP_LIB=$F SDR_FIR_VARIANT=4x1r || exit 1
  b "stream fma rep$rep" SDR_FIR_STREAM=1 SDRHIP_LIB=$F || exit 1
  CFG=cfg2u8 b "u8 exact rep$rep" || exit 1
  CFG=cfg2u8 b "u8 fma rep$rep" SDRHIP_LIB=$F || exit 1
  CFG=cfg2u8 b "u8 fma 4x1r rep$rep" SDRHIP_LIB=$F SDR_FIR_VARIANT=4x1r || exit 1
done
exit 0
