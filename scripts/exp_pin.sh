#!/bin/bash
# Same-box A/B of the staging build switches (cfg2 exact) against the previous commit's build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=$ROOT/gpurun_out/exp_pin; mkdir -p "$OUT"
RES=$OUT/results.txt
b() { local label=$1 dir=$2; shift 2
  r=$(cd "$dir" && env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 40 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r" | tee -a "$RES"; return $rc; }
for rep in 1 2 3; do
  b "head rep$rep" ab/head || exit 1
  b "tree rep$rep" . || exit 1
  for v in nopin nodrain neither; do b "$v rep$rep" . SDRHIP_LIB=$ROOT/ab/$v.so || exit 1; done
done
exit 0
