#!/bin/bash
# GPU parity, then same-box A/B (warm): previous commit's library vs the tree, cfg2 / cfg2u8 / mono0.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
ROOT=$PWD
OUT=$ROOT/gpurun_out/exp_u8pf; mkdir -p "$OUT"
timeout -k 10 400 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
   > "$OUT/pytest.log" 2>&1
rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 100 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'], d.get('fma_variant',{}).get('ms_per_step'))")
  rc=$?; echo "$label: $r" | tee -a "$OUT/results.txt"; return $rc; }
for rep in 1 2; do
  for c in cfg2 cfg2u8 mono0; do
    CFG=$c b "$c prev rep$rep" SDRHIP_LIB=$ROOT/ab/prev.so || exit 1
    CFG=$c b "$c tree rep$rep" || exit 1
  done
done
