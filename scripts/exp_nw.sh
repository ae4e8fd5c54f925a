#!/bin/bash
# cfg2 warm: 1-, 2-, 4-wave workgroups sharing a span (SGPR taps, prefetch 1); parity of each first.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_nw; mkdir -p "$OUT"
for v in 2x2r 2x4r; do
  SDR_FIR_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -k "frontend" -p no:cacheprovider \
    --timeout 120 --timeout-method thread > "$OUT/pytest_$v.log" 2>&1
  rc=$?; echo "parity $v: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --steps 100 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'], d.get('fma_variant',{}).get('ms_per_step'))")
  rc=$?; echo "$label: $r" | tee -a "$OUT/results.txt"; return $rc; }
for rep in 1 2; do
  b "default rep$rep" || exit 1
  for v in 2x2r 2x4r; do for w in 16 32 64; do b "$v wpc$w rep$rep" SDR_FIR_VARIANT=$v SDR_WG_PER_CU=$w || exit 1; done; done
done
