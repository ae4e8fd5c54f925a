#!/bin/bash
# Parity of the explicit-wait staging, then same-box A/B vs the HEAD build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_wait; mkdir -p "$OUT"
RES=$OUT/results.txt
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 30 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r" | tee -a "$RES"; return $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
   > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
for rep in 1 2; do
  b "old tile rep$rep" SDR_FIR_STREAM=0 SDRHIP_LIB=$PWD/ab/old.so || exit 1
  b "new tile exact rep$rep" SDR_FIR_STREAM=0 || exit 1
  b "new tile fma rep$rep" SDR_FIR_STREAM=0 SDR_BENCH_ARITH=fma || exit 1
  b "new tile exact wpc16 rep$rep" SDR_FIR_STREAM=0 SDR_WG_PER_CU=16 || exit 1
  b "new tile exact wpc32 rep$rep" SDR_FIR_STREAM=0 SDR_WG_PER_CU=32 || exit 1
done
exit 0
