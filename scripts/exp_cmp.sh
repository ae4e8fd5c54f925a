#!/bin/bash
# Same-box A/B of the front-end engines on cfg2: fir_stream (loader/consumer)
# vs fir_tile (register-staged), alternating, results appended to a file.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_cmp; mkdir -p "$OUT"
RES=$OUT/results.txt
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 30 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r" | tee -a "$RES"; return $rc; }
if [ "${SKIP_TESTS:-0}" != 1 ]; then
  timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
     -k "frontend or fir_decim or block_size or full_size" > "$OUT/pytest.log" 2>&1
  rc=$?; tail -2 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
fi
for rep in 1 2; do
  b "stream(default) rep$rep" SDR_FIR_STREAM=1 || exit 1
  b "tile rep$rep" SDR_FIR_STREAM=0 || exit 1
  for v in ${VARIANTS:-}; do b "$v rep$rep" SDRHIP_LIB=$PWD/ab/$v.so || exit 1; done
done
exit 0
