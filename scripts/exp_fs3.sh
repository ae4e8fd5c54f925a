#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_fs; mkdir -p "$OUT"
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 30 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r"; return $rc; }
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
   -k "frontend or fir_decim or block_size or full_size" > "$OUT/pytest3.log" 2>&1
rc=$?; tail -2 "$OUT/pytest3.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
for l in nl1 nl2 nl4; do for a in 0 1 2; do b "$l ablate=$a" SDRHIP_LIB=$PWD/ab/$l.so SDR_ABLATE=$a || exit 1; done; done
exit 0
