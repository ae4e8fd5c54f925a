#!/bin/bash
# fir_stream (loader/consumer) bring-up: parity subset, then A/B against fir_tile.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_fs
mkdir -p "$OUT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
   -k "frontend or fir_decim or block_size or full_size" > "$OUT/pytest.log" 2>&1
rc=$?; tail -15 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
b() {  # label, env...
  local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 30 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r"; return $rc
}
for rep in 1 2; do
  b "stream nt" X=1 || exit 1
  b "stream plain" SDR_FIR_STREAM_NT=0 || exit 1
  b "tile" SDR_FIR_STREAM=0 || exit 1
done
CFG=cfg4 b "cfg4 stream" X=1 || exit 1
CFG=cfg4 b "cfg4 tile" SDR_FIR_STREAM=0 || exit 1
exit 0
