#!/bin/bash
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_fs; mkdir -p "$OUT"
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 30 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
  rc=$?; echo "$label: $r"; return $rc; }
for a in 0 1 2 3 4; do b "stream ablate=$a" SDR_ABLATE=$a || exit 1; done
for a in 0 1 2; do b "tile ablate=$a" SDR_ABLATE=$a SDR_FIR_STREAM=0 || exit 1; done
exit 0
