#!/bin/bash
# stereo with 16k streams per step (stereo0w) vs 1k (stereo0), warm.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_stw; mkdir -p "$OUT"
for c in stereo0 stereo0w; do
  timeout -k 10 240 python bench.py --config $c --steps 10 --warmup 2 --no-cpu-baseline > "$OUT/$c.json" 2>>"$OUT/err.log" || exit 1
  python -c "import json;d=json.load(open('$OUT/$c.json'));print('$c', d['ms_per_step'], d['value'], d['roofline']['frac'])"
done
export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/prof" -o bench \
  -- python3 bench.py --config stereo0w --steps 5 --warmup 1 --no-cpu-baseline > "$OUT/prof.json" 2>>"$OUT/err.log"
echo "rocprof rc=$?"
