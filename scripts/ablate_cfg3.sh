#!/bin/bash
# cfg3 ablations of the default resampler kernel (timing only; outputs wrong)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
. scripts/timing_lib.sh  # SDR_ABLATE etc. need the timing build
OUT=gpurun_out/${TAG:-abl}
mkdir -p "$OUT"
for ab in ${ABL:-0 1 2}; do
  SDR_ABLATE=$ab timeout -k 10 300 python bench.py --config cfg3 --steps 100 --warmup 3 --no-cpu-baseline \
    > "$OUT/cfg3_ablate$ab.json" 2>> "$OUT/bench.err"
  rc=$?; python3 -c "import json;d=json.load(open('$OUT/cfg3_ablate$ab.json'));print('ablate $ab', d['ms_per_step'])"
  [ $rc -eq 0 ] || exit $rc
done
