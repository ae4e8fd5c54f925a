#!/bin/bash
# r04v: cfg5h anatomy -- kernel trace of fir_long_mfma under each timing ablation
# (SDR_ABLATE 0 full, 1 one cached input chunk, 2 no MFMA, 3 no tap staging, 4 no output stores)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out/r04v; mkdir -p $OUT
for ab in 0 1 2 3 4; do
  SDR_ABLATE=$ab timeout -k 10 120 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/ab$ab" -o k \
    -- python3 bench.py --config cfg5h --steps 100 --warmup 3 --no-cpu-baseline --no-fma-variant --sustain-seconds 0 \
    > $OUT/bench_ab$ab.json 2>>$OUT/err.log || exit 1
  f=$(find $OUT/ab$ab -name '*kernel_stats.csv' | head -1)
  echo "ablate $ab: step $(python3 -c "import json;print(json.load(open('$OUT/bench_ab$ab.json'))['ms_per_step'])") ms; $(grep fir_long_mfma $f | cut -d, -f1-5)"
done
