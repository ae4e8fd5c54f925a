#!/bin/bash
# r06d: per-kernel times of stereo0 under the three PLL/NCO builds (rocprofv3 kernel trace)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/${TAG:-r06d}; mkdir -p $OUT
export TMPDIR=/tmp
for lib in ${LIBS:-old_stereo new_inline new_value}; do
  SDRHIP_LIB=$PWD/ab/$lib.so timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/p_$lib" -o b \
    -- python3 bench.py --config stereo0 --steps 20 --warmup 3 --no-cpu-baseline --sustain-seconds 0 --no-graph \
    > $OUT/b_$lib.json 2>> $OUT/prof.err || exit 1
  f=$(find $OUT/p_$lib -name '*kernel_stats.csv' | head -1)
  echo "== $lib"; python3 -c "
import csv
rows=list(csv.DictReader(open('$f')))
for r in sorted(rows, key=lambda r:-float(r['TotalDurationNs']))[:8]: print(r['Name'][:80], r['Calls'], round(float(r['AverageNs'])/1e3,1))
"
done
find $OUT -name '*kernel_trace.csv' -delete
