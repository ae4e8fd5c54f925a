#!/bin/bash
# r06y: where mono0's audio FIR (fir_tile_grp, D = 5) spends its 12 us: timing-build ablations
# (0 full, 1 no global loads, 2 no FIR math, 9 no tile-0 extras; wrong outputs), kernel trace each
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06y; mkdir -p $OUT
export TMPDIR=/tmp
export SDRHIP_LIB="$PWD/3dy4-real-time-software-defined-radio-_amd/libsdrhip_timing.so"
for a in 0 1 2 9; do
  SDR_ABLATE=$a timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$PWD/$OUT/p$a" -o b \
    -- python3 bench.py --config mono0 --steps 100 --warmup 5 --no-cpu-baseline --sustain-seconds 0 \
    > $OUT/b$a.json 2>> $OUT/prof.err || exit 1
  python3 scripts/prof_timed.py "$(find $OUT/p$a -name '*kernel_trace.csv' | head -1)" 100 $OUT/t$a.json $OUT/b$a.json > /dev/null || exit 1
  python3 -c "
import json; d=json.load(open('$OUT/t$a.json'))
print('ablate $a', [(k['kernel'].split('<')[0].split('::')[-1], k.get('avg_us_timed')) for k in d['kernels'][:2]])"
done
find $OUT -name '*kernel_trace.csv' -delete
exit 0
