#!/bin/bash
# r06c: same-box A/B of the PLL / NCO transcendental routines: OCML (the round-5 stereo.hip), libm_exact
# inlined, libm_exact with out-of-line double-double paths -- stereo0 and stereo0w, two rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06c; mkdir -p $OUT
for r in 1 2; do
  for lib in old_stereo new_inline new_noinline; do
    for c in stereo0 stereo0w; do
      SDRHIP_LIB=$PWD/ab/$lib.so timeout -k 10 300 python bench.py --config $c --steps 50 --warmup 3 --no-cpu-baseline \
        --sustain-seconds 1 > $OUT/b_${lib}_${c}_$r.json 2>>$OUT/bench.err || exit 1
      python3 -c "import json;d=json.load(open('$OUT/b_${lib}_${c}_$r.json'));print('$r $lib $c', d['ms_per_step'], d.get('sustained',{}).get('ms_per_step'))"
    done
  done
done
