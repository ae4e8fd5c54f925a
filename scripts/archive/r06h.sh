#!/bin/bash
# r06h: old OCML PLL vs libm_exact (out-of-line chunk re-run): stereo0 with and without the forked side branch,
# stereo0w; two rounds
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06h; mkdir -p $OUT
for r in 1 2; do
  for lib in old_stereo new_chunk; do
    for fork in -1 0; do
      SDR_STEREO_FORK=$fork SDRHIP_LIB=$PWD/ab/$lib.so timeout -k 10 300 python bench.py --config stereo0 --steps 50 --warmup 3 \
        --no-cpu-baseline --sustain-seconds 1 --stereo-pipeline 0 > $OUT/b_${lib}_f${fork}_$r.json 2>>$OUT/bench.err || exit 1
      python3 -c "import json;d=json.load(open('$OUT/b_${lib}_f${fork}_$r.json'));print('$r $lib fork=$fork stereo0 pipe0', d['ms_per_step'], d.get('sustained',{}).get('ms_per_step'))"
    done
    SDRHIP_LIB=$PWD/ab/$lib.so timeout -k 10 300 python bench.py --config stereo0 --steps 50 --warmup 3 \
        --no-cpu-baseline --sustain-seconds 1 > $OUT/b_${lib}_pipe_$r.json 2>>$OUT/bench.err || exit 1
    python3 -c "import json;d=json.load(open('$OUT/b_${lib}_pipe_$r.json'));print('$r $lib stereo0 pipe1', d['ms_per_step'], d.get('sustained',{}).get('ms_per_step'))"
    SDRHIP_LIB=$PWD/ab/$lib.so timeout -k 10 300 python bench.py --config stereo0w --steps 30 --warmup 3 \
        --no-cpu-baseline --sustain-seconds 1 > $OUT/b_${lib}_w_$r.json 2>>$OUT/bench.err || exit 1
    python3 -c "import json;d=json.load(open('$OUT/b_${lib}_w_$r.json'));print('$r $lib stereo0w', d['ms_per_step'], d.get('sustained',{}).get('ms_per_step'))"
  done
done
