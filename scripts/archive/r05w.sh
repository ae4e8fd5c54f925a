#!/bin/bash
# r05w: the round's closing record on one box -- the whole GPU suite and
# smoke, every bench config with its CPU baseline, rocprof timed-region
# summaries (cfg2, cfg2u8, cfg3, cfg5h, mono0), PMC HBM traffic (cfg2,
# cfg2u8, cfg3, cfg5h), the rank path rehearsed (two torchrun ranks on GPU 0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05w; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 120 --timeout-method thread \
  > $OUT/pytest_gpu.log 2>&1; rc=$?
tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_gpu.log | head; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1; rc=$?
tail -2 $OUT/smoke.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python bench.py > $OUT/bench_cfg2.json 2> $OUT/bench.err || exit 1
for c in cfg2u8 cfg3 cfg4 cfg4x8 cfg5 cfg5h mono0 stereo0 stereo0w; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 3 > $OUT/bench_$c.json 2>>$OUT/bench.err || exit 1
done
for f in $OUT/bench_*.json; do python3 -c "import json;d=json.load(open('$f'));c=d['cpu_baseline'] or {};print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['roofline']['frac'], d.get('sustained',{}).get('ms_per_step'), c.get('value'), c.get('kind'))"; done
TAG=r05w CFGS="cfg2 cfg2u8 cfg3 cfg5h mono0" bash scripts/prof_cfg.sh || exit 1
export TMPDIR=/tmp
for cfg in cfg2 cfg2u8 cfg3 cfg5h; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/pmc_${cfg}_$ctr" -o pmc \
      -- python3 bench.py --config $cfg --steps 3 --warmup 1 --warm-seconds 0 --no-cpu-baseline --no-fma-variant --no-graph --sustain-seconds 0 \
      > /dev/null 2>> "$OUT/prof.err"
    rc=$?; echo "pmc $cfg $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  k=fir_tile_sc; [ $cfg = cfg3 ] && k=resample_lp; [ $cfg = cfg5h ] && k=fir_long_mfma
  python scripts/pmc_traffic.py "$(find $OUT/pmc_${cfg}_FETCH_SIZE -name '*counter_collection.csv' | head -1)" \
    "$(find $OUT/pmc_${cfg}_WRITE_SIZE -name '*counter_collection.csv' | head -1)" $k "$OUT/traffic_$cfg.json" || exit 1
done
SDR_BENCH_DEVICES=0,0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29523 bench.py --gpus 2 --steps 50 --warmup 3 > $OUT/bench_ranks2.json 2> $OUT/ranks.err || exit 1
find $OUT -name '*kernel_trace.csv' -delete
find $OUT -name 'pmc_*' -type d -prune -exec rm -rf {} +
exit 0
