set -u
OUT=gpurun_out/${TAG:-final1}; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread > $OUT/pytest_gpu.log 2>&1; rc=$?; tail -2 $OUT/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1 || exit 1; tail -1 $OUT/smoke.log
timeout -k 10 300 python bench.py > $OUT/bench_default.json 2>$OUT/bench.err || exit 1
for c in cfg2u8 cfg3 cfg4 cfg4x8 cfg5 cfg5h mono0 stereo0 stereo0w; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 3 --no-cpu-baseline > $OUT/bench_$c.json 2>>$OUT/bench.err || exit 1
done
SDR_BENCH_DEVICES=0,0 timeout -k 10 300 python bench.py --gpus 2 --steps 50 --warmup 3 --no-cpu-baseline > $OUT/bench_rehearse2.json 2>>$OUT/bench.err || exit 1
for f in $OUT/bench_*.json; do python3 -c "import json,sys;d=json.load(open('$f'));print('$f'.split('/')[-1], d['value'], d['ms_per_step'], d['roofline'].get('frac'))"; done
