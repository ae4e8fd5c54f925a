#!/bin/bash
# r05f: bench with the timed window in one graph replay (cfg5h's short steps),
# stereo configs with 100-step pipelined graphs, the rank path's stdout (one
# JSON line), and mono0 / stereo0 kernel traces.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05f; mkdir -p $OUT
for c in cfg5h cfg5h cfg2 stereo0 mono0; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 3 --no-cpu-baseline >> $OUT/bench_100.jsonl 2>>$OUT/bench.err || exit 1
done
for c in cfg5h cfg2; do
  timeout -k 10 300 python bench.py --config $c --steps 20 --warmup 3 --no-cpu-baseline >> $OUT/bench_20.jsonl 2>>$OUT/bench.err || exit 1
done
python3 -c "
import json
for f in ('$OUT/bench_100.jsonl', '$OUT/bench_20.jsonl'):
    for l in open(f):
        d = json.loads(l); print(f.split('/')[-1], d['config']['workload'][:40], d['ms_per_step'], d['roofline']['frac'], d['sustained']['ms_per_step'], d['config']['launch'])
"
SDR_BENCH_DEVICES=0,0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29521 bench.py --gpus 2 --steps 20 --warmup 3 > $OUT/bench_ranks2.out 2> $OUT/ranks.err || exit 1
wc -l $OUT/bench_ranks2.out; python3 -c "import json; d=json.loads(open('$OUT/bench_ranks2.out').read()); print('ranks ok', d['value'], d['n_gpus'])" || exit 1
TAG=r05f CFGS="mono0 stereo0" bash scripts/prof_cfg.sh || exit 1
find $OUT -name '*kernel_trace.csv' -delete
exit 0
