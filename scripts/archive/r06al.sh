#!/bin/bash
# r06al: the rank path rehearsed at the driver's larger N on one GPU: 4 and 8 torchrun
# ranks all on GPU 0 (SDR_BENCH_DEVICES), one clean JSON line each (this rehearses the code
# path -- launch, gloo barrier, max over ranks, aggregation -- not the scaling)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
OUT=gpurun_out/r06al; mkdir -p $OUT
for n in 4 8; do
  devs=$(python3 -c "print(','.join(['0']*$n))")
  SDR_BENCH_DEVICES=$devs timeout -k 10 400 python -m torch.distributed.run --nnodes=1 --nproc-per-node $n \
    --master-addr 127.0.0.1 --master-port 2953$n bench.py --gpus $n --steps 20 --warmup 3 \
    > $OUT/bench_ranks$n.json 2> $OUT/ranks$n.err || { tail -20 $OUT/ranks$n.err; exit 1; }
  python3 -c "import json;d=json.load(open('$OUT/bench_ranks$n.json'));print($n, d['n_gpus'], d['value'], d['ms_per_step'], d['config']['devices_opened'], len(d['per_gpu']['value']))"
done
exit 0
