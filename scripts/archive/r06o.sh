#!/bin/bash
# r06o: closing record, part 2 -- rocprof timed-region summaries, PMC HBM
# traffic for every single-kernel config and mono0, SQ counters of the two
# kernels the verdict names (cfg3 resample_lp, cfg2u8 fir_tile_sc), and the
# rank path rehearsed (two torchrun ranks on GPU 0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
T=${TAG:-r06o}; OUT=gpurun_out/$T; mkdir -p $OUT
TAG=$T CFGS="cfg2 cfg2u8 cfg3 cfg5 cfg5b cfg5h cfg5hb mono0 stereo0" bash scripts/prof_cfg.sh || exit 1
TAG=$T CFGS="cfg2 cfg2u8 cfg3 cfg4 cfg4x8 cfg5 cfg5b cfg5h cfg5hb mono0" bash scripts/pmc_cfg.sh || exit 1
TAG=$T/sq_cfg3 CFG=cfg3 KERNEL=resample_lp bash scripts/pmc_sq.sh || exit 1
TAG=$T/sq_cfg2u8 CFG=cfg2u8 KERNEL=fir_tile_sc bash scripts/pmc_sq.sh || exit 1
SDR_BENCH_DEVICES=0,0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29523 bench.py --gpus 2 --steps 50 --warmup 3 > $OUT/bench_ranks2.json 2> $OUT/ranks.err || exit 1
cat $OUT/bench_ranks2.json
find $OUT -name '*kernel_trace.csv' -delete
find $OUT -name 'p[0-9]*' -type d -prune -exec rm -rf {} +
exit 0
