#!/bin/bash
# r05b: resampler software-pipelined scan (ab/pipe.so) parity + same-box A/B;
# cfg2u8 / cfg3 kernel traces, cfg2u8 HBM traffic and SQ counters of
# fir_tile_sc<U8> (VERDICT r4 missing 3); the rank path rehearsed on one GPU
# (two torchrun ranks, SDR_BENCH_DEVICES=0,0).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05b; mkdir -p $OUT
for l in pipe split pipesplit; do
  SDRHIP_LIB=$PWD/ab/$l.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
    -p no:cacheprovider --timeout 120 --timeout-method thread -k "resample or cfg3" > $OUT/pytest_$l.log 2>&1; rc=$?
  tail -1 $OUT/pytest_$l.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_$l.log | head; exit $rc; }
done
ARMS="tree ab/pipe.so ab/split.so ab/pipesplit.so" CFGS="cfg3" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_pipe.txt 2>&1; rc=$?; cat $OUT/ab_pipe.txt; [ $rc -eq 0 ] || exit $rc
SDRHIP_LIB=$PWD/ab/pk.so timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread -k "u8 or odd_shapes or batched" > $OUT/pytest_pk.log 2>&1; rc=$?
tail -2 $OUT/pytest_pk.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_pk.log | head; exit $rc; }
ARMS="tree ab/pk.so" CFGS="cfg2u8 mono0" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_pk.txt 2>&1; rc=$?; cat $OUT/ab_pk.txt; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16 or cfg5" > $OUT/pytest_f16plan.log 2>&1; rc=$?
tail -2 $OUT/pytest_f16plan.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_f16plan.log | head; exit $rc; }
ARMS="tree:SDR_BENCH_F16_PLAN=1 tree:SDR_BENCH_F16_PLAN=0" CFGS="cfg5h" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_f16plan.txt 2>&1; rc=$?
cat $OUT/ab_f16plan.txt; [ $rc -eq 0 ] || exit $rc
TAG=r05b CFGS="cfg2u8 cfg3 cfg5h" bash scripts/prof_cfg.sh || exit 1
export TMPDIR=/tmp
for ctr in FETCH_SIZE WRITE_SIZE; do
  timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/pmc_cfg2u8_$ctr" -o pmc \
    -- python3 bench.py --config cfg2u8 --steps 3 --warmup 1 --warm-seconds 0 --no-cpu-baseline --no-fma-variant --no-graph --sustain-seconds 0 \
    > /dev/null 2>> "$OUT/prof.err"
  rc=$?; echo "pmc cfg2u8 $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
python scripts/pmc_traffic.py "$(find $OUT/pmc_cfg2u8_FETCH_SIZE -name '*counter_collection.csv' | head -1)" \
  "$(find $OUT/pmc_cfg2u8_WRITE_SIZE -name '*counter_collection.csv' | head -1)" fir_tile_sc "$OUT/traffic_cfg2u8.json" || exit 1
TAG=r05b/sq_cfg2u8 CFG=cfg2u8 KERNEL=fir_tile_sc bash scripts/pmc_sq.sh || exit 1
SDR_BENCH_DEVICES=0,0 timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 \
  --master-port 29517 bench.py --gpus 2 --steps 50 --warmup 3 > $OUT/bench_ranks2.json 2> $OUT/ranks.err; rc=$?
tail -3 $OUT/ranks.err; cat $OUT/bench_ranks2.json; [ $rc -eq 0 ] || exit $rc
find $OUT -name '*kernel_trace.csv' -delete
exit 0
