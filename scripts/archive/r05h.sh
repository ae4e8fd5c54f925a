#!/bin/bash
# r05h: fp16 MFMA A reads conflict-free (row permutation + copy stride 32 mod
# 128 halves): f16 parity, same-box A/B against the previous tree, phase trace
# and LDS counters; u8 ragged-row buffer load with a uniform row offset.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05h; mkdir -p $OUT
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q \
  -p no:cacheprovider --timeout 120 --timeout-method thread -k "f16 or cfg5 or u8 or frontend or cfg2" > $OUT/pytest_f16.log 2>&1; rc=$?
tail -1 $OUT/pytest_f16.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" $OUT/pytest_f16.log | head; exit $rc; }
ARMS="tree ab/f16old.so" CFGS="cfg5h cfg2u8" REPS=3 bash scripts/ab_libs.sh > $OUT/ab_f16lds.txt 2>&1; rc=$?; cat $OUT/ab_f16lds.txt; [ $rc -eq 0 ] || exit $rc
SDRHIP_LIB=$PWD/ab/timing.so SDR_F16_TRACE=1 REPS=2 timeout -k 10 200 python -u scripts/f16_trace.py > $OUT/f16_trace.txt 2>&1; rc=$?
cat $OUT/f16_trace.txt; [ $rc -eq 0 ] || exit $rc
GROUPS_OVERRIDE="SQ_INSTS_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY
SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16" TAG=r05h/sq_cfg5h CFG=cfg5h KERNEL=fir_long_mfma bash scripts/pmc_sq.sh || exit 1
TAG=r05h CFGS="cfg5h" bash scripts/prof_cfg.sh || exit 1
find $OUT -name '*kernel_trace.csv' -delete
exit 0
