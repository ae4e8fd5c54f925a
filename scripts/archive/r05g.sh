#!/bin/bash
# r05g: fir_long_mfma phase anatomy (timing build, wall-clock stamps) and SQ
# counters of cfg5h's kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05g; mkdir -p $OUT
SDRHIP_LIB=$PWD/ab/timing.so SDR_F16_TRACE=1 timeout -k 10 200 python -u scripts/f16_trace.py > $OUT/f16_trace.txt 2>&1; rc=$?
cat $OUT/f16_trace.txt; [ $rc -eq 0 ] || exit $rc
GROUPS_OVERRIDE="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_INSTS_VMEM_RD SQ_INSTS_VMEM_WR
GRBM_GUI_ACTIVE GRBM_COUNT
SQ_VALU_MFMA_BUSY_CYCLES SQ_INSTS_VALU_MFMA_MOPS_F16" TAG=r05g/sq_cfg5h CFG=cfg5h KERNEL=fir_long_mfma bash scripts/pmc_sq.sh || exit 1
exit 0
