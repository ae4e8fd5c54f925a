#!/bin/bash
# r05ao: SQ counter record of the final tree's kernels (one pass per group,
# --pmc only): cfg2u8 and mono0's fir_tile_sc<..., U8>, cfg5h's
# fir_long_mfma (+ SQ_VALU_MFMA_BUSY_CYCLES).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r05ao/cfg2u8 CFG=cfg2u8 KERNEL=fir_tile_sc bash scripts/pmc_sq.sh || exit 1
TAG=r05ao/mono0 CFG=mono0 KERNEL=fir_tile_sc bash scripts/pmc_sq.sh || exit 1
GROUPS_OVERRIDE="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA
SQ_VALU_MFMA_BUSY_CYCLES
GRBM_GUI_ACTIVE GRBM_COUNT" TAG=r05ao/cfg5h CFG=cfg5h KERNEL=fir_long_mfma bash scripts/pmc_sq.sh || exit 1
find gpurun_out/r05ao -mindepth 2 -maxdepth 2 -type d -name 'p*' -exec rm -rf {} +
exit 0
