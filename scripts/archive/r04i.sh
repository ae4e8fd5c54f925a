#!/bin/bash
# r04i: is the u8 front end clock (power) limited?  rocm-smi clocks during long
# cfg2u8 runs per mode, then SQ counters + GRBM of fir_tile_sc<U8>.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r04i_clk CFG=cfg2u8 STEPS=50000 SETTLE=6 bash scripts/clock_probe.sh || exit 1
GROUPS_OVERRIDE="GRBM_GUI_ACTIVE GRBM_COUNT SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_ACTIVE_INST_VALU
SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_LDS SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAVES" \
  TAG=r04i_pmc CFG=cfg2u8 KERNEL=fir_tile_sc bash scripts/pmc_sq.sh || exit 1
