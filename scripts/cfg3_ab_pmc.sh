#!/bin/bash
# cfg3 resampler session: parity (resampler cases + the bench-shape test),
# same-box A/B of the tree against ab/base.so, then per-kernel SQ/LDS
# counters for both (stall breakdown + bank conflicts).
#   TAG=r04b bash scripts/cfg3_ab_pmc.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-cfg3ab}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -m gpu -x -q -p no:cacheprovider \
  -rf --timeout 300 --timeout-method thread -k "${TESTK:-resample or cfg3}" > "$OUT/pytest.log" 2>&1
rc=$?; tail -3 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
ARMS="${ARMS:-tree:default ab/base.so:default}" CFGS=cfg3 REPS=${REPS:-2} bash scripts/sweep_lib_env.sh || exit 1
for arm in ${PMC_ARMS:-tree ab/base.so}; do
  if [ $arm = tree ]; then unset SDRHIP_LIB; else export SDRHIP_LIB=$PWD/$arm; fi
  name=$(basename $arm .so)
  TAG=${TAG:-cfg3ab}/pmc_$name CFG=cfg3 KERNEL=resample_lp GROUPS_OVERRIDE="SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_WAIT_INST_LDS SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_ACTIVE_INST_SCA GRBM_GUI_ACTIVE" \
    bash scripts/pmc_sq.sh || exit 1
done
