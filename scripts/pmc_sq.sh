#!/bin/bash
# SQ/LDS counter passes for one kernel of one bench config (one pass per
# group, no tracing domains beside --pmc; <= 8 SQ counters per pass).
#   TAG=pmc CFG=cfg2 KERNEL=fir_tile [SDR_ABLATE=1] bash scripts/pmc_sq.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc}
mkdir -p "$OUT"
export TMPDIR=/tmp
CFG=${CFG:-cfg2}
i=0
while IFS= read -r grp; do
  [ -z "$grp" ] && continue
  i=$((i+1))
  timeout -s KILL 120 rocprofv3 --pmc $grp --output-format csv -d "$PWD/$OUT/p$i" -o pmc \
     -- python3 bench.py --config $CFG --steps 3 --warmup 1 --warm-seconds 0 --no-cpu-baseline --no-fma-variant --sustain-seconds 0 \
        --no-graph > /dev/null 2>> "$OUT/err.log"
  rc=$?; echo "pass $i ($grp) rc=$rc"; [ $rc -eq 0 ] || exit $rc
done <<GROUPS
${GROUPS_OVERRIDE:-SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_ACTIVE_INST_LDS
SQ_INSTS_VALU SQ_INSTS_LDS SQ_INSTS_SALU SQ_INSTS_SMEM SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_WAIT_INST_LDS SQ_ACTIVE_INST_SCA
GRBM_GUI_ACTIVE GRBM_COUNT}
GROUPS
python3 scripts/pmc_summary.py "$OUT" ${KERNEL:-fir_tile} | tee "$OUT/summary.txt"
