#!/bin/bash
# cfg3: resample_lp vs resample_sp2, guide lane groups vs consecutive (ab/consec.so), bench arms + LDS counters
set -u
OUT=gpurun_out/r03_lds; mkdir -p $OUT
ARMS="tree:SDR_RESAMPLE_SP2=0 ab/consec.so:SDR_RESAMPLE_SP2=0 tree:SDR_RESAMPLE_SP2=1 ab/consec.so:SDR_RESAMPLE_SP2=1" CFGS=cfg3 REPS=2 bash scripts/sweep_lib_env.sh || exit 1
export TMPDIR=/tmp
for arm in "tree lp 0" "tree sp2 1" "consec lp 0"; do set -- $arm
  if [ $1 = tree ]; then unset SDRHIP_LIB; else export SDRHIP_LIB=$PWD/ab/$1.so; fi
  SDR_RESAMPLE_SP2=$3 timeout -s KILL 120 rocprofv3 --pmc SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE SQ_INSTS_LDS SQ_WAVES --output-format csv -d "$PWD/$OUT/pmc_$1_$2/p1" -o pmc -- python3 bench.py --config cfg3 --steps 3 --warmup 1 --warm-seconds 0 --no-cpu-baseline --no-fma-variant --no-graph > /dev/null 2>> $OUT/err.log || exit 1
  python3 scripts/pmc_summary.py "$OUT/pmc_$1_$2" resample > $OUT/summary_$1_$2.txt 2>&1; echo "== $arm"; cat $OUT/summary_$1_$2.txt | tail -8
done
