#!/bin/bash
# Same-box A/B over library builds and env settings:
#   ARMS="tree:SDR_FIR_IQ=1 tree:SDR_FIR_IQ=0 ab/pf2.so:SDR_FIR_IQ=1" CFGS="cfg2" REPS=3 bash scripts/ab_libs.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in $(seq ${REPS:-3}); do
  for cfg in ${CFGS:-cfg2}; do
    for arm in ${ARMS}; do
      l=${arm%%:*}; envs=${arm#*:}; [ "$envs" = "$arm" ] && envs=""
      if [ "$l" = tree ]; then unset SDRHIP_LIB; else export SDRHIP_LIB=$PWD/$l; fi
      r=$(env ${envs//,/ } timeout -k 10 120 python bench.py --config $cfg --steps ${STEPS:-100} --warmup 3 --no-cpu-baseline 2>>gpurun_out/ab_libs.err |
          python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'], (d.get('fma_variant') or {}).get('ms_per_step'), (d.get('sustained') or {}).get('frac'))")
      rc=$?; echo "rep $rep $cfg $arm: $r"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
