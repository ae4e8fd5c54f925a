#!/bin/bash
# Same-box A/B over (library, env) arms:  ARMS="tree ab/prev.so tree:A=1,B=2" CFGS=cfg2 REPS=2
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in $(seq ${REPS:-2}); do
  for cfg in ${CFGS:-cfg2}; do
    for arm in ${ARMS}; do
      l=${arm%%:*}; e=""; [ "$l" != "$arm" ] && e="${arm#*:}"
      if [ "$l" = tree ]; then unset SDRHIP_LIB; else export SDRHIP_LIB=$PWD/$l; fi
      r=$(env ${e//,/ } timeout -k 10 120 python bench.py --config $cfg --steps ${STEPS:-100} --warmup 3 --no-cpu-baseline --no-fma-variant 2>>gpurun_out/ab_mix.err |
          python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'])")
      rc=$?; echo "rep $rep $cfg $arm: $r"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
