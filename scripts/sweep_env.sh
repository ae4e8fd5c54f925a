#!/bin/bash
# Same-box sweep of env settings on bench configs:
#   ARMS="A=1,B=2 A=0" CFGS="cfg2" REPS=2 bash scripts/sweep_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in $(seq ${REPS:-2}); do
  for cfg in ${CFGS:-cfg2}; do
    for arm in ${ARMS}; do
      e=""; [ "$arm" = default ] || e="${arm//,/ }"
      r=$(env $e timeout -k 10 120 python bench.py --config $cfg --steps ${STEPS:-100} --warmup 3 --no-cpu-baseline --no-fma-variant --sustain-seconds ${SUS:-0} 2>>gpurun_out/sweep.err |
          python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'])")
      rc=$?; echo "rep $rep $cfg $arm: $r"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
