#!/bin/bash
# Same-box sweep of one environment switch over bench configs:
#   VAR=SDR_WG_PER_CU VALUES="14 28 64" CFGS="cfg2" REPS=2 bash scripts/sweep.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in $(seq ${REPS:-2}); do
  for cfg in ${CFGS:-cfg2}; do
    for v in ${VALUES}; do
      r=$(env $VAR=$v timeout -k 10 120 python bench.py --config $cfg --steps ${STEPS:-100} --warmup 5 --no-cpu-baseline \
          --no-fma-variant 2>/dev/null | python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
      rc=$?; echo "rep $rep $cfg $VAR=$v: $r"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
