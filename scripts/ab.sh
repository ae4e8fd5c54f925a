#!/bin/bash
# Same-box A/B: alternate the in-tree library with ab/*.so builds.
#   LIBS="ab/prev.so" CFGS="cfg2 cfg4" REPS=2 bash scripts/ab.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in $(seq ${REPS:-2}); do
  for cfg in ${CFGS:-cfg2}; do
    for l in tree ${LIBS:-}; do
      if [ "$l" = tree ]; then unset SDRHIP_LIB; else export SDRHIP_LIB=$PWD/$l; fi
      r=$(timeout -k 10 120 python bench.py --config $cfg --steps ${STEPS:-50} --warmup 5 --no-cpu-baseline 2>/dev/null |
          python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['value'], d['roofline']['frac'])")
      rc=$?; echo "rep $rep $cfg $l: $r"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
