#!/bin/bash
# resample_lp A/B on one box: chains per lane (SDR_LP_K) x LDS prefetch depth (ab/pd2.so)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in 1 2; do
  for v in "tree:7" "tree:4" "ab/pd2.so:4"; do
    l=${v%%:*}; k=${v#*:}
    if [ "$l" = tree ]; then unset SDRHIP_LIB; else export SDRHIP_LIB=$PWD/$l; fi
    r=$(SDR_LP_K=$k timeout -k 10 120 python bench.py --config cfg3 --steps 100 --warmup 3 --no-cpu-baseline 2>/dev/null |
        python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'])")
    rc=$?; echo "rep $rep $l K=$k: $r"; [ $rc -eq 0 ] || exit $rc
  done
done
