#!/bin/bash
# Same-box sweep over (library, env) arms on bench configs:
#   ARMS="tree:A=1 ab/x.so:B=2,C=3 tree:default" CFGS="cfg3" REPS=2 bash scripts/sweep_lib_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for rep in $(seq ${REPS:-2}); do
  for cfg in ${CFGS:-cfg2}; do
    for arm in ${ARMS}; do
      lib=${arm%%:*}; envs=${arm#*:}
      e=""; [ "$envs" = default ] || e="${envs//,/ }"
      if [ "$lib" = tree ]; then unset SDRHIP_LIB; else export SDRHIP_LIB=$PWD/$lib; fi
      r=$(env $e timeout -k 10 120 python bench.py --config $cfg --steps ${STEPS:-100} --warmup 3 --no-cpu-baseline --no-fma-variant --sustain-seconds 0 2>>gpurun_out/sweep.err |
          python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'])")
      rc=$?; echo "rep $rep $cfg $arm: $r"; [ $rc -eq 0 ] || exit $rc
    done
  done
done
