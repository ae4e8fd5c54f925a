#!/bin/bash
# Where does the fused front-end kernel spend its time?  SDR_ABLATE=1 drops
# the global loads, =2 the FIR math, =3 the output stores, =4 two of the
# three tap passes (timings only; outputs garbage).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
. scripts/timing_lib.sh  # SDR_ABLATE etc. need the timing build
for ab in ${ABLATIONS:-0 1 2 3 4}; do
  for cfg in ${CFGS:-cfg2 cfg2u8}; do
    r=$(SDR_ABLATE=$ab timeout -k 10 300 python bench.py --config $cfg --steps 50 --warmup 5 --no-cpu-baseline \
        --no-fma-variant 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")
    rc=$?; echo "ablate $ab $cfg: $r ms"; [ $rc -eq 0 ] || exit $rc
  done
done
