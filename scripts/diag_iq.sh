#!/bin/bash
# fir_tile_iq vs fir_tile: ablations (no loads / no math / one tap pass) and
# SQ counters of each, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
. scripts/timing_lib.sh  # SDR_ABLATE etc. need the timing build
OUT=gpurun_out/${TAG:-diag_iq}
mkdir -p "$OUT"
for v in 1 0; do
  for ab in ${ABLATIONS:-0 1 2 4}; do
    r=$(SDR_FIR_IQ=$v SDR_ABLATE=$ab timeout -k 10 120 python bench.py --config cfg2 --steps 50 --warmup 3 \
        --no-cpu-baseline --no-fma-variant 2>>"$OUT/bench.err" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")
    rc=$?; echo "SDR_FIR_IQ=$v ablate $ab: $r ms"; [ $rc -eq 0 ] || exit $rc
  done
done
for v in 1 0; do
  SDR_FIR_IQ=$v TAG=${TAG:-diag_iq}/pmc_iq$v CFG=cfg2 KERNEL=fir_tile bash scripts/pmc_sq.sh || exit $?
done
