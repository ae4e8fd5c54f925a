#!/bin/bash
# Timeline traces of fir_tile (diagnostic build ab/trace.so) under several
# launch shapes: TAG=... bash scripts/trace_fir.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
. scripts/timing_lib.sh  # SDR_ABLATE etc. need the timing build
OUT=gpurun_out/${TAG:-trace}
mkdir -p "$OUT"
export SDRHIP_LIB=$PWD/ab/trace.so SDR_FIR_IQ=0
for arm in ${ARMS:-default SDR_WG_PER_CU=14 SDR_WG_PER_CU=3 SDR_ABLATE=2}; do
  e=""; [ "$arm" = default ] || e="$arm"
  env $e timeout -k 10 120 python tools/fir_trace.py > "$OUT/$arm.json" 2>> "$OUT/err.log"
  rc=$?; echo "$arm rc=$rc"; [ $rc -eq 0 ] || exit $rc
done
