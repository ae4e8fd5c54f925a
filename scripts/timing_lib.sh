# Sourced by the timing-experiment scripts (ablate.sh, ablate_cfg3.sh,
# clock_probe.sh, diag_iq.sh, trace_fir.sh): SDR_ABLATE, the shape overrides
# and the phase traces exist only in a timing build (make TIMING=1 ->
# libsdrhip_timing.so, objects in build-timing/), never in the shipped
# libsdrhip.so, which ignores them.  Builds that library if SDRHIP_LIB is
# unset and points sdrhip (bench.py, the tests) at it; refuses anything else.
PKG_DIR="$(pwd)/3dy4-real-time-software-defined-radio-_amd"
if [ -z "${SDRHIP_LIB:-}" ]; then
  make -s -C "$PKG_DIR" TIMING=1 -j16 > /dev/null || { echo "timing build failed" >&2; exit 1; }
  export SDRHIP_LIB="$PKG_DIR/libsdrhip_timing.so"
fi
case "$SDRHIP_LIB" in
  *timing*) ;;
  *) echo "SDRHIP_LIB=$SDRHIP_LIB is not a timing build (make TIMING=1): SDR_ABLATE would do nothing" >&2; exit 2 ;;
esac
