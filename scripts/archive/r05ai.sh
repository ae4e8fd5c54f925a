#!/bin/bash
# r05ai: PMC HBM traffic (FETCH_SIZE / WRITE_SIZE, one counter per pass) for
# the configs whose bench lines still carried "traffic": null -- cfg4,
# cfg4x8 (fir_tile_sc), cfg5 (fir_long exact), mono0 (both kernels of a step:
# the u8 front end and the audio FIR, summed).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/r05ai; mkdir -p $OUT
export TMPDIR=/tmp
for cfg in cfg4 cfg4x8 cfg5 mono0; do
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/pmc_${cfg}_$ctr" -o pmc \
      -- python3 bench.py --config $cfg --steps 3 --warmup 1 --warm-seconds 0 --no-cpu-baseline --no-fma-variant --no-graph --sustain-seconds 0 \
      > /dev/null 2>> "$OUT/prof.err"
    rc=$?; echo "pmc $cfg $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  F="$(find $OUT/pmc_${cfg}_FETCH_SIZE -name '*counter_collection.csv' | head -1)"
  W="$(find $OUT/pmc_${cfg}_WRITE_SIZE -name '*counter_collection.csv' | head -1)"
  case $cfg in
    cfg5) ks="fir_long<" ;;
    mono0) ks="fir_tile_sc fir_tile_grp" ;;
    *) ks="fir_tile_sc" ;;
  esac
  parts=""
  for k in $ks; do
    python scripts/pmc_traffic.py "$F" "$W" "$k" "$OUT/traffic_${cfg}_$k.json" || exit 1
    parts="$parts $OUT/traffic_${cfg}_$k.json"
  done
  python3 - "$OUT/traffic_$cfg.json" $parts <<'PY' || exit 1
import json, sys
out, parts = sys.argv[1], sys.argv[2:]
ds = [json.load(open(p)) for p in parts]
res = {"kernel": " + ".join(d["kernel"] for d in ds), "parts": ds,
       "read_bytes_per_launch": sum(d["read_bytes_per_launch"] for d in ds),
       "write_bytes_per_launch": sum(d["write_bytes_per_launch"] for d in ds),
       "hbm_bytes_per_launch": sum(d["hbm_bytes_per_launch"] for d in ds),
       "correction": ds[0]["correction"] + ("; per step = the sum over the step's kernels" if len(ds) > 1 else "")}
json.dump(res, open(out, "w"), indent=1)
print(out, res["hbm_bytes_per_launch"])
PY
done
find $OUT -name 'pmc_*' -type d -prune -exec rm -rf {} +
exit 0
