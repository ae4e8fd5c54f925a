#!/bin/bash
# PMC HBM traffic of bench configs: FETCH_SIZE and WRITE_SIZE, one counter
# per pass (MI355X_MICROARCH.md's HBM section), summed over the kernels of one
# step, written as $OUT/traffic_<cfg>.json (the shape bench.py reads from
# profiles/traffic_<cfg>.json).
#   TAG=r06o CFGS="cfg2 cfg3 mono0" bash scripts/pmc_cfg.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-pmc}; mkdir -p "$OUT"
export TMPDIR=/tmp
for cfg in ${CFGS:-cfg2}; do
  case $cfg in
    cfg3) ks="resample_lp" ;;
    cfg5|cfg5b) ks="fir_long<" ;;
    cfg5h|cfg5hb) ks="fir_long_mfma" ;;
    mono0) ks="fir_tile_sc fir_tile_grp" ;;
    cfg2|cfg2u8|cfg4|cfg4x8) ks="fir_tile_sc" ;;
    *) echo "no kernel list for $cfg"; exit 1 ;;
  esac
  # the fp16 error sweep (setup) launches the same kernel at other shapes: keep it out of the average
  extra=""; case $cfg in cfg5h|cfg5hb) extra="--no-f16-sweep" ;; esac
  for ctr in FETCH_SIZE WRITE_SIZE; do
    timeout -k 10 300 rocprofv3 --pmc $ctr --output-format csv -d "$PWD/$OUT/pmc_${cfg}_$ctr" -o pmc \
      -- python3 bench.py --config $cfg --steps 3 --warmup 1 --warm-seconds 0 --no-cpu-baseline --no-fma-variant --no-graph --sustain-seconds 0 $extra \
      > /dev/null 2>> "$OUT/pmc.err"
    rc=$?; echo "pmc $cfg $ctr rc=$rc"; [ $rc -eq 0 ] || exit $rc
  done
  F="$(find $OUT/pmc_${cfg}_FETCH_SIZE -name '*counter_collection.csv' | head -1)"
  W="$(find $OUT/pmc_${cfg}_WRITE_SIZE -name '*counter_collection.csv' | head -1)"
  parts=""
  for k in $ks; do
    python3 scripts/pmc_traffic.py "$F" "$W" "$k" "$OUT/traffic_${cfg}_$k.json" > /dev/null || exit 1
    parts="$parts $OUT/traffic_${cfg}_$k.json"
  done
  python3 - "$OUT/traffic_$cfg.json" $parts <<'PY' || exit 1
import json, sys
out, parts = sys.argv[1], sys.argv[2:]
ds = [json.load(open(p)) for p in parts]
if len(ds) == 1:
    res = ds[0]
else:
    res = {"kernel": " + ".join(d["kernel"] for d in ds), "parts": ds,
           "read_bytes_per_launch": sum(d["read_bytes_per_launch"] for d in ds),
           "write_bytes_per_launch": sum(d["write_bytes_per_launch"] for d in ds),
           "hbm_bytes_per_launch": sum(d["hbm_bytes_per_launch"] for d in ds),
           "correction": ds[0]["correction"] + "; per step = the sum over the step's kernels"}
json.dump(res, open(out, "w"), indent=1)
print(out.split("/")[-1], res["hbm_bytes_per_launch"])
PY
  rm -f $parts
done
find $OUT -name 'pmc_*' -type d -prune -exec rm -rf {} +
exit 0
