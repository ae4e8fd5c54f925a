#!/bin/bash
# Parity + throughput of each front-end tile variant (R outputs/lane x waves/WG).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-sweep}
mkdir -p "$OUT"
for v in ${VARIANTS:-2x1 2x4 4x1 4x2}; do
  SDR_FIR_VARIANT=$v timeout -k 10 600 python -m pytest tests/test_gpu_parity.py -m gpu -q -p no:cacheprovider \
      -k "frontend or fir_decim or block_size" > "$OUT/pytest_$v.log" 2>&1
  rc=$?; echo "variant $v pytest rc=$rc: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -le 1 ] || exit $rc
  for cfg in ${CFGS:-cfg2 cfg2u8}; do
    SDR_FIR_VARIANT=$v timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline \
        > "$OUT/bench_${cfg}_$v.json" 2>>"$OUT/bench.err"
    rc=$?; [ $rc -eq 0 ] || exit $rc
    python -c "import json;d=json.load(open('$OUT/bench_${cfg}_$v.json'));print('  $v $cfg', d['value'], 'MS/s', d['ms_per_step'],'ms', d['roofline']['frac'])"
  done
done
