#!/bin/bash
# Split-channel fir_tile (one LDS buffer): parity under the variant switch, then warm A/B, same box.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_split; mkdir -p "$OUT"
for v in 2x1s 4x1s; do
  SDR_FIR_VARIANT=$v timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -m gpu -x -q -p no:cacheprovider \
    --timeout 120 --timeout-method thread > "$OUT/pytest_$v.log" 2>&1
  rc=$?; echo "parity $v: $(tail -1 $OUT/pytest_$v.log)"; [ $rc -eq 0 ] || exit $rc
done
b() { local label=$1; shift
  r=$(env "$@" timeout -k 10 120 python bench.py --config ${CFG:-cfg2} --steps 100 --warmup 5 --no-cpu-baseline 2>>"$OUT/err.log" |
      python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'], d.get('fma_variant',{}).get('ms_per_step'))")
  rc=$?; echo "$label: $r" | tee -a "$OUT/results.txt"; return $rc; }
for rep in 1 2; do
  b "cfg2 default rep$rep" || exit 1
  for w in 32 64 96; do b "cfg2 split wpc$w rep$rep" SDR_FIR_VARIANT=2x1s SDR_WG_PER_CU=$w || exit 1; done
  CFG=cfg2u8 b "u8 default rep$rep" || exit 1
  for w in 32 64; do CFG=cfg2u8 b "u8 split wpc$w rep$rep" SDR_FIR_VARIANT=2x1s SDR_WG_PER_CU=$w || exit 1; done
  CFG=mono0 b "mono0 default rep$rep" || exit 1
  CFG=mono0 b "mono0 split rep$rep" SDR_FIR_VARIANT=2x1s || exit 1
done
