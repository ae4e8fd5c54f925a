#!/bin/bash
# Same-box A/B of one env switch on one bench config, after the tests that
# cover it: VAR=<env name> CFG=<config> TESTK=<pytest -k> bash scripts/ab_env.sh
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/${TAG:-ab_env}
mkdir -p "$OUT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py -m gpu -x -q -p no:cacheprovider -rf \
  --timeout 120 --timeout-method thread -k "${TESTK}" > "$OUT/pytest.log" 2>&1
rc=$?; tail -4 "$OUT/pytest.log"; [ $rc -eq 0 ] || { echo "pytest rc=$rc"; exit $rc; }
for rep in 1 2 3; do
  for v in 1 0; do
    r=$(env "$VAR=$v" timeout -k 10 120 python bench.py --config "$CFG" --steps 100 --warmup 3 --no-cpu-baseline --sustain-seconds 0 2>>"$OUT/bench.err" |
        python -c "import json,sys;d=json.loads(sys.stdin.read());print(d['ms_per_step'], d['roofline']['frac'])")
    rc=$?; echo "rep $rep $VAR=$v: $r"; [ $rc -eq 0 ] || exit $rc
  done
done
