#!/bin/bash
# r04n: PLL certified domain extended to a saturated trigOffset (2^24): PLL / stereo parity, then
# stereo0 timed vs sustained (the sustained window crosses 2^24 samples per stream)
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_scale.py tests/test_dropin.py -m gpu -x -q -p no:cacheprovider --timeout 300 --timeout-method thread -k "pll or stereo or sdr_project" > gpurun_out/r04n_pytest.log 2>&1; rc=$?
tail -3 gpurun_out/r04n_pytest.log; [ $rc -eq 0 ] || { grep -E "FAILED|Error|assert" gpurun_out/r04n_pytest.log | head; exit $rc; }
for c in stereo0 stereo0w; do
  timeout -k 10 300 python bench.py --config $c --steps 100 --warmup 3 --no-cpu-baseline > gpurun_out/r04n_bench_$c.json 2>>gpurun_out/r04n.err || exit 1
  python3 -c "import json;d=json.load(open('gpurun_out/r04n_bench_$c.json'));print('$c', d['ms_per_step'], d['sustained']['ms_per_step'], d['sustained']['steps'])"
done
