set -u
OUT=gpurun_out/r03_pllg; mkdir -p $OUT
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_dropin.py tests/test_gpu_scale.py -m gpu -x -q -p no:cacheprovider -rf --timeout 120 --timeout-method thread -k "pll or stereo" > $OUT/pytest.log 2>&1
rc=$?; tail -4 $OUT/pytest.log; [ $rc -eq 0 ] || exit $rc
ARMS="tree:SDR_PLL_GUARD=1 tree:SDR_PLL_GUARD=0" CFGS="stereo0 stereo0w" REPS=2 bash scripts/ab_libs.sh
