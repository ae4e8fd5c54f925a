#!/bin/bash
# Where does the fused front-end kernel spend its time?  SDR_ABLATE=1 drops
# the global loads, =2 drops the FIR math (timings only; outputs garbage).
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
for v in ${VARIANTS:-2x1}; do
  for ab in 0 1 2; do
    for cfg in cfg2 cfg2u8; do
      r=$(SDR_ABLATE=$ab SDR_FIR_VARIANT=$v timeout -k 10 300 python bench.py --config $cfg --steps 20 --warmup 5 --no-cpu-baseline 2>/dev/null | python -c "import json,sys; d=json.loads(sys.stdin.read()); print(d['ms_per_step'])")
      echo "variant $v ablate $ab $cfg: $r ms"
    done
  done
done
