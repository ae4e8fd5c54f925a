#!/bin/bash
# GPU clock/power while cfg2 (exact, then fma) runs back to back; torchrun N=1 rehearsal.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
OUT=gpurun_out/exp_clock; mkdir -p "$OUT"
( for i in $(seq 1 40); do date +%s.%N; amd-smi metric -g 0 -p -c 2>&1 | grep -iE "SOCKET_POWER|GFX_0|CLK|POWER" | head -12; sleep 0.5; done ) > "$OUT/idle_then_busy.txt" 2>&1 &
SP=$!
sleep 3
timeout -k 10 120 python bench.py --steps 30000 --warmup 5 --no-cpu-baseline --no-fma-variant > "$OUT/exact.json" 2>>"$OUT/err.log" || { kill $SP; exit 1; }
timeout -k 10 120 python bench.py --steps 30000 --warmup 5 --no-cpu-baseline --no-fma-variant --arith fma > "$OUT/fma.json" 2>>"$OUT/err.log" || { kill $SP; exit 1; }
wait $SP
timeout -k 10 180 python -m torch.distributed.run --nnodes=1 --nproc-per-node 1 --master-addr 127.0.0.1 --master-port 29531 \
  bench.py --gpus 1 --steps 10 --warmup 3 > "$OUT/torchrun1.json" 2>>"$OUT/err.log"
rc=$?; cat "$OUT/torchrun1.json"; exit $rc
