set -u
cd "${GRAFT_REPO_ROOT}"
mkdir -p gpurun_out/warm
for ws in 0.25 1.0 0.25 2.0; do
  for st in 100 1000; do
    timeout -k 10 120 python bench.py --config cfg2 --steps $st --warmup 5 --warm-seconds $ws --no-cpu-baseline --no-fma-variant > gpurun_out/warm/o.json 2>/dev/null || exit 1
    python3 -c "import json;d=json.load(open('gpurun_out/warm/o.json'));print('warm $ws steps $st', d['ms_per_step'], d['roofline']['frac'])"
  done
done
