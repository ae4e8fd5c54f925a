"""cfg3 resample_lp launches for the per-wave phase trace of profiles/r02_resample_trace/
(needs the temporary SDR_RESAMPLE_TRACE build described there; the tree does not carry it): times of
workgroup 0 (s_memtime ticks) printed by the launcher to stderr."""
import os
import sys

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "3dy4-real-time-software-defined-radio-_amd"))
import torch  # noqa: E402

import sdrhip  # noqa: E402

up, down, T, n, S = 147, 800, 151 * 147, 65600, 1024
ctx = sdrhip.Context(0)
dev = torch.device("cuda:0")
h = torch.from_numpy(sdrhip.taps_lpf(240e3 * 147, 16e3, T, 147)).to(dev)
x = torch.randn(S * n, device=dev) * 0.1
ny = sdrhip.resample_out_len(up, down, n)
y = torch.empty(S * ny, device=dev)
ns = T // up - 1
st = torch.zeros(S * ns, device=dev)
plan = ctx.resample_plan(up, down, h, T)
torch.cuda.synchronize()
for i in range(int(os.environ.get("REPS", "4"))):
    print(f"launch {i}", file=sys.stderr, flush=True)
    plan.resample_dev(x, n, S, n, st, ns, y, ny)
torch.cuda.synchronize()
