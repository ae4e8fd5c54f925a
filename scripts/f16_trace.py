"""Phase anatomy of fir_long_mfma on cfg5h's launch (2 x 1,048,576, 1024 taps,
tap plan) from a TIMING build's per-wave wall-clock stamps (SDR_F16_TRACE=1):
    SDRHIP_LIB=ab/timing.so SDR_F16_TRACE=1 python scripts/f16_trace.py
Stamps are 100 MHz (10 ns); every figure is relative to the launch's first
wave entry.  Phases per wave: entry -> staging barrier -> MFMA loop done ->
stores issued -> stores complete."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3dy4-real-time-software-defined-radio-_amd"))
import sdrhip  # noqa: E402

W = 40  # stamps per workgroup (kMfTraceW)
n, T, ns = 1048576, 1024, 1023
dev = torch.device("cuda:0")
ctx = sdrhip.Context(0)
g = torch.Generator(device="cpu").manual_seed(5)
x = (torch.rand(2 * n, generator=g) * 2 - 1).to(dev)
xh = torch.empty(2 * n, dtype=torch.float16, device=dev)
ctx.f32_to_f16_dev(x, 2 * n, xh)
h = (torch.rand(T, generator=g) * 2 - 1).div(T).to(dev)
st = torch.zeros(2 * ns, dtype=torch.float16, device=dev)
y = torch.empty(2 * n, dtype=torch.float32, device=dev)
plan = ctx.fir_f16_plan(h, T)
L = sdrhip.lib()
L.sdr_timing_f16_trace.restype = C.c_longlong
L.sdr_timing_f16_trace.argtypes = [C.c_void_p, C.c_longlong]
reps = int(os.environ.get("REPS", "5"))
rows = []
for r in range(50 + reps):
    plan.fir_block_f16_dev(xh, n, 2, n, st, ns, y, n)
    if r >= 50:
        cnt = L.sdr_timing_f16_trace(None, 0)
        buf = np.zeros(cnt, dtype=np.uint64)
        L.sdr_timing_f16_trace(buf.ctypes.data, cnt)
        t = buf.reshape(-1, 5, 8).astype(np.int64)
        nw = int((t[:, 0, :] != 0).any(axis=0).sum())  # waves per workgroup (4 or 8)
        rows.append(t[:, :, :nw])
for r, t in enumerate(rows):
    t0 = t[:, 0, :].min()
    rel = (t - t0) * 10e-3  # us
    entry, bar, mf, iss, done = (rel[:, k, :] for k in range(5))
    def q(v):
        return "min %5.2f  p50 %5.2f  p90 %5.2f  max %5.2f" % (v.min(), np.median(v), np.percentile(v, 90), v.max())
    print(f"launch {r}: {t.shape[0]} workgroups, span {done.max():.2f} us (first entry -> last store complete)")
    print("  entry (dispatch spread)      ", q(entry))
    print("  barrier (staging wait)       ", q(bar - entry))
    print("  MFMA loop                    ", q(mf - bar))
    print("  output stores issued         ", q(iss - mf))
    print("  stores complete after issue  ", q(done - iss))
    print("  barrier time (abs)           ", q(bar))
    print("  MFMA done (abs)              ", q(mf))
    print("  done (abs)                   ", q(done))
    stw = (bar - entry).max(axis=1)  # per workgroup: slowest wave's staging wait
    worst = np.argsort(stw)[-6:][::-1]
    print("  slowest staging (workgroup: us):", ", ".join(f"{w}: {stw[w]:.2f}" for w in worst),
          "| workgroup 0:", f"{stw[0]:.2f}", "| last of stream 0:", f"{stw[t.shape[0] // 2 - 1]:.2f}")
    for w in (0, 1, t.shape[0] // 2):
        e = (t[w, 0, :] - t[w, 0, :].min()) * 10e-3
        b = (t[w, 1, :] - t[w, 0, :].min()) * 10e-3
        print(f"  workgroup {w}: wave entries +" + " ".join(f"{v:.2f}" for v in e) + " | past barrier +" +
              " ".join(f"{v:.2f}" for v in b))
    wg_first = t[:, 0, :].min(axis=1)
    order = np.argsort(wg_first)
    print("  last-entry workgroups:", order[-4:].tolist(), "first-entry:", order[:4].tolist())
