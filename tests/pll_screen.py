"""Screen of the device PLL's certified short path against its exact-library
path at receiver scale: the same pilot blocks through fm_pll_dev with
SDR_PLL_FAST=1 (csrc/pll_fast.hpp: certified short-chain atan2 / sincos, an
uncertified chunk re-run on libm_exact) and SDR_PLL_FAST=0 (every step on
csrc/libm_exact.hpp, whose floats are glibc's: tests/test_libm_exact.py,
tests/test_gpu_libm.py), state carried across blocks, every NCO output and
every state float compared bitwise on the device.

The reference's fmPLL (src/filter.cpp:174-228) runs on the stereo pilot:
the pilot band-pass output, a ~19 kHz tone at 240 kHz.  The streams here vary
its frequency offset (+-60 Hz), amplitude (1e-3 .. 1), phase and noise level
(0.1 % .. 30 % of the amplitude); 1/16 of them add exact zeros, 1/16 wild
samples (2^-40 .. 2^40 with random signs); trigOffset starts at 0, at random
points below 2^24, or just below 2^24 (where fp32's trigOffset++ stops
advancing), so long screens cover the whole oscillator domain.

    python tests/pll_screen.py --streams 16384 --blocks 200    (GPU; one JSON line)

tests/test_gpu_scale.py::test_pll_fast_vs_library_screen runs a short one in a
child process (torch must open the device before the library does).
"""
from __future__ import annotations

import argparse
import json
import math
import os
import sys
import time

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(os.path.dirname(HERE), "3dy4-real-time-software-defined-radio-_amd"))

FS, F0, NCO_SCALE, PHASE_ADJ, NORM_BW = 240e3, 19e3, 2.0, 0.0, 0.01


def screen(ctx, streams: int, blocks: int, n: int = 5120, seed: int = 1, progress=None, fs: float = FS) -> dict:
    import torch

    import sdrhip

    dev = torch.device("cuda", torch.cuda.current_device())
    g = torch.Generator(device=dev).manual_seed(seed)

    def u(lo, hi, shape=(streams, 1)):
        return lo + (hi - lo) * torch.rand(shape, generator=g, device=dev, dtype=torch.float64)

    f = F0 + u(-60.0, 60.0)
    amp = torch.pow(10.0, u(-3.0, 0.0))
    phi = u(0.0, 2 * math.pi)
    noise = amp * torch.pow(10.0, u(-3.0, -0.5))
    kind = torch.randint(0, 16, (streams, 1), generator=g, device=dev)
    st0 = torch.zeros((streams, 6), dtype=torch.float32, device=dev)
    st0[:, 0] = 1.0
    st0[:, 5] = 1.0
    tk = torch.randint(0, 4, (streams,), generator=g, device=dev)
    late = torch.floor(u(0.0, max(0.0, 16777216.0 - n * blocks), (streams,))).float()
    edge = (16777216.0 - torch.floor(u(0.0, 4.0 * n, (streams,)))).float()
    st0[:, 4] = torch.where(tk == 1, late, torch.where(tk == 2, edge, torch.zeros_like(late)))
    st = {"1": st0.clone(), "0": st0.clone()}
    out = {k: torch.empty((streams, n), dtype=torch.float32, device=dev) for k in st}
    mism_out = mism_state = 0
    t0 = time.time()
    dt = {"1": 0.0, "0": 0.0}
    try:
        for b in range(blocks):
            t = torch.arange(b * n, (b + 1) * n, device=dev, dtype=torch.float64)[None, :]
            x = amp * torch.cos(2 * math.pi * f / fs * t + phi) + noise * torch.randn(
                (streams, n), generator=g, device=dev, dtype=torch.float64)
            zeros = (kind == 0) & (torch.rand((streams, n), generator=g, device=dev) < 0.01)
            x = torch.where(zeros, torch.zeros_like(x), x)
            wild = torch.sign(torch.randn((streams, n), generator=g, device=dev, dtype=torch.float64)) * torch.pow(
                2.0, 80.0 * torch.rand((streams, n), generator=g, device=dev, dtype=torch.float64) - 40.0)
            x = torch.where(kind == 1, wild, x).float().contiguous()
            torch.cuda.synchronize()
            for fast in ("1", "0"):
                sdrhip.set_switch("SDR_PLL_FAST", int(fast))
                c0 = time.time()
                ctx.fm_pll_dev(x, n, streams, n, F0, fs, NCO_SCALE, PHASE_ADJ, NORM_BW, st[fast], None, n, out[fast], n)
                ctx.synchronize()
                dt[fast] += time.time() - c0
            mism_out += int((out["1"].view(torch.int32) != out["0"].view(torch.int32)).sum())
            mism_state += int((st["1"].view(torch.int32) != st["0"].view(torch.int32)).sum())
            if progress is not None and (b + 1) % 50 == 0:
                progress(b + 1, mism_out, mism_state)
    finally:
        sdrhip.set_switch("SDR_PLL_FAST", 1)
    trig = st["1"][:, 4]
    return {"streams": streams, "blocks": blocks, "samples_per_block": n, "seed": seed, "fs": fs,
            "pll_steps": streams * n * blocks, "output_mismatches": mism_out, "state_mismatches": mism_state,
            "trigoffset_max": float(trig.max()), "streams_at_2p24": int((trig >= 16777216.0).sum()),
            "seconds_fast": round(dt["1"], 3), "seconds_library": round(dt["0"], 3),
            "seconds": round(time.time() - t0, 1)}


def main():
    ap = argparse.ArgumentParser(description=__doc__, formatter_class=argparse.RawDescriptionHelpFormatter)
    ap.add_argument("--streams", type=int, default=16384)
    ap.add_argument("--blocks", type=int, default=200)
    ap.add_argument("--n", type=int, default=5120)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--fs", type=float, default=FS,
                    help="the PLL's sample rate: the IF rate of the reference's modes (0/2: 240e3, 1: 288e3, 3: 384e3)")
    a = ap.parse_args()
    import torch

    # torch's HIP runtime first: created after the library's context, it finds no device
    torch.zeros(1, device="cuda")
    import sdrhip

    ctx = sdrhip.Context(0)
    def progress(b, mo, ms):
        print(f"block {b}/{a.blocks}: mismatches {mo} outputs, {ms} state words", file=sys.stderr, flush=True)

    print(json.dumps(screen(ctx, a.streams, a.blocks, a.n, a.seed, progress, a.fs)), flush=True)


if __name__ == "__main__":
    main()
