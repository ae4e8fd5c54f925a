"""Timing probe (no parity claim): how much of mono0's audio stage would hide
under the next block's front end if the two ran on two streams.

Per step: the u8 front end (1,024 x 51,200 pairs, FIR101 / 10 + demod) into
one of two row slots, then the audio FIR / 5 of that slot (sdr_fir_decim).
  serial:    both on one stream;
  pipelined: front(k) on stream A, decim(k) on stream B after front(k);
             front(k) waits for decim(k-2) (the slot's previous reader).
Random taps, one synthetic batch; prints ms per step for each."""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..",
                                "3dy4-real-time-software-defined-radio-_amd"))
import sdrhip  # noqa: E402

S, n, D, DA = 1024, 51200, 10, 5
nd, na = n // D, n // D // DA
dev = torch.device("cuda:0")
g = torch.Generator(device="cpu").manual_seed(1)
h = ((torch.rand(101, generator=g) * 2 - 1) / 101).to(dev)
ha = ((torch.rand(101, generator=g) * 2 - 1) / 101).to(dev)
sA, sB = torch.cuda.Stream(dev), torch.cuda.Stream(dev)
ctx, ctx2 = sdrhip.Context(0), sdrhip.Context(0)
ctx.set_stream(sA.cuda_stream)
ctx2.set_stream(sB.cuda_stream)
iq = torch.empty(S * 2 * n, dtype=torch.uint8, device=dev)
ctx.synth_fm_u8_dev(iq, n, S, 2 * n, 7)
z = lambda k: torch.zeros(k, dtype=torch.float32, device=dev)  # noqa: E731
st0, st1, p0, p1, sa = z(S * 100), z(S * 100), z(S), z(S), z(S * 100)
slots = [z(S * nd), z(S * nd)]
out = z(S * na)
ev_f = [sdrhip.Event(ctx) for _ in range(2)]
ev_b = [sdrhip.Event(ctx) for _ in range(2)]


def front(k, c):
    c.frontend_u8_dev(D, iq, n, S, 2 * n, h, 101, st0, st1, 100, p0, p1, slots[k % 2], nd)


def back(k, c):
    c.fir_decim_dev(DA, slots[k % 2], nd, S, nd, ha, 101, sa, 100, out, na)


def serial(k0, K):
    for k in range(k0, k0 + K):
        front(k, ctx)
        back(k, ctx)


def piped(k0, K):
    for j in range(K):
        k = k0 + j
        if j >= 2:
            ev_b[k % 2].wait(ctx)
        front(k, ctx)
        ev_f[k % 2].record(ctx)
        ev_f[k % 2].wait(ctx2)
        back(k, ctx2)
        ev_b[k % 2].record(ctx2)
    ev_b[(k0 + K - 1) % 2].wait(ctx)


def timed(fn, K=100, reps=3):
    res = []
    for _ in range(reps):
        fn(0, 20)
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record(sA)
        fn(0, K)
        e1.record(sA)
        torch.cuda.synchronize()
        res.append(e0.elapsed_time(e1) / K)
    return res


for name, fn in (("serial", serial), ("pipelined", piped), ("serial", serial), ("pipelined", piped)):
    print(name, " ".join(f"{v:.4f}" for v in timed(fn)), "ms/step", flush=True)
