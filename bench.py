#!/usr/bin/env python3
"""Benchmark: IQ MSamples/s through FIR + decimate + FM demod on MI355X.

Default workload (BASELINE.json configs[1]): the mode-0 RF front end -- a
101-tap LPF (impulseResponseLPF(2.4e6, 100e3, 101), src/filter.cpp:14-29),
decimate by 10 and the FM discriminator (src/project.cpp:86-90) -- on
blocks of 65,540 IQ pairs (65,536 rounded up to a multiple of 10, the
reference's own precondition), fp32 planar I/Q resident in HBM.  One step =
the next block of each of 1024 independent synthetic streams (state carried
across steps exactly as the reference carries it between blocks), i.e. one
batched launch of the fused kernel over 67.1 M IQ pairs.

Multi-GPU: one process per GPU (torch.distributed.run); every rank runs
its own 1024 streams (weak scaling, no data-path collective -- the streams
are independent); the only collectives are the timing barrier and the
max-over-ranks of the elapsed time.

Prints ONE JSON line (rank 0).  Other workloads: --config cfg2u8 (u8 wire
input fused in), cfg3 (polyphase resampler 147/800, 151 taps/phase),
cfg4 (8 long streams x 32 x 262,150-pair blocks per GPU), cfg5 (1024-tap
FIR, no decimation).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "3dy4-real-time-software-defined-radio-_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
FP32_VALU_PEAK_TFLOPS = 157.3

CONFIGS = {
    # name: (kind, D or (up, down), ntaps, pairs per stream per step, streams per GPU)
    "cfg2": dict(kind="frontend_f32", D=10, ntaps=101, n=65540, streams=1024,
                 workload="fir101_dec10_fmdemod_f32_block65540"),
    "cfg2u8": dict(kind="frontend_u8", D=10, ntaps=101, n=65540, streams=1024,
                   workload="fir101_dec10_fmdemod_u8wire_block65540"),
    "cfg3": dict(kind="resample", up=147, down=800, ntaps=151 * 147, n=65600, streams=1024,
                 workload="polyphase_resampler_147_800_151pp_block65600"),
    "cfg4": dict(kind="frontend_f32", D=10, ntaps=101, n=262150 * 32, streams=8,
                 workload="fir101_dec10_fmdemod_f32_8streams_x32blocks_of_262150"),
    "cfg5": dict(kind="fir_block", D=1, ntaps=1024, n=1048576, streams=2,
                 workload="fir1024_block1M_f32_IandQ"),
    # SURVEY 8(f) 2+4: the reference program's whole mono path (mode 0) on the device,
    # u8 IQ -> front end -> delay -> audio FIR+dec5 -> s16 PCM, 51,200-pair reference blocks
    "mono0": dict(kind="mono_u8", D=10, up=1, down=5, ntaps=101, n=51200, streams=1024,
                  workload="mode0_mono_u8iq_to_s16pcm_block51200"),
    # SURVEY 8(f) 2 (stereo half): the whole mode-0 stereo path, PLL one lane per stream
    "stereo0": dict(kind="stereo_u8", D=10, up=1, down=5, ntaps=101, n=51200, streams=1024,
                    workload="mode0_stereo_u8iq_to_s16pcm_LR_block51200"),
    # the same with 16x the streams: the PLL recurrence is latency-bound per stream (one lane
    # each), so 1,024 streams occupy 16 waves of the chip; more streams per step fill it
    "stereo0w": dict(kind="stereo_u8", D=10, up=1, down=5, ntaps=101, n=51200, streams=16384,
                     workload="mode0_stereo_u8iq_to_s16pcm_LR_block51200_16k_streams"),
    # BASELINE config 5's fp16 arm: fp16 storage, fp32 accumulation (v_dot2_f32_f16); not
    # bit-exact -- the line carries its error against the exact fp32 path
    "cfg5h": dict(kind="fir_block_f16", D=1, ntaps=1024, n=1048576, streams=2,
                  workload="fir1024_block1M_f16storage_IandQ"),
}


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", default="cfg2", choices=sorted(CONFIGS))
    ap.add_argument("--cpu-seconds", type=float, default=12.0, help="CPU-baseline sample budget (rank 0, N=1)")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--warm-seconds", type=float, default=0.25,
                    help="after the W warmup steps, keep running untimed steps for this long (clock ramp)")
    ap.add_argument("--no-fma-variant", action="store_true", help="skip the SDR_ARITH_FMA side measurement")
    ap.add_argument("--arith", choices=("exact", "fma"), default=os.environ.get("SDR_BENCH_ARITH", "exact"),
                    help="front-end FIR arithmetic: the reference's bits (exact) or one fused multiply-add per tap "
                         "(fma, tolerance-tested)")
    return ap.parse_args()


def cpu_baseline(seconds: float):
    """The reference's own front end (oracle/_ref, kind 'reference') or, if it
    was not built, the bit-exact C restatement (kind 'port'), timed on this
    host's cores over a bounded sample of the same workload: 65,540-pair
    mode-0 blocks, one independent stream per thread."""
    sys.path.insert(0, os.path.join(REPO, "oracle"))
    import oracle as orc
    from sdrhip.synth import fm_planar

    h = orc.Oracle().taps_lpf(2.4e6, 100e3, 101, 1)
    blocks = [fm_planar(65540, seed=900 + i) for i in range(4)]
    if orc.available_reference():
        ref = orc.Reference()
        kind = "reference"

        def make_runner():
            r = ref.frontend_runner(h, 100)
            return lambda I, Q: r.run(10, I, Q)
    else:
        o = orc.Oracle()
        kind = "port"

        def make_runner():
            si, sq, pv = np.zeros(100, np.float32), np.zeros(100, np.float32), np.zeros(2, np.float32)
            return lambda I, Q: o.frontend(10, I, Q, h, si, sq, pv)

    def measure(nthreads: int, budget: float):
        counts = [0] * nthreads
        stop = time.perf_counter() + budget

        def work(t):
            run = make_runner()
            i = t
            while time.perf_counter() < stop:
                I, Q = blocks[i % len(blocks)]
                run(I, Q)
                counts[t] += len(I)
                i += 1

        t0 = time.perf_counter()
        ths = [threading.Thread(target=work, args=(t,)) for t in range(nthreads)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        return sum(counts) / (time.perf_counter() - t0) / 1e6, sum(counts)

    try:
        ncpu = len(os.sched_getaffinity(0))
    except AttributeError:
        ncpu = os.cpu_count() or 1
    threads = max(1, min(16, ncpu))
    one, n1 = measure(1, seconds / 3)
    many, nm = measure(threads, 2 * seconds / 3)
    import platform

    model = "unknown"
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    model = line.split(":", 1)[1].strip()
                    break
    except OSError:
        pass
    return {"value": round(many, 2), "unit": "MS/s", "cores": threads, "kind": kind,
            "value_1core": round(one, 2),
            "sample": f"{nm + n1} IQ pairs in 65,540-pair mode-0 blocks (101-tap FIR+dec10 on I and Q, then the "
                      f"discriminator), {threads} threads x independent streams for {2 * seconds / 3:.0f} s + 1 "
                      f"thread for {seconds / 3:.0f} s; host {model} ({platform.machine()}), "
                      f"{ncpu} cores visible"}


def main():
    args = parse()
    import torch
    import torch.distributed as dist

    import sdrhip

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus and rank == 0:
        print(f"warning: --gpus {args.gpus} but WORLD_SIZE {world}", file=sys.stderr)
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    if world > 1:
        dist.init_process_group("nccl", rank=rank, world_size=world, device_id=dev)

    cfg = CONFIGS[args.config]
    ctx = sdrhip.Context(local)
    # one dedicated (non-null) HIP stream shared by torch and the library, so
    # torch.cuda.Event timestamps bracket exactly the kernels we launch
    stream = torch.cuda.Stream(dev)
    torch.cuda.set_stream(stream)
    ctx.set_stream(stream.cuda_stream)
    ctx.set_arith(sdrhip.ARITH_FMA if args.arith == "fma" else sdrhip.ARITH_EXACT)

    S, n, T = cfg["streams"], cfg["n"], cfg["ntaps"]
    seed = 1234 + 7919 * rank
    # taps: the product's coefficient design (C ABI sdr_taps_lpf, bit-identical
    # to the reference's impulseResponseLPF); setup, not timed
    if cfg["kind"] == "resample":
        taps = sdrhip.taps_lpf(240e3 * 147, 16e3, T, 147)
    else:
        taps = sdrhip.taps_lpf(2.4e6, 100e3, T, 1)
    if cfg["kind"] in ("mono_u8", "stereo_u8"):  # src/project.cpp:263-273: audio LPF (+ BPFs) of mode 0
        d_ha = torch.from_numpy(sdrhip.taps_lpf(240e3, 16e3, 101, 1)).to(dev)
        d_hp = torch.from_numpy(sdrhip.taps_bpf(240e3, 18.5e3, 19.5e3, 101, 1)).to(dev)
        d_hs = torch.from_numpy(sdrhip.taps_bpf(240e3, 22e3, 54e3, 101, 1)).to(dev)
    d_h = torch.from_numpy(taps).to(dev)

    # synthetic input generated on the device (no host traffic), then kept resident
    iq = torch.empty(S * 2 * n, dtype=torch.uint8, device=dev)
    ctx.synth_fm_u8_dev(iq, n, S, 2 * n, seed)
    kind = cfg["kind"]
    if kind in ("frontend_f32", "fir_block", "fir_block_f16", "resample"):
        I = torch.empty(S * n, dtype=torch.float32, device=dev)
        Q = torch.empty(S * n, dtype=torch.float32, device=dev)
        ctx.u8_to_planar_dev(iq, n, S, 2 * n, I, Q, n)
        torch.cuda.synchronize(dev)
        del iq
    ns = {"resample": 150, "fir_block": T - 1, "fir_block_f16": T - 1}.get(kind, 100)
    st0 = torch.zeros(S * ns, dtype=torch.float32, device=dev)
    st1 = torch.zeros(S * ns, dtype=torch.float32, device=dev)
    p0 = torch.zeros(S, dtype=torch.float32, device=dev)
    p1 = torch.zeros(S, dtype=torch.float32, device=dev)

    if kind == "mono_u8":
        D, up, down = cfg["D"], cfg["up"], cfg["down"]
        na = sdrhip.resample_out_len(up, down, n // D)
        sd = torch.zeros(S * 50, dtype=torch.float32, device=dev)
        sa = torch.zeros(S * 100, dtype=torch.float32, device=dev)
        pcm = torch.empty(S * na, dtype=torch.int16, device=dev)
        step = lambda: ctx.mono_pcm_u8_dev(D, iq, n, S, 2 * n, d_h, T, st0, st1, ns, p0, p1, sd, 50, up, down,  # noqa
                                           d_ha, 101, sa, 100, pcm, na)
        units = S * n
        bytes_per_pair = 2.0 + 2.0 * na / n  # u8 IQ in, s16 PCM out (intermediates are algorithmically free)
        flops_per_unit = 2 * 2 * T / D + 10 + 2.0 * 101 / (D * down) + 1
        unit = "MS/s"
        metric = "IQ MSamples/sec through the mode-0 mono path (u8 IQ -> s16 PCM)"
        bound = "valu"
    elif kind == "stereo_u8":
        D, up, down = cfg["D"], cfg["up"], cfg["down"]
        na = sdrhip.resample_out_len(up, down, n // D)
        z = lambda k: torch.zeros(S * k, dtype=torch.float32, device=dev)  # noqa: E731
        sbuf = dict(delay=z(50), audio=z(100), slp=z(100), pilot=z(100), stereo=z(100),
                    pll=torch.tensor([1, 0, 0, 0, 0, 1], dtype=torch.float32, device=dev).repeat(S))
        taps_s = sdrhip.StereoTaps(d_h.data_ptr(), T, d_ha.data_ptr(), 101, d_hp.data_ptr(), d_hs.data_ptr(), 101)
        state_s = sdrhip.StereoState(st0.data_ptr(), st1.data_ptr(), ns, p0.data_ptr(), p1.data_ptr(),
                                     sbuf["delay"].data_ptr(), 50, sbuf["audio"].data_ptr(), sbuf["slp"].data_ptr(),
                                     100, sbuf["pilot"].data_ptr(), sbuf["stereo"].data_ptr(), 100,
                                     sbuf["pll"].data_ptr())
        pcm = torch.empty(S * 2 * na, dtype=torch.int16, device=dev)
        step = lambda: ctx.stereo_pcm_u8_dev(D, iq, n, S, 2 * n, up, down, 240e3, taps_s, state_s, pcm,  # noqa
                                             2 * na)
        units = S * n
        bytes_per_pair = 2.0 + 4.0 * na / n
        # front end + mono LPF + 2 BPFs + stereo LPF (2 FLOP per tap) + demod/PLL/mixer
        flops_per_unit = 2 * 2 * T / D + 10 + (2.0 * 101 * 2 / (D * down) + 2 * 2.0 * 101 / D) + 1
        unit = "MS/s"
        metric = "IQ MSamples/sec through the mode-0 stereo path (u8 IQ -> interleaved s16 L/R PCM)"
        bound = "valu"
    elif kind in ("frontend_f32", "frontend_u8"):
        D = cfg["D"]
        nout = n // D
        out = torch.empty(S * nout, dtype=torch.float32, device=dev)
        if kind == "frontend_f32":
            step = lambda: ctx.frontend_dev(D, I, Q, n, S, n, d_h, T, st0, st1, ns, p0, p1, out, nout)  # noqa: E731
            bytes_per_pair = 8.0 + 4.0 / D
        else:
            step = lambda: ctx.frontend_u8_dev(D, iq, n, S, 2 * n, d_h, T, st0, st1, ns, p0, p1, out, nout)  # noqa
            bytes_per_pair = 2.0 + 4.0 / D
        units = S * n  # IQ pairs per step
        flops_per_unit = 2 * 2 * T / D + 10
        unit = "MS/s"
        metric = "IQ MSamples/sec through FIR+decimate+FM-demod"
        # f32 planar input: 8.4 B against ~41 FLOP per pair -> HBM-bound; the u8
        # wire format moves 2.4 B per pair, which puts the exact (no-FMA) FIR
        # arithmetic above the ridge -> VALU-bound
        bound = "hbm" if kind == "frontend_f32" else "valu"
    elif kind == "resample":
        up, down = cfg["up"], cfg["down"]
        ny = sdrhip.resample_out_len(up, down, n)
        out = torch.empty(S * ny, dtype=torch.float32, device=dev)
        step = lambda: ctx.resample_dev(up, down, I, n, S, n, d_h, T, st0, ns, out, ny)  # noqa: E731
        units = S * n  # input samples per step
        bytes_per_pair = 4.0 + 4.0 * up / down
        flops_per_unit = 2.0 * (T / up) * up / down
        unit = "MS/s"
        metric = "IF MSamples/sec (input) through the polyphase resampler"
        bound = "hbm"
    elif kind == "fir_block":  # I and Q as two streams
        out = torch.empty(S * n, dtype=torch.float32, device=dev)
        IQ = torch.stack([I[:n], Q[:n]])
        step = lambda: ctx.fir_block_dev(IQ, n, 2, n, d_h, T, st0, ns, out, n)  # noqa: E731
        units = n  # IQ pairs per step (I and Q each n samples)
        bytes_per_pair = 16.0
        flops_per_unit = 2.0 * 2 * T
        unit = "MS/s"
        metric = "IQ MSamples/sec through a 1024-tap FIR"
        bound = "valu"
    else:  # fir_block_f16: fp16 storage of I and Q (converted once, untimed)
        IQ = torch.stack([I[:n], Q[:n]])
        IQh = torch.empty(2 * n, dtype=torch.float16, device=dev)
        ctx.f32_to_f16_dev(IQ, 2 * n, IQh)
        sth = torch.zeros(2 * ns, dtype=torch.float16, device=dev)
        out = torch.empty(2 * n, dtype=torch.float32, device=dev)
        step = lambda: ctx.fir_block_f16_dev(IQh, n, 2, n, d_h, T, sth, ns, out, n)  # noqa: E731
        units = n
        bytes_per_pair = 2.0 * 2 + 8.0  # fp16 in, fp32 out
        flops_per_unit = 2.0 * 2 * T
        unit = "MS/s"
        metric = "IQ MSamples/sec through a 1024-tap FIR"
        bound = "valu"
        # error of this arm against the exact fp32 path on the same first block
        ref = torch.empty(2 * n, dtype=torch.float32, device=dev)
        z32 = torch.zeros(2 * ns, dtype=torch.float32, device=dev)
        ctx.fir_block_dev(IQ, n, 2, n, d_h, T, z32, ns, ref, n)
        z16 = torch.zeros(2 * ns, dtype=torch.float16, device=dev)
        got = torch.empty(2 * n, dtype=torch.float32, device=dev)
        ctx.fir_block_f16_dev(IQh, n, 2, n, d_h, T, z16, ns, got, n)
        torch.cuda.synchronize(dev)
        err = float((got - ref).abs().max())
        scale = float(d_h.abs().sum()) * float(IQ.abs().max())
        tolerance = {"max_abs_err_vs_fp32_exact": err, "normalized": err / scale,
                     "norm": "sum|h| * max|x|", "rms_err": float((got - ref).pow(2).mean().sqrt())}

    # W warmup steps, then more of the same launches until >= --warm-seconds
    # of wall time has passed: an idle MI355X sits at ~0.1 GHz and its clock
    # ramps over tens of ms; a few warmup steps (<1 ms) would time part of
    # the ramp, not the sustained rate a streaming receiver runs at.
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize(dev)
    t_warm = time.perf_counter()
    while time.perf_counter() - t_warm < args.warm_seconds:
        for _ in range(10):
            step()
        torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    e0 = torch.cuda.Event(enable_timing=True)
    e1 = torch.cuda.Event(enable_timing=True)
    t_wall = time.perf_counter()
    e0.record(stream)
    for _ in range(args.steps):
        step()
    e1.record(stream)
    torch.cuda.synchronize(dev)
    wall = time.perf_counter() - t_wall
    if world > 1:
        dist.barrier()
    ms_gpu = e0.elapsed_time(e1)
    ms = torch.tensor([ms_gpu, wall * 1e3], dtype=torch.float64, device=dev)
    if world > 1:
        dist.all_reduce(ms, op=dist.ReduceOp.MAX)
    ms_events, ms_wall = float(ms[0]), float(ms[1])

    ms_per_step = ms_events / args.steps
    total_units = units * args.steps * world
    value = total_units / (ms_events * 1e-3) / 1e6
    launch_s = ms_per_step * 1e-3
    if bound == "hbm":
        achieved = units * bytes_per_pair / launch_s / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4)}
    else:
        achieved = units * flops_per_unit / launch_s / 1e12
        # fp16 arm: v_dot2_f32_f16 retires two products per lane per issue -> twice the fp32 vector peak
        peak = FP32_VALU_PEAK_TFLOPS * (2 if kind == "fir_block_f16" else 1)
        roof = {"bound": "valu", "achieved": round(achieved, 2), "peak": peak, "unit": "TFLOP/s",
                "frac": round(achieved / peak, 4)}
    traffic = None
    tpath = os.path.join(REPO, "profiles", f"traffic_{args.config}.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            t = json.load(f)
        traffic = t.get("hbm_bytes_per_launch")
        roof["traffic_source"] = os.path.relpath(tpath, REPO)
    roof["traffic"] = traffic
    roof["algorithmic_bytes_per_launch"] = int(units * bytes_per_pair)

    if kind != "fir_block_f16":
        tolerance = None
    # Side measurement (1 GPU, fused front end, exact run only): the same
    # launches under SDR_ARITH_FMA -- one fused multiply-add per tap, not the
    # reference's bits (tolerance-tested).  Reported beside the
    # headline, never as `value`.
    fma_variant = None
    if world == 1 and args.arith == "exact" and kind in ("frontend_f32", "frontend_u8") and not args.no_fma_variant:
        ctx.set_arith(sdrhip.ARITH_FMA)
        for _ in range(max(args.warmup, 2)):
            step()
        torch.cuda.synchronize(dev)
        t_warm = time.perf_counter()
        while time.perf_counter() - t_warm < args.warm_seconds:
            for _ in range(10):
                step()
            torch.cuda.synchronize(dev)
        f0 = torch.cuda.Event(enable_timing=True)
        f1 = torch.cuda.Event(enable_timing=True)
        f0.record(stream)
        for _ in range(args.steps):
            step()
        f1.record(stream)
        torch.cuda.synchronize(dev)
        ctx.set_arith(sdrhip.ARITH_EXACT)
        fms = f0.elapsed_time(f1) / args.steps
        fval = units / (fms * 1e-3) / 1e6
        if bound == "hbm":
            ffrac = units * bytes_per_pair / (fms * 1e-3) / 1e9 / HBM_PEAK_GBS
        else:
            ffrac = units * flops_per_unit / (fms * 1e-3) / 1e12 / FP32_VALU_PEAK_TFLOPS
        fma_variant = {"arith": "fma (SDR_ARITH_FMA): one fused multiply-add per tap; within the fp32 tolerance, "
                                "not the reference's bits",
                       "value": round(fval, 1), "ms_per_step": round(fms, 4), "roofline_frac": round(ffrac, 4)}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline and args.config in ("cfg2", "cfg2u8", "cfg4"):
        cpu = cpu_baseline(args.cpu_seconds)
    if rank == 0:
        line = {
            "metric": metric, "value": round(value, 1), "unit": unit, "n_gpus": world, "steps": args.steps,
            "warmup": args.warmup, "ms_per_step": round(ms_per_step, 4), "higher_is_better": True,
            "scaling": "weak", "vs_baseline": None, "dtype": "f16" if kind == "fir_block_f16" else "f32",
            "data": "synthetic",
            "config": {"workload": cfg["workload"], "streams_per_gpu": S, "pairs_per_stream_per_step": n,
                       "ntaps": T, "parallelism": f"{world} GPU(s) x independent streams, no data-path collective",
                       "state_carried_across_steps": True,
                       "arith": ("fma: one fused multiply-add per tap, tolerance-tested (DESIGN.md 2)"
                                 if args.arith == "fma" else "exact: the reference's bits")},
            "roofline": roof, "cpu_baseline": cpu,
            **({"tolerance": tolerance} if tolerance else {}),
            **({"fma_variant": fma_variant} if fma_variant else {}),
            "wall_ms": round(ms_wall, 3),
        }
        print(json.dumps(line), flush=True)
    ctx.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
