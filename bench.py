#!/usr/bin/env python3
"""Benchmark: IQ MSamples/s through FIR + decimate + FM demod on MI355X.

Default workload (BASELINE.json configs[1]): the mode-0 RF front end -- a
101-tap LPF (impulseResponseLPF(2.4e6, 100e3, 101), src/filter.cpp:14-29),
decimate by 10 and the FM discriminator (src/project.cpp:86-90) -- on
blocks of 65,540 IQ pairs (65,536 rounded up to a multiple of 10, the
reference's own precondition), fp32 planar I/Q resident in HBM.  One step =
the next block of each of 1024 independent synthetic streams (state carried
across steps exactly as the reference carries it between blocks), i.e. one
batched launch of the fused kernel over 67.1 M IQ pairs.  The steps cycle
over --batches distinct input batches (2 by default: 1.07 GB for cfg2, four
times the 256 MiB Infinity Cache), so no step re-reads a batch the previous
one left on chip.

Multi-GPU: the streams are independent, so every GPU runs
its own streams (weak scaling) and nothing is exchanged -- no RCCL anywhere.
  * ``python bench.py --gpus N`` runs the N devices from ONE process, one
    persistent host thread per device (its own sdr context, HIP stream and
    on-device synthetic input), started together from a host barrier; each
    device is timed with HIP events on its own stream; the aggregate is all
    devices' IQ pairs / the slowest device's time.
  * under ``torch.distributed.run`` (WORLD_SIZE set) every rank runs one
    device (LOCAL_RANK); the timing barrier and the max-over-ranks reduction
    go over a CPU ``gloo`` group -- again no device collective.

Timed steps are replayed from a HIP graph of --graph-steps steps (the
library's sdr_graph_* capture of the same calls), so N host threads never
bound the launch rate; --no-graph launches them one by one.

Prints ONE JSON line.  Other workloads: --config cfg2u8 (u8 wire input
fused in), cfg3 (polyphase resampler 147/800, 151 taps/phase), cfg4 (one
long stream per GPU, 256 x 262,150-pair blocks per step), cfg4x8 (8 streams
per GPU x 32 blocks), cfg5/cfg5h (1024-tap FIR, fp32 / fp16 storage), mono0,
stereo0, stereo0w (the reference program's mode-0 paths on the device).
"""
from __future__ import annotations

import argparse
import json
import os
import subprocess
import sys
import threading
import time

import numpy as np

REPO = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(REPO, "3dy4-real-time-software-defined-radio-_amd")
sys.path.insert(0, PKG)

HBM_PEAK_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md, chip table)
FP32_VALU_PEAK_TFLOPS = 157.3
F16_MFMA_PEAK_TFLOPS = 2500.0  # dense FP16 MFMA (MI355X_MICROARCH.md chip table; not the 2:1-sparse figure)
# discriminator per decimated output (src/filter.cpp:88-98): I*I + Q*Q (3), the two
# differences and products (4), a - b and the divide (2)
DEMOD_FLOP = 9.0

CONFIGS = {
    # name: (kind, D or (up, down), ntaps, pairs per stream per step, streams per GPU)
    "cfg2": dict(kind="frontend_f32", D=10, ntaps=101, n=65540, streams=1024,
                 workload="fir101_dec10_fmdemod_f32_block65540"),
    "cfg2u8": dict(kind="frontend_u8", D=10, ntaps=101, n=65540, streams=1024,
                   workload="fir101_dec10_fmdemod_u8wire_block65540"),
    "cfg3": dict(kind="resample", up=147, down=800, ntaps=151 * 147, n=65600, streams=1024,
                 workload="polyphase_resampler_147_800_151pp_block65600"),
    # BASELINE config 4: one independent stream per GPU; a step is 256 consecutive
    # 262,150-pair blocks of it in one call (block-size independence, src/filter.cpp:139)
    "cfg4": dict(kind="frontend_f32", D=10, ntaps=101, n=262150 * 256, streams=1,
                 workload="fir101_dec10_fmdemod_f32_1stream_x256blocks_of_262150"),
    "cfg4x8": dict(kind="frontend_f32", D=10, ntaps=101, n=262150 * 32, streams=8,
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
    # config 5 as the kernel's streaming rate rather than one launch's fixed cost: 32
    # independent 1 M-sample I/Q blocks (64 channel rows) per launch
    "cfg5b": dict(kind="fir_block", D=1, ntaps=1024, n=1048576, streams=32, blocks=32,
                  workload="fir1024_32blocks_of_1M_f32_IandQ"),
    "cfg5hb": dict(kind="fir_block_f16", D=1, ntaps=1024, n=1048576, streams=32, blocks=32,
                   workload="fir1024_32blocks_of_1M_f16storage_IandQ"),
}
# the fp16 arm's error sweep (cfg5h / cfg5hb lines): input amplitudes x tap counts
F16_SWEEP_AMPS = [2.0 ** -k for k in range(8, -1, -1)]
F16_SWEEP_TAPS = (64, 256, 1024, 4096)


def parse(argv=None):
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
    ap.add_argument("--no-f16-sweep", action="store_true", help="cfg5h/cfg5hb: skip the fp16 error sweep (setup)")
    ap.add_argument("--arith", choices=("exact", "fma"), default=os.environ.get("SDR_BENCH_ARITH", "exact"),
                    help="front-end FIR arithmetic: the reference's bits (exact) or one fused multiply-add per tap "
                         "(fma, tolerance-tested)")
    ap.add_argument("--batches", type=int, default=2, help="distinct input batches the steps cycle over")
    ap.add_argument("--graph-steps", type=int, default=0,
                    help="steps per replayed HIP graph (0: min(--steps, 100), so the timed window is one or a few "
                         "replays and the host's launch rate never bounds a short step)")
    ap.add_argument("--no-graph", action="store_true", help="launch every step directly")
    ap.add_argument("--stereo-pipeline", type=int, choices=(-1, 0, 1, 2),
                    default=int(os.environ.get("SDR_BENCH_STEREO_PIPE", "-1")),
                    help="stereo configs: 1 = each step as two stages on two contexts' streams (front end + band-pass "
                         "filters | PLL recurrence onwards), step b+1's front overlapping step b's recurrence; 2 = the "
                         "second stream runs the recurrences alone, step b's post stage (NCO, stereo resampler, PCM) "
                         "following step b+1's front stage on the first; 0 = one call per step; -1 (default) = 2 while "
                         "the recurrence's waves fill at most a quarter of the CUs, else 1 (DESIGN.md 5.2)")
    ap.add_argument("--mono-pipeline", type=int, choices=(0, 1),
                    default=int(os.environ.get("SDR_BENCH_MONO_PIPE", "0")),
                    help="mono0: 1 = each step as two stages on two contexts' streams (front end | delay + audio "
                         "filter + PCM), step b+1's front end beside step b's audio stage; 0 = one call per step "
                         "(the default: the pipelined form measured 2-7 %% slower, profiles/r06k/)")
    ap.add_argument("--sustain-seconds", type=float, default=3.0,
                    help="after the timed window, time this many seconds of back-to-back steps (the "
                         "`sustained` field: a receiver runs the block loop continuously); 0 skips it")
    return ap.parse_args(argv)


# --------------------------------------------------------------- planning --
def plan_devices(gpus: int, env: dict, visible: int) -> dict:
    """How this invocation maps onto devices (pure: unit-tested on CPU).

    torch.distributed.run sets WORLD_SIZE: one device per process (LOCAL_RANK),
    gloo for the timing barrier/reduction.  Otherwise one process drives
    `gpus` devices with one host thread each."""
    world = int(env.get("WORLD_SIZE", "1"))
    if world > 1:
        if gpus != world:
            raise SystemExit(f"--gpus {gpus} but WORLD_SIZE {world}: launch with --nproc-per-node {gpus}")
        local = int(env.get("LOCAL_RANK", "0"))
        if env.get("SDR_BENCH_DEVICES"):
            # rehearsal hook for the rank path: rank r runs device list[LOCAL_RANK]
            # (e.g. "0,0": two ranks on a one-GPU box, the real kernels and the
            # gloo barrier; n_gpus then counts ranks)
            devs = [int(x) for x in env["SDR_BENCH_DEVICES"].split(",")]
            if len(devs) != world or any(d < 0 or d >= visible for d in devs):
                raise SystemExit(f"SDR_BENCH_DEVICES={env['SDR_BENCH_DEVICES']} does not name {world} visible devices")
            return {"mode": "ranks", "rank": int(env.get("RANK", "0")), "world": world, "devices": [devs[local]]}
        if local >= visible:
            raise SystemExit(f"LOCAL_RANK {local} but only {visible} device(s) visible")
        return {"mode": "ranks", "rank": int(env.get("RANK", "0")), "world": world, "devices": [local]}
    if gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if env.get("SDR_BENCH_DEVICES"):
        # rehearsal hook: an explicit device list (e.g. "0,0" drives the
        # threaded N = 2 path on a one-GPU box); n_gpus then counts threads
        devs = [int(x) for x in env["SDR_BENCH_DEVICES"].split(",")]
        if len(devs) != gpus or any(d < 0 or d >= visible for d in devs):
            raise SystemExit(f"SDR_BENCH_DEVICES={env['SDR_BENCH_DEVICES']} does not name {gpus} visible devices")
        return {"mode": "threads", "rank": 0, "world": 1, "devices": devs}
    if gpus > visible:
        raise SystemExit(f"--gpus {gpus} but only {visible} device(s) visible")
    return {"mode": "threads", "rank": 0, "world": 1, "devices": list(range(gpus))}


def aggregate(per_device_ms: list, units_per_device: int, steps: int) -> dict:
    """Whole-job throughput over a common start: all devices' units / the
    slowest device's elapsed time (pure: unit-tested on CPU)."""
    ms = max(per_device_ms)
    total = units_per_device * steps * len(per_device_ms)
    return {"ms": ms, "ms_per_step": ms / steps, "value": total / (ms * 1e-3) / 1e6,
            "per_gpu_value": [units_per_device * steps / (m * 1e-3) / 1e6 for m in per_device_ms]}


# ----------------------------------------------------------- CPU baseline --
# per config: the reference code the CPU baseline times (oracle/cpu_bench.cpp) and its block
CPU_KERNELS = {
    "cfg2": ("frontend", 65540), "cfg2u8": ("frontend", 65540), "cfg4": ("frontend", 262150),
    "cfg4x8": ("frontend", 262150),
    # the resampler on the bench's 65,600-sample blocks (src/filter.cpp:142-173)
    "cfg3": ("resample", 65600),
    # the 1024-tap block FIR on I and Q (src/filter.cpp:66-83); a 131,072-sample block keeps one
    # block of the sample within the time budget -- the rate per pair does not depend on it
    "cfg5": ("fir1024", 131072), "cfg5h": ("fir1024", 131072), "cfg5b": ("fir1024", 131072),
    "cfg5hb": ("fir1024", 131072),
    # the reference PROGRAM (src/project.cpp, mode 0), u8 IQ on stdin -> s16 PCM on stdout
    "mono0": ("program", "mono"), "stereo0": ("program", "stereo"), "stereo0w": ("program", "stereo"),
}


def _host_model() -> str:
    try:
        with open("/proc/cpuinfo") as f:
            for line in f:
                if line.startswith("model name"):
                    return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(seconds: float, config: str):
    """The reference's own code timed on this host's cores by
    the native timer oracle/cpu_bench.cpp, for THIS config's workload:
    (i) the config's kernel -- the mode-0 front end (cfg2/cfg2u8/cfg4/cfg4x8),
    the 147/800 resampler (cfg3), the 1024-tap block FIR on I and Q
    (cfg5/cfg5h) -- on 1 thread and on every core of the process's CPU share
    (the affinity set capped by the cgroup CPU quota and OMP_NUM_THREADS: a
    GPU box grants 16 of its 256 cores), one independent stream per
    std::thread; or, for the program configs (mono0, stereo0, stereo0w), the
    reference program `project 0 mono|stereo` as 1 process and as one process
    per core; (ii) for the front-end configs also BASELINE config 1 -- the
    reference program `project 0 mono` on 51,200-pair blocks.  The reference
    build (oracle/_ref, kind 'reference') when present, else the C
    restatement (kind 'port', kernels only)."""
    ref = os.path.join(REPO, "oracle", "_ref", "cpu_bench")
    port = os.path.join(REPO, "oracle", "cpu_bench_port")
    exe, kind = (ref, "reference") if os.path.exists(ref) else (port, "port")
    if not os.path.exists(exe) or config not in CPU_KERNELS:
        return None
    kernel, block = CPU_KERNELS[config]
    proj = os.path.join(REPO, "oracle", "_ref", "project_ref")
    model = _host_model()

    def run(*a):
        out = subprocess.run([exe, *map(str, a)], capture_output=True, text=True, check=True, timeout=600).stdout
        return json.loads(out)

    rate = lambda d: d["pairs"] / d["seconds"] / 1e6  # noqa: E731

    def program(channel, budget):
        """The reference program: ~budget/2 s as one process, then one process per core."""
        p1 = run("program", proj, 300, 1, channel)
        per_block = max(p1["seconds"], 1e-3) / 300
        b1 = max(50, int(budget / 2 / per_block))
        if b1 > 300:
            p1 = run("program", proj, b1, 1, channel)
        pn = run("program", proj, max(50, int(b1 * 0.5)), 0, channel)
        return p1, pn

    if kernel == "program":
        if kind != "reference" or not os.path.exists(proj):
            return None
        p1, pn = program(block, seconds)
        bpb = {"mono": 1024 * 2, "stereo": 1024 * 4}[block]  # PCM bytes per 51,200-pair block, mode 0
        return {"value": round(rate(pn), 2), "unit": "MS/s", "cores": pn["procs"], "kind": kind,
                "value_1core": round(rate(p1), 2),
                "sample": f"the reference program `project 0 {block}` (src/project.cpp), u8 IQ on stdin in "
                          f"51,200-pair blocks -> s16 PCM on stdout, wall clock: {p1['pairs']} IQ pairs in one "
                          f"process, {pn['pairs']} in {pn['procs']} concurrent processes (one per CPU of the share); "
                          f"host {model}",
                "pcm_ok": p1["pcm_bytes"] == p1["pairs"] // 51200 * bpb and pn["pcm_bytes"] == pn["pairs"] // 51200 * bpb}

    cores = int(subprocess.run([exe, "cores"], capture_output=True, text=True, check=True).stdout)
    one = run(kernel, block, seconds / 4, 1)
    share = run(kernel, block, seconds / 4, 0)
    # SURVEY 8(d) asks for all host cores: one thread per CPU of the affinity
    # set, even where the cgroup quota grants fewer (they then time-share)
    many = run(kernel, block, seconds / 4, share["affinity"]) if share["affinity"] > share["threads"] else share
    # the headline is the faster of the two all-core runs: on a box whose
    # cgroup quota grants fewer CPUs than its affinity set, one thread per
    # affinity CPU time-shares the quota and runs slower than the share
    best = many if rate(many) >= rate(share) else share
    what = {"frontend": f"{block:,}-pair mode-0 blocks (101-tap FIR+dec10 on I and Q, then the discriminator: "
                        f"src/project.cpp:86-90)",
            "resample": f"{block:,}-sample blocks through resampleBlockConvolveFIR 147/800, 151 taps per phase "
                        f"(src/filter.cpp:142-173); unit = input samples",
            "fir1024": f"{block:,}-sample blocks of I and Q through blockConvolveFIR with the 1024-tap LPF "
                       f"(src/filter.cpp:66-83); unit = IQ pairs"}[kernel]
    res = {"value": round(rate(best), 2), "unit": "MS/s", "cores": best["threads"], "kind": kind,
           "value_1core": round(rate(one), 2), "value_share": round(rate(share), 2),
           "value_affinity": round(rate(many), 2), "threads_affinity": many["threads"],
           "sample": f"{one['pairs'] + share['pairs'] + (many['pairs'] if many is not share else 0)} units in "
                     f"{what}, one independent stream per std::thread: {many['threads']} threads "
                     f"(every CPU of the affinity set) for {seconds / 4:.0f} s, {share['threads']} threads (the "
                     f"CPU share: affinity capped by the cgroup quota) for {seconds / 4:.0f} s and 1 thread for "
                     f"{seconds / 4:.0f} s (at least one block each); host {model}",
           "cpu_share": {"cores": share["threads"], "affinity": share["affinity"],
                         "cgroup_quota": share["cgroup_quota"] or None,
                         "omp_num_threads": share["omp_num_threads"] or None}}
    if kernel == "frontend" and kind == "reference" and os.path.exists(proj):
        # config 1: ~1 s of the single-process program, then one process per core
        p1 = run("program", proj, 1500, 1, "mono")
        blocks = max(50, int(1500 * min(1.0, (seconds / 4) / max(p1["seconds"], 1e-3))))
        pn = run("program", proj, blocks, 0, "mono")
        res["cfg1"] = {
            "workload": "BASELINE config 1: the reference program `project 0 mono` (src/project.cpp), u8 IQ on "
                        "stdin in 51,200-pair blocks -> s16 PCM on stdout, wall clock",
            "value_1proc": round(rate(p1), 2), "value": round(rate(pn), 2), "unit": "MS/s",
            "procs": pn["procs"], "blocks_per_proc": [1500, blocks],
            "pcm_ok": p1["pcm_bytes"] == 1500 * 1024 * 2 and pn["pcm_bytes"] == pn["procs"] * blocks * 1024 * 2}
    return res


# ------------------------------------------------------------ device jobs --
class Job:
    """One device's share of the workload: its sdr context, HIP stream,
    resident synthetic inputs and the step launcher."""

    def __init__(self, cfg_name: str, device: int, seed: int, args):
        import torch

        import sdrhip

        self.torch, self.sdrhip = torch, sdrhip
        cfg = CONFIGS[cfg_name]
        self.cfg = cfg
        torch.cuda.set_device(device)
        dev = self.dev = torch.device("cuda", device)
        ctx = self.ctx = sdrhip.Context(device)
        # one dedicated (non-null) HIP stream shared by torch and the library, so
        # events bracket exactly the kernels we launch and the stream can be captured
        self.stream = torch.cuda.Stream(dev)
        torch.cuda.set_stream(self.stream)
        ctx.set_stream(self.stream.cuda_stream)
        ctx.set_arith(sdrhip.ARITH_FMA if args.arith == "fma" else sdrhip.ARITH_EXACT)
        self.args = args
        S, n, T = cfg["streams"], cfg["n"], cfg["ntaps"]
        kind = self.kind = cfg["kind"]
        nb = max(1, args.batches)
        # taps: the product's coefficient design (C ABI sdr_taps_lpf, bit-identical
        # to the reference's impulseResponseLPF); setup, not timed
        if kind == "resample":
            taps = sdrhip.taps_lpf(240e3 * 147, 16e3, T, 147)
        else:
            taps = sdrhip.taps_lpf(2.4e6, 100e3, T, 1)
        if kind in ("mono_u8", "stereo_u8"):  # src/project.cpp:263-273: audio LPF (+ BPFs) of mode 0
            d_ha = torch.from_numpy(sdrhip.taps_lpf(240e3, 16e3, 101, 1)).to(dev)
            d_hp = torch.from_numpy(sdrhip.taps_bpf(240e3, 18.5e3, 19.5e3, 101, 1)).to(dev)
            d_hs = torch.from_numpy(sdrhip.taps_bpf(240e3, 22e3, 54e3, 101, 1)).to(dev)
        d_h = self.d_h = torch.from_numpy(taps).to(dev)

        # synthetic input generated on the device (no host traffic), kept resident;
        # nb distinct batches (different seeds)
        iqs = []
        for b in range(nb):
            iq = torch.empty(S * 2 * n, dtype=torch.uint8, device=dev)
            ctx.synth_fm_u8_dev(iq, n, S, 2 * n, seed + 104729 * b)
            iqs.append(iq)
        planar = []
        if kind in ("frontend_f32", "fir_block", "fir_block_f16", "resample"):
            for iq in iqs:
                I = torch.empty(S * n, dtype=torch.float32, device=dev)
                Q = torch.empty(S * n, dtype=torch.float32, device=dev)
                ctx.u8_to_planar_dev(iq, n, S, 2 * n, I, Q, n)
                planar.append((I, Q))
            torch.cuda.synchronize(dev)
            iqs = []
        ns = {"resample": 150, "fir_block": T - 1, "fir_block_f16": T - 1}.get(kind, 100)
        st0 = torch.zeros(S * ns, dtype=torch.float32, device=dev)
        st1 = torch.zeros(S * ns, dtype=torch.float32, device=dev)
        p0 = torch.zeros(S, dtype=torch.float32, device=dev)
        p1 = torch.zeros(S, dtype=torch.float32, device=dev)
        self.keep = [st0, st1, p0, p1, planar, iqs]
        self.tolerance = None
        steps = []

        if kind == "mono_u8":
            D, up, down = cfg["D"], cfg["up"], cfg["down"]
            na = sdrhip.resample_out_len(up, down, n // D)
            sd = torch.zeros(S * 50, dtype=torch.float32, device=dev)
            sa = torch.zeros(S * 100, dtype=torch.float32, device=dev)
            pcm = torch.empty(S * na, dtype=torch.int16, device=dev)
            self.keep += [sd, sa, pcm, d_ha]
            if args.mono_pipeline:
                # the step cut after the front end (sdr_mono_front_u8_dev | sdr_mono_back_dev,
                # disjoint state): front stages on this context's stream, the audio stages on a
                # second context's, two work objects in a ring -- block b+1's front end runs
                # beside block b's audio filter (the stereo pair's scheme)
                ctx2 = self.ctx2 = sdrhip.Context(device)
                self.stream2 = torch.cuda.Stream(dev)
                ctx2.set_stream(self.stream2.cuda_stream)
                nslot = 2
                works = [ctx.mono_work(D, n, up, down, S, 50, d_h, T, ns, d_ha, 101, 100) for _ in range(nslot)]
                ev_f = [sdrhip.Event(ctx) for _ in range(nslot)]
                ev_b = [sdrhip.Event(ctx) for _ in range(nslot)]
                self.keep += [works, ev_f, ev_b]

                def seq(j0, k):
                    """k consecutive steps (see the stereo sequencer)."""
                    for j in range(k):
                        slot = (j0 + j) % nslot
                        if j >= nslot:
                            ev_b[slot].wait(ctx)
                        ctx.mono_front_u8_dev(iqs[(j0 + j) % len(iqs)], 2 * n, d_h, T, st0, st1, ns, p0, p1,
                                              works[slot])
                        ev_f[slot].record(ctx)
                        ev_f[slot].wait(ctx2)
                        ctx2.mono_back_dev(d_ha, 101, sa, 100, sd, works[slot], pcm, na)
                        ev_b[slot].record(ctx2)
                    if k:
                        ev_b[(j0 + k - 1) % nslot].wait(ctx)
                self.seq = seq
            for iq in iqs:
                steps.append(lambda iq=iq: ctx.mono_pcm_u8_dev(D, iq, n, S, 2 * n, d_h, T, st0, st1, ns, p0, p1, sd,
                                                               50, up, down, d_ha, 101, sa, 100, pcm, na))
            self.units = S * n
            self.bytes_per_pair = 2.0 + 2.0 * na / n  # u8 IQ in, s16 PCM out (intermediates are algorithmically free)
            # FIR MACs at 2 FLOP each (front end, audio LPF at the IF rate / 5) + the discriminator
            self.flops_per_unit = 2 * 2 * T / D + 2.0 * 101 / (D * down) + DEMOD_FLOP / D
            self.metric = "IQ MSamples/sec through the mode-0 mono path (u8 IQ -> s16 PCM)"
            self.bound = "valu"
        elif kind == "stereo_u8":
            D, up, down = cfg["D"], cfg["up"], cfg["down"]
            if args.stereo_pipeline < 0:
                # the split schedule moves the post stage onto the front stream: a win while the
                # one-lane-per-stream recurrence leaves the chip mostly idle (stereo0: 16 waves,
                # -3.3 %), a loss once the front stage is as long as the recurrence (stereo0w:
                # 256 waves, +15 %; profiles/r06ae/) -- the stereo call's own fork rule
                cus = torch.cuda.get_device_properties(dev).multi_processor_count
                args.stereo_pipeline = 2 if (S + 63) // 64 <= cus // 4 else 1
            na = sdrhip.resample_out_len(up, down, n // D)
            z = lambda k: torch.zeros(S * k, dtype=torch.float32, device=dev)  # noqa: E731
            sbuf = dict(delay=z(50), audio=z(100), slp=z(100), pilot=z(100), stereo=z(100),
                        pll=torch.tensor([1, 0, 0, 0, 0, 1], dtype=torch.float32, device=dev).repeat(S))
            taps_s = sdrhip.StereoTaps(d_h.data_ptr(), T, d_ha.data_ptr(), 101, d_hp.data_ptr(), d_hs.data_ptr(), 101)
            state_s = sdrhip.StereoState(st0.data_ptr(), st1.data_ptr(), ns, p0.data_ptr(), p1.data_ptr(),
                                         sbuf["delay"].data_ptr(), 50, sbuf["audio"].data_ptr(),
                                         sbuf["slp"].data_ptr(), 100, sbuf["pilot"].data_ptr(),
                                         sbuf["stereo"].data_ptr(), 100, sbuf["pll"].data_ptr())
            pcm = torch.empty(S * 2 * na, dtype=torch.int16, device=dev)
            self.keep += [sbuf, taps_s, state_s, pcm, d_ha, d_hp, d_hs]
            if args.stereo_pipeline:
                # the step cut where the PLL recurrence starts (sdr_stereo_front_u8_dev |
                # sdr_stereo_back_dev, disjoint state): front stages on this context's
                # stream, back stages on a second context's, two work objects in a ring --
                # front(b) waits for back(b-2), back(b) for front(b) (host/sdr_project.cpp)
                ctx2 = self.ctx2 = sdrhip.Context(device)
                self.stream2 = torch.cuda.Stream(dev)
                ctx2.set_stream(self.stream2.cuda_stream)
                nslot = 2
                works = [ctx.stereo_work(D, n, up, down, S) for _ in range(nslot)]
                ev_f = [sdrhip.Event(ctx) for _ in range(nslot)]
                ev_b = [sdrhip.Event(ctx) for _ in range(nslot)]
                self.keep += [works, ev_f, ev_b]

                def seq(j0, k):
                    """k consecutive steps; the first nslot wait on nothing (whatever ran
                    before has completed: a graph replay or a synchronised direct run),
                    and the sequence ends with this stream joined to the last stage."""
                    for j in range(k):
                        slot = (j0 + j) % nslot
                        if j >= nslot:
                            ev_b[slot].wait(ctx)  # the work slot's previous step is done
                        ctx.stereo_front_u8_dev(iqs[(j0 + j) % len(iqs)], 2 * n, taps_s, state_s, works[slot])
                        ev_f[slot].record(ctx)
                        ev_f[slot].wait(ctx2)
                        ctx2.stereo_back_dev(240e3, taps_s, state_s, works[slot], pcm, 2 * na)
                        ev_b[slot].record(ctx2)
                    if k:
                        ev_b[(j0 + k - 1) % nslot].wait(ctx)
                if args.stereo_pipeline == 2:
                    ev_p = [sdrhip.Event(ctx) for _ in range(nslot)]
                    self.keep.append(ev_p)

                    def seq(j0, k):  # noqa: F811
                        """k consecutive steps, the recurrences alone on the second stream:
                        front(b) and then post(b-1) (after recurrence b-1) on this stream,
                        recurrence b (after front b) on the second.  A slot's work is free
                        again when post(b-2) -- earlier on this stream -- has run."""
                        for j in range(k):
                            slot = (j0 + j) % nslot
                            ctx.stereo_front_u8_dev(iqs[(j0 + j) % len(iqs)], 2 * n, taps_s, state_s, works[slot])
                            ev_f[slot].record(ctx)
                            ev_f[slot].wait(ctx2)
                            ctx2.stereo_pll_dev(240e3, state_s, works[slot])
                            ev_p[slot].record(ctx2)
                            if j:
                                prev = (slot - 1) % nslot
                                ev_p[prev].wait(ctx)
                                ctx.stereo_post_dev(taps_s, state_s, works[prev], pcm, 2 * na)
                        if k:
                            last = (j0 + k - 1) % nslot
                            ev_p[last].wait(ctx)
                            ctx.stereo_post_dev(taps_s, state_s, works[last], pcm, 2 * na)
                self.seq = seq
            for iq in iqs:
                steps.append(lambda iq=iq: ctx.stereo_pcm_u8_dev(D, iq, n, S, 2 * n, up, down, 240e3, taps_s,
                                                                 state_s, pcm, 2 * na))
            self.units = S * n
            self.bytes_per_pair = 2.0 + 4.0 * na / n
            # front end + mono and stereo audio LPFs (IF/5 rate) + pilot and stereo BPFs (IF rate)
            self.flops_per_unit = 2 * 2 * T / D + 2 * 2.0 * 101 / (D * down) + 2 * 2.0 * 101 / D + DEMOD_FLOP / D
            self.metric = "IQ MSamples/sec through the mode-0 stereo path (u8 IQ -> interleaved s16 L/R PCM)"
            self.bound = "valu"
        elif kind in ("frontend_f32", "frontend_u8"):
            D = cfg["D"]
            nout = n // D
            out = torch.empty(S * nout, dtype=torch.float32, device=dev)
            self.keep.append(out)
            if kind == "frontend_f32":
                for I, Q in planar:
                    steps.append(lambda I=I, Q=Q: ctx.frontend_dev(D, I, Q, n, S, n, d_h, T, st0, st1, ns, p0, p1,
                                                                   out, nout))
                self.bytes_per_pair = 8.0 + 4.0 / D
            else:
                for iq in iqs:
                    steps.append(lambda iq=iq: ctx.frontend_u8_dev(D, iq, n, S, 2 * n, d_h, T, st0, st1, ns, p0, p1,
                                                                   out, nout))
                self.bytes_per_pair = 2.0 + 4.0 / D
            self.units = S * n  # IQ pairs per step
            # 2 channels x T/D MACs x 2 FLOP, + the discriminator per decimated output
            self.flops_per_unit = 2 * 2 * T / D + DEMOD_FLOP / D
            self.metric = "IQ MSamples/sec through FIR+decimate+FM-demod"
            # f32 planar input: 8.4 B against ~41 FLOP per pair -> HBM-bound; the u8
            # wire format moves 2.4 B per pair, which puts the exact (no-FMA) FIR
            # arithmetic above the ridge -> VALU-bound
            self.bound = "hbm" if kind == "frontend_f32" else "valu"
        elif kind == "resample":
            up, down = cfg["up"], cfg["down"]
            ny = sdrhip.resample_out_len(up, down, n)
            out = torch.empty(S * ny, dtype=torch.float32, device=dev)
            self.keep.append(out)
            # a plan: the tap tables are built once (sdr_resample_plan_create), as a
            # streaming receiver with fixed taps does; one launch per step
            plan = ctx.resample_plan(up, down, d_h, T)
            self.keep.append(plan)
            for I, _ in planar:
                steps.append(lambda I=I: plan.resample_dev(I, n, S, n, st0, ns, out, ny))
            self.units = S * n  # input samples per step
            self.bytes_per_pair = 4.0 + 4.0 * up / down
            self.flops_per_unit = 2.0 * (T / up) * up / down
            self.metric = "IF MSamples/sec (input) through the polyphase resampler"
            # 55.5 FLOP per 4.7 B: above the exact-arithmetic ridge (78.65 TFLOP/s / 8 TB/s)
            self.bound = "valu"
        elif kind == "fir_block":  # I and Q of each block as two channel rows
            nblk = cfg.get("blocks", 1)
            nch = 2 * nblk
            out = torch.empty(nch * n, dtype=torch.float32, device=dev)
            stf = torch.zeros(nch * ns, dtype=torch.float32, device=dev)
            IQs = [self._rows(I, Q, nblk, n) for I, Q in planar]
            self.keep += [out, stf, IQs]
            for IQ in IQs:
                steps.append(lambda IQ=IQ: ctx.fir_block_dev(IQ, n, nch, n, d_h, T, stf, ns, out, n))
            self.units = nblk * n  # IQ pairs per step (I and Q each n samples per block)
            self.bytes_per_pair = 16.0
            self.flops_per_unit = 2.0 * 2 * T
            self.metric = "IQ MSamples/sec through a 1024-tap FIR"
            self.bound = "valu"
        else:  # fir_block_f16: fp16 storage of I and Q (converted once, untimed)
            nblk = cfg.get("blocks", 1)
            nch = 2 * nblk
            IQhs = []
            for I, Q in planar:
                IQ = self._rows(I, Q, nblk, n)
                IQh = torch.empty(nch * n, dtype=torch.float16, device=dev)
                ctx.f32_to_f16_dev(IQ, nch * n, IQh)
                IQhs.append(IQh)
            sth = torch.zeros(nch * ns, dtype=torch.float16, device=dev)
            out = torch.empty(nch * n, dtype=torch.float32, device=dev)
            # a tap plan: the MFMA kernel's fp16 tap copies built once (sdr_fir_f16_plan_create), as a
            # streaming caller with fixed taps would; bitwise the per-call path's outputs (tests)
            fplan = ctx.fir_f16_plan(d_h, T)
            self.keep += [IQhs, sth, out, fplan]
            if os.environ.get("SDR_BENCH_F16_PLAN", "1") != "0":
                for IQh in IQhs:
                    steps.append(lambda IQh=IQh: fplan.fir_block_f16_dev(IQh, n, nch, n, sth, ns, out, n))
            else:  # A/B: the tap copies built in every workgroup of every call
                for IQh in IQhs:
                    steps.append(lambda IQh=IQh: ctx.fir_block_f16_dev(IQh, n, nch, n, d_h, T, sth, ns, out, n))
            self.units = nblk * n
            self.bytes_per_pair = 2.0 * 2 + 8.0  # fp16 in, fp32 out
            self.flops_per_unit = 2.0 * 2 * T
            self.metric = "IQ MSamples/sec through a 1024-tap FIR"
            self.bound = "valu"
            self.f16_kernel = "mfma" if sdrhip.lib().sdr_fir_block_f16_kernel(T) else "dot2"
            # error of this arm against the exact fp32 path (src/filter.cpp:66-83) on the bench's own
            # first block, and the sweep over input amplitudes x tap counts (untimed setup)
            I, Q = planar[0]
            self.tolerance = f16_error(ctx, torch, dev, sdrhip, torch.stack([I[:n], Q[:n]]), n, T)
            if not args.no_f16_sweep:
                self.tolerance["sweep"] = f16_sweep(ctx, torch, dev, sdrhip, torch.stack([I[:n], Q[:n]]), n)
        self.steps = steps
        self.graph = None
        torch.cuda.synchronize(dev)

    def _rows(self, I, Q, nblk, n):
        """[2 * nblk][n] channel rows: block b's I then Q (stream b of the synthetic batch)."""
        return self.torch.stack([I.view(-1, n)[:nblk], Q.view(-1, n)[:nblk]], dim=1).reshape(2 * nblk, n).contiguous()

    # -- launching
    def launch(self, k: int):
        """Enqueue k steps (cycling over the input batches); graphs when captured."""
        i = 0
        if self.graph is not None:
            g, gs = self.graph
            while k - i >= gs:
                g.launch()
                i += gs
        if self.seq is not None:
            self.seq(self._next + i, k - i)
        else:
            for j in range(i, k):
                self.steps[(self._next + j) % len(self.steps)]()
        self._next = (self._next + k) % len(self.steps)

    _next = 0
    seq = None  # a step sequencer (two-stage stereo pipeline) instead of one call per step
    ctx2 = None

    def capture(self, gs: int):
        """Record gs consecutive steps into a HIP graph (gs a multiple of the batch
        count keeps the batch rotation aligned across replays)."""
        if self.graph is not None:
            self.graph[0].close()
        nb = len(self.steps)
        gs = max(nb, gs - gs % nb)
        self._next = 0
        if self.seq is not None:
            self.graph = (self.ctx.capture(lambda: self.seq(0, gs)), gs)
            # the back stage's context: its scratch must not grow under the graph
            self.ctx2.pin_scratch(True)
        else:
            self.graph = (self.ctx.capture(lambda: [self.steps[j % nb]() for j in range(gs)]), gs)

    def warm(self, warmup: int, seconds: float):
        """W warmup steps, then more of the same launches until >= seconds of
        wall time has passed: an idle MI355X sits at ~0.1 GHz and its clock
        ramps over tens of ms; a few warmup steps (<1 ms) would time part of
        the ramp, not the sustained rate a streaming receiver runs at."""
        torch = self.torch
        self.launch(warmup)
        torch.cuda.synchronize(self.dev)
        t = time.perf_counter()
        burst = self.graph[1] if self.graph is not None else 10
        while time.perf_counter() - t < seconds:
            self.launch(burst)
            torch.cuda.synchronize(self.dev)

    def timed(self, k: int, barrier=None):
        """Exactly k steps between HIP events on this device's stream; returns (ms_events, wall_s)."""
        torch = self.torch
        torch.cuda.synchronize(self.dev)
        if barrier is not None:
            barrier()
        e0 = torch.cuda.Event(enable_timing=True)
        e1 = torch.cuda.Event(enable_timing=True)
        t = time.perf_counter()
        e0.record(self.stream)
        self.launch(k)
        e1.record(self.stream)
        torch.cuda.synchronize(self.dev)
        wall = time.perf_counter() - t
        if barrier is not None:
            barrier()
        return e0.elapsed_time(e1), wall

    def sustained(self, seconds: float, ms_per_step: float, barrier=None):
        """Steady state: enough back-to-back steps (whole graph replays) to fill
        `seconds` of device time at the timed window's rate, enqueued at once
        between HIP events.  Returns (ms_events, steps)."""
        gs = self.graph[1] if self.graph is not None else 1
        k = max(gs, int(np.ceil(seconds * 1e3 / max(ms_per_step, 1e-6) / gs)) * gs)
        ms, _ = self.timed(k, barrier)
        return ms, k

    def close(self):
        if self.graph is not None:
            self.graph[0].close()
            self.graph = None
        self.torch.cuda.synchronize(self.dev)
        for k in self.keep:
            for obj in (k if isinstance(k, list) else [k]):
                if hasattr(obj, "close"):
                    obj.close()
        if self.ctx2 is not None:
            self.ctx2.close()
        self.ctx.close()


def f16_error(ctx, torch, dev, sdrhip, IQ, n, T, taps=None):
    """The fp16 arm (fp16 storage, fp32 accumulation) against the exact fp32
    blockConvolveFIR (src/filter.cpp:66-83) on the same two channel rows
    [2][n], zero state: max / rms absolute error and the max normalised by
    sum|h| * max|x|."""
    h = torch.from_numpy(taps if taps is not None else sdrhip.taps_lpf(2.4e6, 100e3, T, 1)).to(dev)
    ns = T - 1
    ref = torch.empty(2 * n, dtype=torch.float32, device=dev)
    ctx.fir_block_dev(IQ, n, 2, n, h, T, torch.zeros(2 * ns, dtype=torch.float32, device=dev), ns, ref, n)
    IQh = torch.empty(2 * n, dtype=torch.float16, device=dev)
    ctx.f32_to_f16_dev(IQ, 2 * n, IQh)
    got = torch.empty(2 * n, dtype=torch.float32, device=dev)
    ctx.fir_block_f16_dev(IQh, n, 2, n, h, T, torch.zeros(2 * ns, dtype=torch.float16, device=dev), ns, got, n)
    torch.cuda.synchronize(dev)
    d = (got.double() - ref.double()).abs()
    err = float(d.max())
    scale = float(h.abs().sum()) * float(IQ.abs().max())
    return {"max_abs_err_vs_fp32_exact": err, "normalized": err / scale, "norm": "sum|h| * max|x|",
            "rms_err": float(d.pow(2).mean().sqrt()), "rms_ref": float(ref.double().pow(2).mean().sqrt())}


def f16_sweep(ctx, torch, dev, sdrhip, IQ, n):
    """BASELINE config 5's fp32-vs-fp16 tolerance sweep: the fp16 arm's error
    against the exact fp32 path for the synthetic I/Q scaled to each amplitude
    in F16_SWEEP_AMPS, through impulseResponseLPF(2.4e6, 100e3, T) for each T
    in F16_SWEEP_TAPS (untimed)."""
    rows = []
    for T in F16_SWEEP_TAPS:
        taps = sdrhip.taps_lpf(2.4e6, 100e3, T, 1)
        for a in F16_SWEEP_AMPS:
            e = f16_error(ctx, torch, dev, sdrhip, (IQ * a).contiguous(), n, T, taps)
            rows.append({"taps": T, "amplitude": a, "max_abs": e["max_abs_err_vs_fp32_exact"],
                         "rms": e["rms_err"], "normalized": e["normalized"],
                         "rms_rel": e["rms_err"] / e["rms_ref"] if e["rms_ref"] else None})
    return rows


def run_device(cfg_name, device, seed, args, barrier=None, side=True):
    """Setup + warmup + the timed region on one device (a host thread or a rank)."""
    job = Job(cfg_name, device, seed, args)
    res = {"device": device}
    try:
        # the first launches run directly: they size the library's scratch
        # (allocations cannot happen inside a capture); then record the graph
        job.launch(args.warmup)
        job.torch.cuda.synchronize(job.dev)
        if not args.no_graph:
            job.capture(args.graph_steps or min(max(args.steps, 1), 100))
        job.warm(0, args.warm_seconds)
        res["ms"], res["wall"] = job.timed(args.steps, barrier)
        if args.sustain_seconds > 0:
            res["sus_ms"], res["sus_steps"] = job.sustained(args.sustain_seconds, res["ms"] / args.steps, barrier)
        # Side measurement (fused front end, exact run only): the same launches
        # under SDR_ARITH_FMA -- one fused multiply-add per tap, not the
        # reference's bits (tolerance-tested); never `value`.
        if side and args.arith == "exact" and job.kind in ("frontend_f32", "frontend_u8") \
                and not args.no_fma_variant:
            job.ctx.set_arith(job.sdrhip.ARITH_FMA)
            job.graph[0].close() if job.graph else None
            job.graph = None
            job.launch(max(args.warmup, 2))
            job.torch.cuda.synchronize(job.dev)
            if not args.no_graph:
                job.capture(args.graph_steps or min(max(args.steps, 1), 100))
            job.warm(0, args.warm_seconds)
            res["fma_ms"], _ = job.timed(args.steps)
            job.ctx.set_arith(job.sdrhip.ARITH_EXACT)
        res["job"] = {k: getattr(job, k, None) for k in ("units", "bytes_per_pair", "flops_per_unit", "metric",
                                                        "bound", "kind", "tolerance", "f16_kernel")}
    finally:
        job.close()
    return res


def roofline(job: dict, ms_per_step: float, config: str, arith: str = "exact") -> dict:
    """Both roofs of the dominant kernel, `frac` against the binding one: the roof
    whose ceiling time (algorithmic bytes / HBM peak, or FLOP / VALU peak) is the
    longer.  The VALU peak is arithmetic-specific: the reference's bits need a
    separately rounded v_mul_f32 and v_add_f32 per multiply-add, one FLOP per lane
    per VALU issue -- half the FMA-counted fp32 peak; the FMA arm gets the FMA peak
    and the fp16 arm's v_dot2_f32_f16 two multiply-adds per issue."""
    launch_s = ms_per_step * 1e-3
    units = job["units"]
    f16_mfma = job["kind"] == "fir_block_f16" and job.get("f16_kernel") == "mfma"
    if f16_mfma:
        vpeak = F16_MFMA_PEAK_TFLOPS
    elif job["kind"] == "fir_block_f16":
        vpeak = FP32_VALU_PEAK_TFLOPS * 2
    elif arith == "fma":
        vpeak = FP32_VALU_PEAK_TFLOPS
    else:
        vpeak = FP32_VALU_PEAK_TFLOPS / 2
    bw = units * job["bytes_per_pair"] / launch_s / 1e9
    fl = units * job["flops_per_unit"] / launch_s / 1e12
    hbm_frac, valu_frac = bw / HBM_PEAK_GBS, fl / vpeak
    t_hbm = units * job["bytes_per_pair"] / (HBM_PEAK_GBS * 1e9)
    t_valu = units * job["flops_per_unit"] / (vpeak * 1e12)
    if t_hbm >= t_valu:
        roof = {"bound": "hbm", "achieved": round(bw, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(hbm_frac, 4)}
    else:
        # the fp16 arm's compute roof is the matrix cores' (dense fp16 MFMA); every
        # other compute-bound line is priced against the VALU issue of its arithmetic
        roof = {"bound": "mfma" if f16_mfma else "valu", "achieved": round(fl, 2), "peak": round(vpeak, 2),
                "unit": "TFLOP/s", "frac": round(valu_frac, 4)}
    roof["hbm_frac"] = round(hbm_frac, 4)
    roof["valu_frac"] = round(valu_frac, 4)
    roof["valu_peak_tflops"] = round(vpeak, 2)
    roof["arith"] = (arith if job["kind"] != "fir_block_f16" else
                     "f16 storage, f32 accumulation on v_mfma_f32_32x32x16_f16 (dense peak)" if f16_mfma else
                     "f16 storage, f32 dot2 accumulation")
    traffic = None
    tpath = os.path.join(REPO, "profiles", f"traffic_{config}.json")
    if os.path.exists(tpath):
        with open(tpath) as f:
            traffic = json.load(f).get("hbm_bytes_per_launch")
        roof["traffic_source"] = os.path.relpath(tpath, REPO)
    roof["traffic"] = traffic
    roof["algorithmic_bytes_per_launch"] = int(units * job["bytes_per_pair"])
    return roof


def main(argv=None):
    args = parse(argv)
    import torch

    plan = plan_devices(args.gpus, os.environ, torch.cuda.device_count())
    cfg = CONFIGS[args.config]
    results = []
    if plan["mode"] == "threads":
        devs = plan["devices"]
        bar = threading.Barrier(len(devs))
        errors = []

        def worker(i, d):
            try:
                results.append(run_device(args.config, d, 1234 + 7919 * i, args,
                                          barrier=bar.wait if len(devs) > 1 else None, side=len(devs) == 1))
            except BaseException as e:  # noqa: BLE001 -- reported below, after every thread ended
                errors.append((d, e))
                bar.abort()

        ths = [threading.Thread(target=worker, args=(i, d)) for i, d in enumerate(devs)]
        for th in ths:
            th.start()
        for th in ths:
            th.join()
        if errors:
            d, e = errors[0]
            raise RuntimeError(f"device {d} failed") from e
        results.sort(key=lambda r: r["device"])  # stable: rehearsal lists may repeat a device
        rank, world = 0, len(devs)
        per_ms = [r["ms"] for r in results]
        sus = [(r.get("sus_ms", 0.0), r.get("sus_steps", 0)) for r in results]
        distinct = len(set(devs))
        wall = max(r["wall"] for r in results)
    else:
        import torch.distributed as dist

        rank, world = plan["rank"], plan["world"]
        # CPU (gloo) group: the timing barrier and max-over-ranks only; the data
        # path has no collective at all
        # gloo's native connect prints "[Gloo] Rank r is connected to ..." on fd 1;
        # stdout carries exactly one JSON line, so fd 1 points at stderr meanwhile
        sys.stdout.flush()
        saved = os.dup(1)
        os.dup2(2, 1)
        try:
            dist.init_process_group("gloo", rank=rank, world_size=world)
        finally:
            os.dup2(saved, 1)
            os.close(saved)
        try:
            r = run_device(args.config, plan["devices"][0], 1234 + 7919 * rank, args, barrier=dist.barrier,
                           side=False)
            t = torch.tensor([r["ms"], r["wall"], r.get("sus_ms", 0.0), r.get("sus_steps", 0)],
                             dtype=torch.float64)
            allt = [torch.zeros(4, dtype=torch.float64) for _ in range(world)]
            dist.all_gather(allt, t)
        finally:
            dist.destroy_process_group()
        results = [r]
        distinct = len(set(int(x) for x in os.environ["SDR_BENCH_DEVICES"].split(","))) \
            if os.environ.get("SDR_BENCH_DEVICES") else world
        per_ms = [float(x[0]) for x in allt]
        wall = max(float(x[1]) for x in allt)
        sus = [(float(x[2]), int(x[3])) for x in allt]

    job = results[0]["job"]
    agg = aggregate(per_ms, job["units"], args.steps)
    roof = roofline(job, agg["ms_per_step"], args.config, args.arith)
    sustained = None
    if args.sustain_seconds > 0 and all(k > 0 for _, k in sus):
        # devices may pick different step counts (each fills the same seconds at its
        # own rate): all devices' units over the slowest device's elapsed time
        sms = max(m for m, _ in sus)
        sval = job["units"] * sum(k for _, k in sus) / (sms * 1e-3) / 1e6
        sstep = max(m / k for m, k in sus)
        sroof = roofline(job, sstep, args.config, args.arith)
        sustained = {"seconds": round(sms * 1e-3, 3), "steps": [k for _, k in sus],
                     "ms_per_step": round(sstep, 5), "value": round(sval, 1),
                     "frac": sroof["frac"], "bound": sroof["bound"], "hbm_frac": sroof["hbm_frac"],
                     "valu_frac": sroof["valu_frac"],
                     "note": "back-to-back steps right after the timed window, one HIP-event pair around all "
                             "of them (steady state of the block loop); reported beside `value`, never as it"}
    fma_variant = None
    if len(results) == 1 and "fma_ms" in results[0]:
        fms = results[0]["fma_ms"] / args.steps
        fval = job["units"] / (fms * 1e-3) / 1e6
        fma_variant = {"arith": "fma (SDR_ARITH_FMA): one fused multiply-add per tap; within the fp32 tolerance, "
                                "not the reference's bits",
                       "value": round(fval, 1), "ms_per_step": round(fms, 4),
                       "roofline_frac": roofline(job, fms, args.config, "fma")["frac"]}
    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        cpu = cpu_baseline(args.cpu_seconds, args.config)
    if rank == 0:
        kind = job["kind"]
        line = {
            "metric": job["metric"], "value": round(agg["value"], 1), "unit": "MS/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(agg["ms_per_step"], 4),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "f16" if kind == "fir_block_f16" else "f32", "data": "synthetic",
            "config": {"workload": cfg["workload"], "streams_per_gpu": cfg["streams"],
                       "pairs_per_stream_per_step": cfg["n"], "ntaps": cfg["ntaps"],
                       "parallelism": f"{world} GPU(s) x independent streams, no data-path collective "
                                      f"({'one host thread per device' if plan['mode'] == 'threads' else 'one process per device, gloo timing barrier'})",
                       "devices_opened": distinct, "input_batches": max(1, args.batches),
                       "launch": "direct" if args.no_graph else
                                 f"HIP graph of {args.graph_steps or min(max(args.steps, 1), 100)} steps",
                       **({"stereo_pipeline": {0: "one call per step",
                                               1: "two stages on two contexts' streams (front | PLL onwards), step "
                                                  "b+1's front overlapping step b's recurrence",
                                               2: "recurrences alone on a second context's stream; step b's post "
                                                  "stage (NCO, stereo resampler, PCM) after step b+1's front stage "
                                                  "on the first"}[args.stereo_pipeline]}
                          if job["kind"] == "stereo_u8" else {}),
                       **({"mono_pipeline": ("two stages on two contexts' streams (front end | delay + audio filter "
                                             "+ PCM), step b+1's front end beside step b's audio stage")
                           if args.mono_pipeline else "one call per step"} if job["kind"] == "mono_u8" else {}),
                       "state_carried_across_steps": True,
                       "arith": ("fma: one fused multiply-add per tap, tolerance-tested (DESIGN.md 2)"
                                 if args.arith == "fma" else "exact: the reference's bits")},
            "per_gpu": {"value": [round(v, 1) for v in agg["per_gpu_value"]],
                        "ms_per_step": [round(m / args.steps, 4) for m in per_ms]},
            "roofline": roof, "cpu_baseline": cpu,
            **({"tolerance": job["tolerance"]} if job["tolerance"] else {}),
            **({"sustained": sustained} if sustained else {}),
            **({"fma_variant": fma_variant} if fma_variant else {}),
            "wall_ms": round(wall * 1e3, 3),
        }
        print(json.dumps(line), flush=True)


if __name__ == "__main__":
    main()
