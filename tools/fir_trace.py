#!/usr/bin/env python3
"""Per-workgroup timeline of the fused front-end kernel (fir_tile) on the
bench's cfg2 launch, from a diagnostic build:

    bash scripts/build_ab_tree.sh trace -DSDR_FIR_TRACE     # ab/trace.so
    SDRHIP_LIB=$PWD/ab/trace.so SDR_FIR_IQ=0 python tools/fir_trace.py [--config cfg2]

Each workgroup of the traced launch records (csrc/fir_tile.hip,
SDR_FIR_TRACE) its hardware slot, the shader clock over its lifetime, s_memtime sums over its tiles of the wait
for a tile's loads, the staging, the scan and the epilogue, its tile count,
and s_memrealtime (100 MHz, chip-wide) at entry and end.  Printed: the phase
durations per tile, and per CU the time-averaged number of resident
workgroups and the idle time between one workgroup's end and the next start.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import sys

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "3dy4-real-time-software-defined-radio-_amd"))


def main():
    import torch  # noqa: F401 -- torch's HIP runtime first, as bench.py loads it

    import bench
    import sdrhip

    cfg = "cfg2"
    if "--config" in sys.argv:
        cfg = sys.argv[sys.argv.index("--config") + 1]
    args = bench.parse(["--config", cfg, "--no-cpu-baseline", "--no-graph"])
    lib = sdrhip.lib()
    fn = lib.sdr_debug_fir_trace
    fn.argtypes = [C.c_void_p, C.c_size_t, C.c_int]
    fn.restype = C.c_int
    job = bench.Job(cfg, 0, 1234, args)
    job.warm(5, 0.3)
    job.torch.cuda.synchronize()
    assert fn(None, 0, 1) == 0
    job.torch.cuda.synchronize()
    job.launch(1)
    job.torch.cuda.synchronize()
    nwg = 1 << 17
    buf = np.zeros(nwg * 10, np.uint64)
    assert fn(buf.ctypes.data, buf.nbytes, 0) == 0
    t = buf.reshape(nwg, 10)
    t = t[t[:, 6] != 0]
    job.close()
    hw = (t[:, 0] & 0xFFFFFFFF).astype(np.int64)
    xcc = (t[:, 0] >> 32).astype(np.int64)
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    simd = (hw >> 4) & 3
    key = ((xcc * 8 + se) * 2 + sh) * 16 + cu
    sums = t[:, 2:6].astype(np.int64)
    ntile = t[:, 6].astype(np.int64)
    r0, r1 = t[:, 1].astype(np.int64), t[:, 7].astype(np.int64)
    per = sums / ntile[:, None]
    ph = {"load wait (tile top -> loads landed)": per[:, 0], "stage (-> LDS staged)": per[:, 1],
          "scan": per[:, 2], "epilogue (demod, stores, state)": per[:, 3], "per tile": per.sum(1),
          "workgroup lifetime (realtime us)": (r1 - r0) / 100.0}
    # shader clock inside the kernel: s_memtime ticks per realtime tick (100 MHz)
    m0, m1 = t[:, 8].astype(np.int64), t[:, 9].astype(np.int64)
    ok = r1 > r0
    clock_mhz = (m1 - m0)[ok] / (r1 - r0)[ok] * 100.0
    out = {"config": cfg, "env": {k: v for k, v in os.environ.items() if k.startswith("SDR_")},
           "workgroups": int(len(t)), "tiles": int(ntile.sum()), "cus_seen": int(len(np.unique(key))),
           "phases_shader_ticks_per_tile": {k: {"p10": round(float(np.percentile(v, 10)), 1),
                                                "median": round(float(np.median(v)), 1),
                                                "mean": round(float(v.mean()), 1),
                                                "p90": round(float(np.percentile(v, 90)), 1)}
                                            for k, v in ph.items()}}
    out["shader_clock_mhz"] = {"median": round(float(np.median(clock_mhz)), 1),
                               "p10": round(float(np.percentile(clock_mhz, 10)), 1),
                               "p90": round(float(np.percentile(clock_mhz, 90)), 1)}
    # realtime (10 ns ticks): the kernel window and per-CU residency
    t0, t1 = r0.min(), r1.max()
    span = t1 - t0
    out["kernel_span_us_realtime"] = span / 100.0
    lo, hi = t0 + span * 0.1, t1 - span * 0.1  # steady state: the middle 80 %
    occ, idle = [], []
    for k in np.unique(key):
        sel = key == k
        a, b = r0[sel], r1[sel]
        # time-averaged resident workgroups within [lo, hi]
        ov = np.clip(np.minimum(b, hi) - np.maximum(a, lo), 0, None).sum()
        occ.append(ov / (hi - lo))
        # idle gaps: at each end, how long until the next start on this CU
        ends, starts = np.sort(b), np.sort(a)
        j = np.searchsorted(starts, ends)
        nxt = starts[np.minimum(j, len(starts) - 1)]
        g = (nxt - ends)[(j < len(starts)) & (ends > lo) & (ends < hi)]
        idle.extend(g.tolist())
    occ = np.array(occ)
    idle = np.array(idle) if idle else np.zeros(1)
    out["resident_wg_per_cu_steady"] = {"mean": round(float(occ.mean()), 2), "p10": round(float(np.percentile(occ, 10)), 2),
                                        "p90": round(float(np.percentile(occ, 90)), 2)}
    out["end_to_next_start_us"] = {"median": float(np.median(idle)) / 100, "p90": float(np.percentile(idle, 90)) / 100}
    out["wg_per_cu"] = {"mean": float(len(t) / len(np.unique(key)))}
    out["simd_share"] = np.bincount(simd, minlength=4).tolist()
    # a time series of chip-wide resident workgroups (20 bins)
    bins = np.linspace(t0, t1, 21)
    series = []
    for i in range(20):
        a0, a1 = bins[i], bins[i + 1]
        series.append(round(float(np.clip(np.minimum(r1, a1) - np.maximum(r0, a0), 0, None).sum() / (a1 - a0)
                                  / len(np.unique(key))), 2))
    out["resident_per_cu_series"] = series
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
