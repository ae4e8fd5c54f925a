"""The N>1 path on CPU (gloo, world_size 2): each rank runs its share of the
work with the oracle as the per-rank compute (stand-in for its GPU), and the
gathered result must equal the single-process result bit for bit.  Covers
both split modes of sdrhip.shard: independent streams (the benchmark) and
one long stream cut into segments with replicated halos.  No collective
sits on the data path: the all_gather here is only the test's check."""
import os
import socket

import numpy as np
import pytest

from conftest import ORACLE_DIR, PKG, assert_bits


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys

    import torch.distributed as dist

    sys.path[:0] = [PKG, ORACLE_DIR]
    from oracle import Oracle
    from sdrhip.shard import segment_plan, streams_of
    from sdrhip.synth import fm_planar

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        o = Oracle()
        h = o.taps_lpf(2.4e6, 100e3, 101, 1)
        # -- independent streams, round robin
        nstreams, n = 5, 5120
        mine = streams_of(rank, nstreams, world)
        local = {}
        for s in mine:
            I, Q = fm_planar(n, seed=100 + s)
            local[s] = o.frontend(10, I, Q, h, np.zeros(100, np.float32), np.zeros(100, np.float32),
                                  np.zeros(2, np.float32))
        gathered = [None] * world
        dist.all_gather_object(gathered, local)
        # -- one stream, contiguous segments with replicated halos
        N = 51200
        I, Q = fm_planar(N, seed=9)
        seg = segment_plan(N, 10, 101, 100, world)[rank]
        si = np.zeros(100, np.float32) if seg.start == 0 else I[seg.start - 100:seg.start].copy()
        sq = np.zeros(100, np.float32) if seg.start == 0 else Q[seg.start - 100:seg.start].copy()
        prev = np.zeros(2, np.float32)
        if seg.start:
            # decimated sample just before the segment, from the halo
            m = seg.start // 10 - 1
            hi = o.fir_decim(10, I[seg.halo_lo:seg.start], h,
                             np.ascontiguousarray(I[seg.halo_lo - 100:seg.halo_lo]) if seg.halo_lo >= 100
                             else np.zeros(100, np.float32))
            hq = o.fir_decim(10, Q[seg.halo_lo:seg.start], h,
                             np.ascontiguousarray(Q[seg.halo_lo - 100:seg.halo_lo]) if seg.halo_lo >= 100
                             else np.zeros(100, np.float32))
            assert (seg.start - seg.halo_lo) % 10 == 0 and m >= 0
            prev[:] = [hi[-1], hq[-1]]
        part = o.frontend(10, I[seg.start:seg.stop], Q[seg.start:seg.stop], h, si, sq, prev)
        parts = [None] * world
        dist.all_gather_object(parts, (seg.start, part))
        if rank == 0:
            q.put((gathered, parts))
    finally:
        dist.destroy_process_group()


def test_sharded_equals_single_process(oracle):
    import torch.multiprocessing as mp

    from sdrhip.shard import stream_ranks
    from sdrhip.synth import fm_planar

    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, parts = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    # independent streams
    assert sorted(k for d in gathered for k in d) == list(range(5))
    assert stream_ranks(5, 2) == [[0, 2, 4], [1, 3]]
    h = oracle.taps_lpf(2.4e6, 100e3, 101, 1)
    for d in gathered:
        for s, got in d.items():
            I, Q = fm_planar(5120, seed=100 + s)
            want = oracle.frontend(10, I, Q, h, np.zeros(100, np.float32), np.zeros(100, np.float32),
                                   np.zeros(2, np.float32))
            assert_bits(got, want, f"stream {s}")
    # one long stream, segmented with halos == unsegmented, bitwise
    I, Q = fm_planar(51200, seed=9)
    whole = oracle.frontend(10, I, Q, h, np.zeros(100, np.float32), np.zeros(100, np.float32),
                            np.zeros(2, np.float32))
    got = np.concatenate([p for _, p in sorted(parts, key=lambda t: t[0])])
    assert_bits(got, whole, "segmented stream")


def test_segment_plan_edges():
    from sdrhip.shard import segment_plan

    segs = segment_plan(65540 * 8, 10, 101, 100, 8)
    assert segs[0].start == 0 and segs[-1].stop == 65540 * 8
    assert all(s.start % 10 == 0 and s.length >= 100 for s in segs)
    assert all(a.stop == b.start for a, b in zip(segs, segs[1:]))
    with pytest.raises(ValueError):
        segment_plan(700, 10, 101, 100, 8)  # segments shorter than the state
    with pytest.raises(ValueError):
        segment_plan(1001, 10, 101, 100, 1)
