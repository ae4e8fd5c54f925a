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


# (D, ntaps, ns): the front end's shape, (T-1) % D != 0, and ns > D + T - 1
SHAPES = [(10, 101, 100), (10, 64, 63), (5, 101, 120)]


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
        _work(rank, world, q, dist, Oracle, segment_plan, streams_of, fm_planar)
    except BaseException:
        import traceback

        q.put(("error", rank, traceback.format_exc()))
        raise
    finally:
        dist.destroy_process_group()


def _work(rank, world, q, dist, Oracle, segment_plan, streams_of, fm_planar):
    if True:
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
        # -- one stream, contiguous segments with replicated halos, for
        # shapes with (T-1) % D != 0 and ns > D + T - 1 too
        parts = {}
        for (D, T, ns) in SHAPES:
            hh = o.taps_lpf(2.4e6, 100e3, T, 1)
            N = 1000 * D
            I, Q = fm_planar(N, seed=9)
            seg = segment_plan(N, D, T, ns, world)[rank]

            def before(x, p):  # the ns samples before p (zeros before the stream start)
                out = np.zeros(ns, np.float32)
                lo = max(p - ns, 0)
                if p > lo:
                    out[ns - (p - lo):] = x[lo:p]
                return out

            si, sq = before(I, seg.start), before(Q, seg.start)
            prev = np.zeros(2, np.float32)
            if seg.start:
                # decimated sample just before the segment, recomputed from the halo only
                assert seg.halo_lo == seg.start - D * (-(-ns // D)) and seg.halo_lo % D == 0
                assert seg.read_lo == max(seg.halo_lo - ns, 0)
                Ih = np.zeros(N, np.float32)
                Qh = np.zeros(N, np.float32)
                Ih[seg.read_lo:seg.stop] = I[seg.read_lo:seg.stop]  # what this rank reads
                Qh[seg.read_lo:seg.stop] = Q[seg.read_lo:seg.stop]
                hi = o.fir_decim(D, Ih[seg.halo_lo:seg.start], hh, before(Ih, seg.halo_lo))
                hq = o.fir_decim(D, Qh[seg.halo_lo:seg.start], hh, before(Qh, seg.halo_lo))
                prev[:] = [hi[-1], hq[-1]]
                si, sq = before(Ih, seg.start), before(Qh, seg.start)
            parts[(D, T, ns)] = (seg.start, o.frontend(D, I[seg.start:seg.stop], Q[seg.start:seg.stop], hh, si, sq,
                                                        prev))
        allparts = [None] * world
        dist.all_gather_object(allparts, parts)
        if rank == 0:
            q.put((gathered, allparts))


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
    got = q.get(timeout=120)
    assert got[0] != "error", f"rank {got[1]} failed:\n{got[2]}"
    gathered, parts = got
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
    for (D, T, ns) in SHAPES:
        hh = oracle.taps_lpf(2.4e6, 100e3, T, 1)
        I, Q = fm_planar(1000 * D, seed=9)
        whole = oracle.frontend(D, I, Q, hh, np.zeros(ns, np.float32), np.zeros(ns, np.float32),
                                np.zeros(2, np.float32))
        got = np.concatenate([p for _, p in sorted((d[(D, T, ns)] for d in parts), key=lambda t: t[0])])
        assert_bits(got, whole, f"segmented stream D={D} T={T} ns={ns}")


def test_segment_plan_edges():
    from sdrhip.shard import segment_plan

    segs = segment_plan(65540 * 8, 10, 101, 100, 8)
    assert segs[0].start == 0 and segs[-1].stop == 65540 * 8
    assert all(s.start % 10 == 0 and s.length >= 100 for s in segs)
    assert all(a.stop == b.start for a, b in zip(segs, segs[1:]))
    assert all(s.halo_lo == s.start - 100 and s.read_lo == s.start - 200 for s in segs[1:])
    segs = segment_plan(64000, 10, 64, 63, 4)
    assert all(s.halo_lo % 10 == 0 for s in segs)
    with pytest.raises(ValueError):
        segment_plan(700, 10, 101, 100, 8)  # segments shorter than the state
    with pytest.raises(ValueError):
        segment_plan(1001, 10, 101, 100, 1)
