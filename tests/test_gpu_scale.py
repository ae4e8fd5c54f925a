"""Bench-scale parity of the device pipelines, and the library under
concurrent host threads.

* The mono and stereo programs (sdr_mono_pcm_u8_dev / sdr_stereo_pcm_u8_dev,
  src/project.cpp:72-133 + 304-314) at the stream counts bench.py runs them
  (mono0 / stereo0: 1,024 streams; stereo0w: 16,384 -- here 4,160, already
  past the 4,096 streams where the stereo call stops forking its side
  branch), two consecutive blocks, every stream's PCM bytes and every carried
  state word (the PLL's six floats included) against the oracle chain, which
  tests/test_dropin.py pins to the reference program's own output.  Both
  launch orders of the stereo call are run: forked (side branch on a second
  HIP stream) and serial, chosen automatically and forced per context.
* Two host threads, each with its own context on the same GPU, running the
  bench's launch pattern (direct calls and a captured HIP graph replayed)
  at the same time; and two threads inside the filter.h drop-in at once
  (src/project.cpp:299-302 calls it from two threads per block).  Every
  output bitwise against the oracle.
"""
from __future__ import annotations

import concurrent.futures as cf
import subprocess
import threading

import numpy as np
import pytest

from conftest import assert_bits
from test_dropin import _mono_setup, _stereo_setup, _stereo_state0

pytestmark = pytest.mark.gpu

WORKERS = 16  # the GPU box's CPU share (os.cpu_count() there reports the whole machine)


def _pmap(fn, items):
    """The oracle is C behind ctypes (the GIL is released inside each call)."""
    with cf.ThreadPoolExecutor(WORKERS) as ex:
        return list(ex.map(fn, items))


def _synth_blocks(gpu_ctx, sdrhip, nstreams, npairs, nblk, seed):
    """nblk device-synthesised u8 IQ blocks [nstreams][2*npairs], also on the host."""
    A = sdrhip.DeviceArray
    out = []
    for b in range(nblk):
        d = A(gpu_ctx, nstreams * 2 * npairs)
        gpu_ctx.synth_fm_u8_dev(d, npairs, nstreams, 2 * npairs, seed=seed + 1000 * b)
        gpu_ctx.synchronize()
        out.append((d, d.download(np.uint8).reshape(nstreams, 2 * npairs)))
    return out


@pytest.mark.parametrize("nstreams,fork", [(1024, "auto"), (1024, "serial"), (4160, "auto"), (4160, "side")])
def test_stereo_pipeline_bench_scale(gpu_ctx, oracle, built_lib, nstreams, fork):
    """stereo0's shape (mode 0, 51,200-pair blocks): 1,024 streams fork the
    side branch by default, 4,160 run serially by default; each is also
    forced the other way.  Two blocks; all PCM and all state bitwise."""
    sdrhip = built_lib
    mode = 0
    rf_fs, D, audio_fs, up, down, block_bytes, taps = _stereo_setup(oracle, mode)
    npairs = block_bytes // 2
    na = sdrhip.resample_out_len(up, down, npairs // D)
    blocks = _synth_blocks(gpu_ctx, sdrhip, nstreams, npairs, 2, 4242 + nstreams)
    A = sdrhip.DeviceArray
    d_taps = {k: A.from_numpy(gpu_ctx, v) for k, v in taps.items()}
    t = sdrhip.StereoTaps(d_taps["rf"].ptr, 101, d_taps["audio"].ptr, len(taps["audio"]), d_taps["pilot"].ptr,
                          d_taps["stereo"].ptr, 101)
    st0 = _stereo_state0()
    d_st = {k: A.from_numpy(gpu_ctx, np.tile(v, nstreams)) for k, v in st0.items() if k != "prev"}
    d_pi = A.from_numpy(gpu_ctx, np.zeros(nstreams, np.float32))
    d_pq = A.from_numpy(gpu_ctx, np.zeros(nstreams, np.float32))
    state = sdrhip.StereoState(d_st["i"].ptr, d_st["q"].ptr, 100, d_pi.ptr, d_pq.ptr, d_st["delay"].ptr, 50,
                               d_st["audio"].ptr, d_st["stereo_lp"].ptr, 100, d_st["pilot"].ptr, d_st["stereo"].ptr,
                               100, d_st["pll"].ptr)
    pcm_stride = 2 * na + 2
    d_pcm = A(gpu_ctx, nstreams * pcm_stride * 2)
    mode_id = {"auto": sdrhip.FORK_AUTO, "serial": sdrhip.FORK_SERIAL, "side": sdrhip.FORK_SIDE}[fork]
    ost = [_stereo_state0() for _ in range(nstreams)]
    gpu_ctx.set_stereo_fork(mode_id)
    try:
        for b, (d_iq, h_iq) in enumerate(blocks):
            gpu_ctx.stereo_pcm_u8_dev(D, d_iq, npairs, nstreams, 2 * npairs, up, down, audio_fs, t, state, d_pcm,
                                      pcm_stride)
            gpu_ctx.synchronize()
            got = d_pcm.download(np.int16).reshape(nstreams, pcm_stride)[:, :2 * na]
            want = _pmap(lambda s: oracle.stereo(D, h_iq[s], taps["rf"], ost[s], up, down, taps["audio"],
                                                 taps["pilot"], taps["stereo"], audio_fs), range(nstreams))
            bad = [s for s in range(nstreams) if not np.array_equal(got[s], want[s])]
            assert not bad, f"{fork}: PCM of {len(bad)} streams differs in block {b} (first {bad[:8]})"
            for k in ("pll", "pilot", "stereo", "stereo_lp", "audio", "delay", "i", "q"):
                assert_bits(d_st[k].download().reshape(nstreams, -1), np.stack([o[k] for o in ost]),
                            f"{fork} {k} block {b}")
            prev = np.stack([d_pi.download(), d_pq.download()], axis=1)
            assert_bits(prev, np.stack([o["prev"] for o in ost]), f"{fork} prev block {b}")
    finally:
        gpu_ctx.set_stereo_fork(sdrhip.FORK_AUTO)


def test_mono_pipeline_bench_scale(gpu_ctx, oracle, built_lib):
    """mono0's shape: 1,024 streams x 51,200-pair mode-0 blocks, two blocks;
    every stream's PCM and carried state bitwise against the oracle chain."""
    sdrhip = built_lib
    mode, nstreams = 0, 1024
    rf_fs, D, up, down, block_bytes, h_rf, h_audio = _mono_setup(oracle, mode)
    npairs = block_bytes // 2
    na = sdrhip.resample_out_len(up, down, npairs // D)
    blocks = _synth_blocks(gpu_ctx, sdrhip, nstreams, npairs, 2, 777)
    A = sdrhip.DeviceArray
    d_hrf, d_ha = A.from_numpy(gpu_ctx, h_rf), A.from_numpy(gpu_ctx, h_audio)
    z = lambda k: A.from_numpy(gpu_ctx, np.zeros(nstreams * k, np.float32))  # noqa: E731
    si, sq, pi, pq, sd, sa = z(100), z(100), z(1), z(1), z(50), z(100)
    pcm_stride = na + 4
    d_pcm = A(gpu_ctx, nstreams * pcm_stride * 2)
    ost = [dict(i=np.zeros(100, np.float32), q=np.zeros(100, np.float32), prev=np.zeros(2, np.float32),
                delay=np.zeros(50, np.float32), audio=np.zeros(100, np.float32)) for _ in range(nstreams)]
    for b, (d_iq, h_iq) in enumerate(blocks):
        gpu_ctx.mono_pcm_u8_dev(D, d_iq, npairs, nstreams, 2 * npairs, d_hrf, len(h_rf), si, sq, 100, pi, pq, sd, 50,
                                up, down, d_ha, len(h_audio), sa, 100, d_pcm, pcm_stride)
        gpu_ctx.synchronize()
        got = d_pcm.download(np.int16).reshape(nstreams, pcm_stride)[:, :na]
        want = _pmap(lambda s: oracle.mono(D, h_iq[s], h_rf, ost[s]["i"], ost[s]["q"], ost[s]["prev"],
                                           ost[s]["delay"], up, down, h_audio, ost[s]["audio"]), range(nstreams))
        bad = [s for s in range(nstreams) if not np.array_equal(got[s], want[s])]
        assert not bad, f"PCM of {len(bad)} streams differs in block {b} (first {bad[:8]})"
        for k, d in (("i", si), ("q", sq), ("delay", sd), ("audio", sa)):
            assert_bits(d.download().reshape(nstreams, -1), np.stack([o[k] for o in ost]), f"{k} block {b}")
        prev = np.stack([pi.download(), pq.download()], axis=1)
        assert_bits(prev, np.stack([o["prev"] for o in ost]), f"prev block {b}")


def test_two_host_threads_two_contexts(built_lib, oracle):
    """bench.py --gpus N's pattern, twice on one GPU at once: each host thread
    owns a Context(0) (its own HIP stream and scratch) and runs the cfg2 front
    end -- a direct call, two calls captured into a HIP graph and replayed,
    another direct call -- three rounds, all concurrently with the other
    thread.  Outputs and carried state bitwise against the oracle."""
    sdrhip = built_lib
    from sdrhip.synth import fm_planar

    D, n, nstreams, nblk, rounds = 10, 65540, 24, 4, 3
    nout = n // D
    h = oracle.taps_lpf(2.4e6, 100e3, 101, 1)
    inputs, wants = [], []
    for th in range(2):
        I = np.empty((nblk, nstreams, n), np.float32)
        Q = np.empty_like(I)
        for s in range(nstreams):
            i, q = fm_planar(n * nblk, seed=500 + 97 * th + s)
            I[:, s], Q[:, s] = i.reshape(nblk, n), q.reshape(nblk, n)
        inputs.append((I, Q))
        want = np.empty((nblk, nstreams, nout), np.float32)
        states = []
        for s in range(nstreams):
            si, sq, pv = np.zeros(100, np.float32), np.zeros(100, np.float32), np.zeros(2, np.float32)
            for b in range(nblk):
                want[b, s] = oracle.frontend(D, I[b, s], Q[b, s], h, si, sq, pv)
            states.append((si, sq, pv))
        wants.append((want, states))
    errors = []
    barrier = threading.Barrier(2)

    def worker(th):
        try:
            with sdrhip.Context(0) as ctx:
                A = sdrhip.DeviceArray
                I, Q = inputs[th]
                d_I = [A.from_numpy(ctx, I[b]) for b in range(nblk)]
                d_Q = [A.from_numpy(ctx, Q[b]) for b in range(nblk)]
                d_out = [A(ctx, nstreams * nout * 4) for _ in range(nblk)]
                d_h = A.from_numpy(ctx, h)
                d_si, d_sq = A(ctx, nstreams * 400), A(ctx, nstreams * 400)
                d_pi, d_pq = A(ctx, nstreams * 4), A(ctx, nstreams * 4)

                def step(b):
                    ctx.frontend_dev(D, d_I[b], d_Q[b], n, nstreams, n, d_h, 101, d_si, d_sq, 100, d_pi, d_pq,
                                     d_out[b], nout)

                def reset():
                    for d in (d_si, d_sq, d_pi, d_pq):
                        d.fill(0)

                reset()
                step(0)  # sizes the context's scratch before the capture
                ctx.synchronize()
                graph = ctx.capture(lambda: (step(1), step(2)))
                barrier.wait()
                for r in range(rounds):
                    reset()
                    for d in d_out:
                        d.fill(0xFF)
                    step(0)
                    graph.launch()
                    step(3)
                    ctx.synchronize()
                    want, states = wants[th]
                    for b in range(nblk):
                        assert_bits(d_out[b].download().reshape(nstreams, nout), want[b], f"thread {th} round {r} block {b}")
                    assert_bits(d_si.download().reshape(nstreams, 100), np.stack([s[0] for s in states]), "state_i")
                    assert_bits(d_sq.download().reshape(nstreams, 100), np.stack([s[1] for s in states]), "state_q")
                    assert_bits(np.stack([d_pi.download(), d_pq.download()], 1), np.stack([s[2] for s in states]),
                                "prev")
                graph.close()
        except Exception as e:  # noqa: BLE001 -- reported by the main thread
            errors.append(f"thread {th}: {e!r}")
            try:
                barrier.abort()
            except Exception:
                pass

    threads = [threading.Thread(target=worker, args=(th,)) for th in range(2)]
    for t_ in threads:
        t_.start()
    for t_ in threads:
        t_.join(timeout=100)
    assert not any(t_.is_alive() for t_ in threads), "worker thread hung"
    assert not errors, errors


def test_dropin_two_threads_at_once(harness, oracle, tmp_path):
    """Two host threads inside libdy4filter_hip.so concurrently (its context
    pool leases one device context per call), each running its own stream's
    block loop: front end + blockConvolveFIR per block, bitwise against the
    oracle (src/project.cpp:299-302 is the reference's two-thread caller)."""
    from sdrhip.synth import fm_iq_u8

    D, block, nblk = 10, 51200, 8
    h = oracle.taps_lpf(2.4e6, 100e3, 101, 1)
    hb = oracle.taps_bpf(240e3, 18.5e3, 19.5e3, 101, 1)
    iqs = [fm_iq_u8(block * nblk, seed=60 + t) for t in range(2)]
    for t, iq in enumerate(iqs):
        iq.tofile(tmp_path / f"iq{t}")
    h.tofile(tmp_path / "h")
    hb.tofile(tmp_path / "hb")
    args = ["threads", D, tmp_path / "iq0", tmp_path / "iq1", tmp_path / "h", tmp_path / "hb", block, nblk,
            tmp_path / "o0", tmp_path / "o1"]
    r = subprocess.run([harness, *map(str, args)], capture_output=True, text=True, timeout=100)
    assert r.returncode == 0, r.stderr
    for t in range(2):
        got = np.fromfile(tmp_path / f"o{t}", np.float32)
        si, sq, sb, pv = (np.zeros(100, np.float32), np.zeros(100, np.float32), np.zeros(100, np.float32),
                          np.zeros(2, np.float32))
        want = []
        for b in range(nblk):
            I, Q = oracle.u8_to_planar(iqs[t][2 * b * block:2 * (b + 1) * block])
            dm = oracle.frontend(D, I, Q, h, si, sq, pv)
            want += [dm, oracle.fir_block(dm, hb, sb)]
        assert_bits(got, np.concatenate(want), f"thread {t}")


@pytest.mark.parametrize("D,T,ns", [(10, 101, 100), (10, 64, 63), (10, 101, 137)])
def test_long_stream_segments_two_threads(built_lib, oracle, D, T, ns):
    """SURVEY 8(e)'s one-long-stream split on the HIP path: a stream of four
    cfg4 blocks (4 x 262,150 pairs) cut by sdrhip.shard.segment_plan into two
    segments, each run by its own host thread and Context(0) -- the per-GPU
    worker of bench.py --gpus N -- from a replicated halo only: the ns inputs
    before its start as the FIR state, and its prev_I/Q recomputed by one
    FIR+decimate call over [halo_lo, start).  The stitched demod and the last
    segment's final state must equal ONE whole-stream call bit for bit, and
    the oracle (state carry src/filter.cpp:139).  (T-1) % D != 0 at T = 64
    (the generic kernel); T = 101 runs the fused fast path, ns = 137 a state
    longer than T-1 and not a multiple of D."""
    sdrhip = built_lib
    from sdrhip.shard import segment_plan
    from sdrhip.synth import fm_planar

    N = 4 * 262150
    nout = N // D
    h = oracle.taps_lpf(2.4e6, 100e3, T, 1)
    I, Q = fm_planar(N, seed=77 + T + ns)
    rng = np.random.default_rng(ns)
    s0 = rng.uniform(-0.7, 0.7, (2, ns)).astype(np.float32)  # the stream's carried state before it
    p0 = np.array([0.3, -0.4], np.float32)

    def before(x, st, p):
        """the ns inputs before p (the carried state before the stream start)"""
        return np.concatenate([st, x[:p]])[p:p + ns].copy()

    segs = segment_plan(N, D, T, ns, 2)
    res, errors = {}, []

    def worker(seg):
        try:
            with sdrhip.Context(0) as ctx:
                A = sdrhip.DeviceArray
                d_h = A.from_numpy(ctx, h)
                prev = p0.copy()
                if seg.start:
                    # prev_* = the decimated I/Q just before the segment, from the halo
                    # [read_lo, start) only: I and Q as the two streams of one call
                    lo, hl = seg.read_lo, seg.halo_lo
                    xs = np.stack([I[hl:seg.start], Q[hl:seg.start]])
                    st = np.stack([before(I, s0[0], hl), before(Q, s0[1], hl)])
                    assert hl - ns >= lo or lo == 0
                    nh = seg.start - hl
                    d_x, d_st = A.from_numpy(ctx, xs), A.from_numpy(ctx, st)
                    d_y = A(ctx, 2 * (nh // D) * 4)
                    ctx.fir_decim_dev(D, d_x, nh, 2, nh, d_h, T, d_st, ns, d_y, nh // D)
                    ctx.synchronize()
                    prev = d_y.download().reshape(2, nh // D)[:, -1].copy()
                si, sq = before(I, s0[0], seg.start), before(Q, s0[1], seg.start)
                n = seg.length
                d_I, d_Q = A.from_numpy(ctx, I[seg.start:seg.stop]), A.from_numpy(ctx, Q[seg.start:seg.stop])
                d_si, d_sq = A.from_numpy(ctx, si), A.from_numpy(ctx, sq)
                d_pi, d_pq = A.from_numpy(ctx, prev[:1]), A.from_numpy(ctx, prev[1:])
                d_out = A(ctx, (n // D) * 4)
                ctx.frontend_dev(D, d_I, d_Q, n, 1, n, d_h, T, d_si, d_sq, ns, d_pi, d_pq, d_out, n // D)
                ctx.synchronize()
                res[seg.rank] = (d_out.download(), d_si.download(), d_sq.download(),
                                 np.concatenate([d_pi.download(), d_pq.download()]))
        except Exception as e:  # noqa: BLE001 -- reported by the main thread
            errors.append(f"segment {seg.rank}: {e!r}")

    threads = [threading.Thread(target=worker, args=(s,)) for s in segs]
    for t_ in threads:
        t_.start()
    for t_ in threads:
        t_.join(timeout=100)
    assert not any(t_.is_alive() for t_ in threads), "worker thread hung"
    assert not errors, errors
    got = np.concatenate([res[r][0] for r in range(2)])
    assert got.shape == (nout,)
    # one whole-stream call on the device
    with sdrhip.Context(0) as ctx:
        A = sdrhip.DeviceArray
        d_I, d_Q, d_h = A.from_numpy(ctx, I), A.from_numpy(ctx, Q), A.from_numpy(ctx, h)
        d_si, d_sq = A.from_numpy(ctx, s0[0]), A.from_numpy(ctx, s0[1])
        d_pi, d_pq = A.from_numpy(ctx, p0[:1]), A.from_numpy(ctx, p0[1:])
        d_out = A(ctx, nout * 4)
        ctx.frontend_dev(D, d_I, d_Q, N, 1, N, d_h, T, d_si, d_sq, ns, d_pi, d_pq, d_out, nout)
        ctx.synchronize()
        whole = d_out.download()
        wstate = (d_si.download(), d_sq.download(), np.concatenate([d_pi.download(), d_pq.download()]))
    assert_bits(got, whole, "two stitched segments vs one whole-stream call")
    for a, b, what in zip(res[1][1:], wstate, ("state_i", "state_q", "prev")):
        assert_bits(a, b, f"last segment's final {what} vs the whole call")
    si, sq, pv = s0[0].copy(), s0[1].copy(), p0.copy()
    want = oracle.frontend(D, I, Q, h, si, sq, pv)
    assert_bits(got, want, "stitched segments vs the oracle")
    assert_bits(res[1][3], pv, "prev vs the oracle")


@pytest.mark.parametrize("sched", ["back", "split"])
@pytest.mark.parametrize("graph", [False, True])
def test_stereo_two_stage_pipeline(built_lib, oracle, graph, sched):
    """bench.py --stereo-pipeline's schedules (and sdr_project's): each block as
    sdr_stereo_front_u8_dev on one context's stream and the back stage on a
    second context's, two work objects in a ring.
    back (--stereo-pipeline 1): sdr_stereo_back_dev, front(b) waiting for
    back(b-2) and back(b) for front(b) by sdr_ctx_wait_event -- block b+1's
    front overlapping block b's PLL recurrence.
    split (--stereo-pipeline 2): sdr_stereo_pll_dev alone on the second
    stream, block b's sdr_stereo_post_dev on the first after block b+1's
    front stage and block b's recurrence.
    128 streams x 5 mode-0 blocks, direct or captured as one HIP graph
    spanning both streams: every PCM byte and every carried state word
    against the oracle chain."""
    sdrhip = built_lib
    mode, nstreams, nblk = 0, 128, 5
    rf_fs, D, audio_fs, up, down, block_bytes, taps = _stereo_setup(oracle, mode)
    npairs = block_bytes // 2
    na = sdrhip.resample_out_len(up, down, npairs // D)
    with sdrhip.Context(0) as ca, sdrhip.Context(0) as cb:  # each on its own HIP stream
        blocks = _synth_blocks(ca, sdrhip, nstreams, npairs, nblk, 777)
        A = sdrhip.DeviceArray
        d_taps = {k: A.from_numpy(ca, v) for k, v in taps.items()}
        t = sdrhip.StereoTaps(d_taps["rf"].ptr, 101, d_taps["audio"].ptr, len(taps["audio"]), d_taps["pilot"].ptr,
                              d_taps["stereo"].ptr, 101)
        st0 = _stereo_state0()
        d_st = {k: A.from_numpy(ca, np.tile(v, nstreams)) for k, v in st0.items() if k != "prev"}
        d_pi = A.from_numpy(ca, np.zeros(nstreams, np.float32))
        d_pq = A.from_numpy(ca, np.zeros(nstreams, np.float32))
        state = sdrhip.StereoState(d_st["i"].ptr, d_st["q"].ptr, 100, d_pi.ptr, d_pq.ptr, d_st["delay"].ptr, 50,
                                   d_st["audio"].ptr, d_st["stereo_lp"].ptr, 100, d_st["pilot"].ptr,
                                   d_st["stereo"].ptr, 100, d_st["pll"].ptr)
        pcm = [A(ca, nstreams * 2 * na * 2) for _ in range(nblk)]
        ns_ = 2
        works = [ca.stereo_work(D, npairs, up, down, nstreams) for _ in range(ns_)]
        ev_f = [sdrhip.Event(ca) for _ in range(ns_)]
        ev_b = [sdrhip.Event(ca) for _ in range(ns_)]

        def run(b0, k):
            if sched == "split":
                for j in range(k):
                    b, slot = b0 + j, (b0 + j) % ns_
                    ca.stereo_front_u8_dev(blocks[b][0], 2 * npairs, t, state, works[slot])
                    ev_f[slot].record(ca)
                    ev_f[slot].wait(cb)
                    cb.stereo_pll_dev(audio_fs, state, works[slot])
                    ev_b[slot].record(cb)
                    if j:
                        ev_b[(slot - 1) % ns_].wait(ca)
                        ca.stereo_post_dev(t, state, works[(slot - 1) % ns_], pcm[b - 1], 2 * na)
                ev_b[(b0 + k - 1) % ns_].wait(ca)
                ca.stereo_post_dev(t, state, works[(b0 + k - 1) % ns_], pcm[b0 + k - 1], 2 * na)
                return
            for j in range(k):
                b, slot = b0 + j, (b0 + j) % ns_
                if j >= ns_:
                    ev_b[slot].wait(ca)
                ca.stereo_front_u8_dev(blocks[b][0], 2 * npairs, t, state, works[slot])
                ev_f[slot].record(ca)
                ev_f[slot].wait(cb)
                cb.stereo_back_dev(audio_fs, t, state, works[slot], pcm[b], 2 * na)
                ev_b[slot].record(cb)
            ev_b[(b0 + k - 1) % ns_].wait(ca)

        try:
            run(0, 1)  # sizes both contexts' scratch (no allocation may happen inside a capture)
            ca.synchronize()
            if graph:
                g = ca.capture(lambda: run(1, nblk - 1))
                g.launch()
            else:
                run(1, nblk - 1)
            ca.synchronize()
            cb.synchronize()
            if graph:
                g.close()
            ost = [_stereo_state0() for _ in range(nstreams)]
            for b in range(nblk):
                got = pcm[b].download(np.int16).reshape(nstreams, 2 * na)
                want = _pmap(lambda s: oracle.stereo(D, blocks[b][1][s], taps["rf"], ost[s], up, down,
                                                     taps["audio"], taps["pilot"], taps["stereo"], audio_fs),
                             range(nstreams))
                bad = [s for s in range(nstreams) if not np.array_equal(got[s], want[s])]
                assert not bad, f"PCM of {len(bad)} streams differs in block {b} (first {bad[:8]})"
            for k in ("pll", "pilot", "stereo", "stereo_lp", "audio", "delay", "i", "q"):
                assert_bits(d_st[k].download().reshape(nstreams, -1), np.stack([o[k] for o in ost]), k)
            assert_bits(np.stack([d_pi.download(), d_pq.download()], axis=1), np.stack([o["prev"] for o in ost]),
                        "prev")
        finally:
            for w in works:
                w.close()
            for e in ev_f + ev_b:
                e.close()


def _stereo_state_dev(ctx, sdrhip, nstreams):
    A = sdrhip.DeviceArray
    st0 = _stereo_state0()
    d_st = {k: A.from_numpy(ctx, np.tile(v, nstreams)) for k, v in st0.items() if k != "prev"}
    d_pi = A.from_numpy(ctx, np.zeros(nstreams, np.float32))
    d_pq = A.from_numpy(ctx, np.zeros(nstreams, np.float32))
    state = sdrhip.StereoState(d_st["i"].ptr, d_st["q"].ptr, 100, d_pi.ptr, d_pq.ptr, d_st["delay"].ptr, 50,
                               d_st["audio"].ptr, d_st["stereo_lp"].ptr, 100, d_st["pilot"].ptr, d_st["stereo"].ptr,
                               100, d_st["pll"].ptr)
    return state, [d_st, d_pi, d_pq]


def test_stereo_work_destroy_waits_for_other_context(built_lib, oracle):
    """a stereo work created on context A whose back stage is still
    queued on context B is destroyed through A.  sdr_stereo_work_destroy must
    wait for B's stream (it records an event on every stream a stage ran on),
    so the freed buffers -- immediately re-allocated and overwritten on A's
    stream -- are not in use: the PCM equals the one-call path's bit for bit."""
    sdrhip = built_lib
    mode, nstreams = 0, 8192  # a back stage of a few ms: long enough to still be queued at destroy
    rf_fs, D, audio_fs, up, down, block_bytes, taps = _stereo_setup(oracle, mode)
    npairs = block_bytes // 2
    nd = npairs // D
    na = sdrhip.resample_out_len(up, down, nd)
    with sdrhip.Context(0) as ca, sdrhip.Context(0) as cb:
        A = sdrhip.DeviceArray
        (d_iq, _), = _synth_blocks(ca, sdrhip, nstreams, npairs, 1, 99)
        d_taps = {k: A.from_numpy(ca, v) for k, v in taps.items()}
        t = sdrhip.StereoTaps(d_taps["rf"].ptr, 101, d_taps["audio"].ptr, len(taps["audio"]), d_taps["pilot"].ptr,
                              d_taps["stereo"].ptr, 101)
        # reference: the one-call path on a fresh state
        st_ref, keep_ref = _stereo_state_dev(ca, sdrhip, nstreams)
        pcm_ref = A(ca, nstreams * 2 * na * 2)
        ca.stereo_pcm_u8_dev(D, d_iq, npairs, nstreams, 2 * npairs, up, down, audio_fs, t, st_ref, pcm_ref, 2 * na)
        ca.synchronize()
        want = pcm_ref.download(np.int16)
        # the two-stage path, destroyed while B's back stage is queued
        st, keep = _stereo_state_dev(ca, sdrhip, nstreams)
        pcm = A(ca, nstreams * 2 * na * 2)
        pcm.fill(0)
        ev = sdrhip.Event(ca)
        w = ca.stereo_work(D, npairs, up, down, nstreams)
        ca.stereo_front_u8_dev(d_iq, 2 * npairs, t, st, w)
        ev.record(ca)
        ev.wait(cb)
        cb.stereo_back_dev(audio_fs, t, st, w, pcm, 2 * na)
        w.close()  # through A, while B may still be running the back stage
        d4, a4, p4 = (nd + 3) // 4 * 4, (na + 3) // 4 * 4, (nd + 4) // 4 * 4
        junk = A(ca, 4 * nstreams * (5 * d4 + 2 * a4 + p4) + nstreams * nd)
        junk.fill(0xFF)  # NaN patterns over whatever was freed
        ca.synchronize()
        cb.synchronize()
        got = pcm.download(np.int16)
        assert np.array_equal(got, want), "PCM after destroying the work mid-flight differs"
        ev.close()
        junk.free()


def test_resample_plan_destroy_waits_for_other_context(built_lib, oracle):
    """a resampler plan created on context A, its launch queued on
    context B, destroyed through A: destroy waits for B's launch (per-stream
    events) before freeing the tables, which are then re-allocated and
    overwritten; the outputs equal a run whose plan outlived it."""
    sdrhip = built_lib
    up, down, T, S, n, ns = 147, 800, 151 * 147, 1024, 65600, 150
    ny = sdrhip.resample_out_len(up, down, n)
    h = oracle.taps_lpf(240e3 * 147, 16e3, T, 147)
    with sdrhip.Context(0) as ca, sdrhip.Context(0) as cb:
        A = sdrhip.DeviceArray
        d_h = A.from_numpy(ca, h)
        d_x = A(ca, S * n * 4)
        d_iq = A(ca, S * 2 * n)
        ca.synth_fm_u8_dev(d_iq, n, S, 2 * n, seed=5)
        d_q = A(ca, S * n * 4)
        ca.u8_to_planar_dev(d_iq, n, S, 2 * n, d_x, d_q, n)
        ca.synchronize()
        outs = []
        for early in (False, True):
            d_st = A.from_numpy(ca, np.zeros(S * ns, np.float32))
            d_y = A(ca, S * ny * 4)
            plan = ca.resample_plan(up, down, d_h, T)
            for _ in range(3):  # three launches queued on B
                plan_ctx = sdrhip.ResamplePlan(cb, plan._p)
                plan_ctx.resample_dev(d_x, n, S, n, d_st, ns, d_y, ny)
            if early:
                plan.close()  # through A while B's launches may still run
                junk = A(ca, 4 * 4 * 147 * 160 + 4096)
                junk.fill(0xFF)
            cb.synchronize()
            if not early:
                plan.close()
            else:
                junk.free()
            outs.append((d_y.download(), d_st.download()))
        assert_bits(outs[1][0], outs[0][0], "outputs with the plan destroyed mid-flight")
        assert_bits(outs[1][1], outs[0][1], "state with the plan destroyed mid-flight")


def test_pll_fast_vs_library_screen(built_lib):
    """fmPLL's certified short path (SDR_PLL_FAST=1) against its exact-library
    path (libm_exact: glibc's floats) at stereo0w's stream count: 16,384
    streams x 6 blocks of 5,120 pilot samples (5.0e8 PLL steps, state carried),
    every NCO output and state float bitwise equal (tests/pll_screen.py; the
    long screens it prints are in profiles/).  src/filter.cpp:174-228.  A
    child process: the screen's torch must open the device before the
    library does."""
    import json
    import os
    import sys

    script = os.path.join(os.path.dirname(os.path.abspath(__file__)), "pll_screen.py")
    p = subprocess.run([sys.executable, script, "--streams", "16384", "--blocks", "6", "--seed", "7"],
                       capture_output=True, text=True, timeout=200)
    assert p.returncode == 0, p.stderr[-2000:]
    r = json.loads(p.stdout.strip().splitlines()[-1])
    assert r["pll_steps"] == 16384 * 5120 * 6, r
    assert r["output_mismatches"] == 0 and r["state_mismatches"] == 0, r
