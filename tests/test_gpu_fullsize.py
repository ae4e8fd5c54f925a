"""GPU parity at BASELINE.json's full sizes, through the exact launches the
benchmark times (f32 planar `frontend_dev`, state carried across steps):

* config 2: 1,024 streams x 65,540 pairs, two consecutive steps -- EVERY
  stream's outputs against the oracle bit for bit (the oracle threaded over
  streams), and every stream's carried state (state_i/q = the block's last
  100 inputs; prev_i/q = its last decimated I/Q, recomputed in numpy in the
  reference's fp32 order) bit for bit;
* config 2 under SDR_ARITH_FMA: every stream within the SURVEY 8(d) bar of
  the exact path;
* config 4: 262,150-pair blocks (2 consecutive, 3 streams), one stream as a
  single 8,388,800-pair call, the bench's cfg4x8 launch (8 streams x
  8,388,800 pairs in ONE batched call) and the bench's cfg4 launch (one
  stream x 67,110,400 pairs in one call), each against the oracle run block
  by block -- block-size independence, src/filter.cpp:139;
* config 5: the 1024-tap FIR over 2 x 1,048,576 samples, EVERY output
  against the oracle: the first window from the real state, every later
  window seeded with the 1,023 inputs before it (src/filter.cpp:82), the
  windows threaded; its fp16 arm over the whole 2 x 1,048,576 within the
  stated tolerance;
* config 3: the resampler plan at the bench's launch (1,024 x 65,600, the
  real 22,197-tap design), two steps, every stream bitwise.
"""
import concurrent.futures as cf

import numpy as np
import pytest

from conftest import assert_bits, load_golden

pytestmark = pytest.mark.gpu


def _z(k):
    return np.zeros(k, np.float32)


def _dev(sdrhip, ctx, a):
    return sdrhip.DeviceArray.from_numpy(ctx, np.ascontiguousarray(a))


def _last_output(h, x, D):
    """Last decimated output of every row of x (y[nout-1] = sum_k h[k] x[n-D-k]),
    accumulated k = 0..T-1 from 0.0f with separately rounded products and sums
    (numpy float32 ops never fuse) -- src/filter.cpp:131-135."""
    n = x.shape[1]
    acc = np.zeros(x.shape[0], np.float32)
    for k in range(len(h)):
        acc = acc + np.float32(h[k]) * x[:, n - D - k]
    return acc


def _planar_batch(sdrhip, ctx, nstreams, n, seed, stride=None):
    """Device synthetic FM, planar f32 rows of `stride` (>= n, a multiple of 4)."""
    stride = stride or n
    iq_stride = (2 * n + 7) // 8 * 8
    d_iq = sdrhip.DeviceArray(ctx, nstreams * iq_stride)
    ctx.synth_fm_u8_dev(d_iq, n, nstreams, iq_stride, seed=seed)
    d_I = sdrhip.DeviceArray(ctx, nstreams * stride * 4)
    d_Q = sdrhip.DeviceArray(ctx, nstreams * stride * 4)
    ctx.u8_to_planar_dev(d_iq, n, nstreams, iq_stride, d_I, d_Q, stride)
    d_iq.free()
    return d_I, d_Q


@pytest.mark.parametrize("kernel", ["tile", "sc"])
def test_cfg2_full_f32_two_steps(gpu_ctx, oracle, built_lib, kswitch, kernel):
    """kernel: fir_tile, or fir_tile_sc (SDR_FIR_SC=1); the bench's launch
    either way.  All 1,024 streams' outputs and states, both steps."""
    kswitch("SDR_FIR_SC", "0" if kernel == "tile" else "1")
    sdrhip = built_lib
    S, n, D = 1024, 65540, 10
    nout = n // D
    h = load_golden("taps")["lpf_rf_mode0"]
    d_h = _dev(sdrhip, gpu_ctx, h)
    d_si, d_sq = _dev(sdrhip, gpu_ctx, np.zeros((S, 100), np.float32)), _dev(sdrhip, gpu_ctx, np.zeros((S, 100), np.float32))
    d_pi, d_pq = _dev(sdrhip, gpu_ctx, _z(S)), _dev(sdrhip, gpu_ctx, _z(S))
    d_out = sdrhip.DeviceArray(gpu_ctx, S * nout * 4)
    ors = [dict(si=_z(100), sq=_z(100), prev=_z(2)) for _ in range(S)]
    for step, seed in enumerate((301, 302)):
        d_I, d_Q = _planar_batch(sdrhip, gpu_ctx, S, n, seed)
        d_out.fill(0xFF)
        gpu_ctx.frontend_dev(D, d_I, d_Q, n, S, n, d_h, 101, d_si, d_sq, 100, d_pi, d_pq, d_out, nout)
        gpu_ctx.synchronize()
        got = d_out.download().reshape(S, nout)
        I = d_I.download().reshape(S, n)
        Q = d_Q.download().reshape(S, n)
        with cf.ThreadPoolExecutor(16) as ex:  # C behind ctypes: the GIL is released
            want = np.stack(list(ex.map(
                lambda s: oracle.frontend(D, I[s], Q[s], h, ors[s]["si"], ors[s]["sq"], ors[s]["prev"]), range(S))))
        assert_bits(got, want, f"step {step}: all {S} streams")
        # every stream's carried state, against the oracle and against the
        # reference's rule restated in numpy
        assert_bits(d_si.download().reshape(S, 100), np.stack([o["si"] for o in ors]), f"step {step} state_i")
        assert_bits(d_sq.download().reshape(S, 100), np.stack([o["sq"] for o in ors]), f"step {step} state_q")
        assert_bits(d_si.download().reshape(S, 100), I[:, n - 100:], f"step {step} state_i (all streams)")
        assert_bits(d_sq.download().reshape(S, 100), Q[:, n - 100:], f"step {step} state_q (all streams)")
        assert_bits(d_pi.download(), _last_output(h, I, D), f"step {step} prev_i (all streams)")
        assert_bits(d_pq.download(), _last_output(h, Q, D), f"step {step} prev_q (all streams)")
        assert_bits(d_pi.download(), np.array([o["prev"][0] for o in ors], np.float32), f"step {step} prev_i")
        assert_bits(d_pq.download(), np.array([o["prev"][1] for o in ors], np.float32), f"step {step} prev_q")
        assert np.isfinite(got).all()
        d_I.free()
        d_Q.free()


def test_cfg2_full_fma_tolerance(gpu_ctx, built_lib):
    """SDR_ARITH_FMA at full size: every stream's demod within 1e-5 of the exact
    path where the decimated envelope I^2+Q^2 >= 1e-3; state exact."""
    sdrhip = built_lib
    S, n, D = 1024, 65540, 10
    nout = n // D
    h = load_golden("taps")["lpf_rf_mode0"]
    d_h = _dev(sdrhip, gpu_ctx, h)
    d_I, d_Q = _planar_batch(sdrhip, gpu_ctx, S, n, 303)
    outs, states = {}, {}
    for mode in (sdrhip.ARITH_EXACT, sdrhip.ARITH_FMA):
        gpu_ctx.set_arith(mode)
        try:
            d_si, d_sq = _dev(sdrhip, gpu_ctx, np.zeros((S, 100), np.float32)), _dev(sdrhip, gpu_ctx, np.zeros((S, 100), np.float32))
            d_pi, d_pq = _dev(sdrhip, gpu_ctx, _z(S)), _dev(sdrhip, gpu_ctx, _z(S))
            d_out = sdrhip.DeviceArray(gpu_ctx, S * nout * 4)
            gpu_ctx.frontend_dev(D, d_I, d_Q, n, S, n, d_h, 101, d_si, d_sq, 100, d_pi, d_pq, d_out, nout)
            gpu_ctx.synchronize()
        finally:
            gpu_ctx.set_arith(sdrhip.ARITH_EXACT)
        outs[mode] = d_out.download().reshape(S, nout)
        states[mode] = (d_si.download(), d_sq.download(), d_pi.download(), d_pq.download())
    # the decimated I/Q envelope, exact (unfused FIR calls)
    d_yi = sdrhip.DeviceArray(gpu_ctx, S * nout * 4)
    d_yq = sdrhip.DeviceArray(gpu_ctx, S * nout * 4)
    for d_x, d_y in ((d_I, d_yi), (d_Q, d_yq)):
        d_s = _dev(sdrhip, gpu_ctx, np.zeros((S, 100), np.float32))
        gpu_ctx.fir_decim_dev(D, d_x, n, S, n, d_h, 101, d_s, 100, d_y, nout)
    gpu_ctx.synchronize()
    yi = d_yi.download().reshape(S, nout).astype(np.float64)
    yq = d_yq.download().reshape(S, nout).astype(np.float64)
    ok = (yi * yi + yq * yq) >= 1e-3
    diff = np.abs(outs[sdrhip.ARITH_FMA].astype(np.float64) - outs[sdrhip.ARITH_EXACT])
    assert ok.mean() > 0.99
    assert diff[ok].max() <= 1e-5, f"FMA demod off by {diff[ok].max():.3g}"
    assert not np.array_equal(outs[sdrhip.ARITH_FMA], outs[sdrhip.ARITH_EXACT])  # it did run the FMA kernel
    for a, b in zip(states[sdrhip.ARITH_FMA][:2], states[sdrhip.ARITH_EXACT][:2]):
        assert_bits(a, b, "FMA state (raw inputs: exact by construction)")
    bound = 4e-6 * float(np.abs(h).sum()) * 1.0
    for a, b in zip(states[sdrhip.ARITH_FMA][2:], states[sdrhip.ARITH_EXACT][2:]):
        assert np.abs(a.astype(np.float64) - b).max() <= bound


def test_cfg4_blocks_vs_oracle(gpu_ctx, oracle, built_lib):
    """3 streams x 2 consecutive 262,150-pair blocks, batched f32 call, bitwise
    with all carried state."""
    sdrhip = built_lib
    S, n, D = 3, 262150, 10
    nout = n // D
    h = load_golden("taps")["lpf_rf_mode0"]
    d_h = _dev(sdrhip, gpu_ctx, h)
    d_si, d_sq = _dev(sdrhip, gpu_ctx, np.zeros((S, 100), np.float32)), _dev(sdrhip, gpu_ctx, np.zeros((S, 100), np.float32))
    d_pi, d_pq = _dev(sdrhip, gpu_ctx, _z(S)), _dev(sdrhip, gpu_ctx, _z(S))
    d_out = sdrhip.DeviceArray(gpu_ctx, S * nout * 4)
    ors = [dict(si=_z(100), sq=_z(100), prev=_z(2)) for _ in range(S)]
    stride = n + 2  # 262,150 is not a multiple of 4: 16-B aligned rows
    for b, seed in enumerate((41, 42)):
        d_I, d_Q = _planar_batch(sdrhip, gpu_ctx, S, n, seed, stride)
        gpu_ctx.frontend_dev(D, d_I, d_Q, n, S, stride, d_h, 101, d_si, d_sq, 100, d_pi, d_pq, d_out, nout)
        gpu_ctx.synchronize()
        got = d_out.download().reshape(S, nout)
        I, Q = d_I.download().reshape(S, stride)[:, :n], d_Q.download().reshape(S, stride)[:, :n]
        for s in range(S):
            want = oracle.frontend(D, np.ascontiguousarray(I[s]), np.ascontiguousarray(Q[s]), h, ors[s]["si"],
                                   ors[s]["sq"], ors[s]["prev"])
            assert_bits(got[s], want, f"block {b} stream {s}")
        assert_bits(d_si.download().reshape(S, 100), np.stack([o["si"] for o in ors]), "state_i")
        assert_bits(d_sq.download().reshape(S, 100), np.stack([o["sq"] for o in ors]), "state_q")
        assert_bits(d_pi.download(), np.array([o["prev"][0] for o in ors], np.float32), "prev_i")
        assert_bits(d_pq.download(), np.array([o["prev"][1] for o in ors], np.float32), "prev_q")


def test_cfg4_single_call_equals_blocks(gpu_ctx, oracle, built_lib):
    """One stream as ONE 8,388,800-pair call (32 x 262,150) == the oracle run
    block by block over the same samples, outputs and state bitwise."""
    sdrhip = built_lib
    nblk, blk, D = 32, 262150, 10
    n = nblk * blk
    h = load_golden("taps")["lpf_rf_mode0"]
    d_h = _dev(sdrhip, gpu_ctx, h)
    d_I, d_Q = _planar_batch(sdrhip, gpu_ctx, 1, n, 4242)
    st0 = np.random.default_rng(3).uniform(-0.7, 0.7, (2, 100)).astype(np.float32)  # a non-zero carried state
    pv0 = np.array([0.25, -0.5], np.float32)
    d_si, d_sq = _dev(sdrhip, gpu_ctx, st0[0]), _dev(sdrhip, gpu_ctx, st0[1])
    d_pi, d_pq = _dev(sdrhip, gpu_ctx, pv0[:1]), _dev(sdrhip, gpu_ctx, pv0[1:])
    d_out = sdrhip.DeviceArray(gpu_ctx, n // D * 4)
    gpu_ctx.frontend_dev(D, d_I, d_Q, n, 1, n, d_h, 101, d_si, d_sq, 100, d_pi, d_pq, d_out, n // D)
    gpu_ctx.synchronize()
    got = d_out.download()
    I, Q = d_I.download(), d_Q.download()
    si, sq, pv = st0[0].copy(), st0[1].copy(), pv0.copy()
    want = np.concatenate([oracle.frontend(D, I[b * blk:(b + 1) * blk], Q[b * blk:(b + 1) * blk], h, si, sq, pv)
                           for b in range(nblk)])
    assert_bits(got, want, "one call vs 32 oracle blocks")
    assert_bits(d_si.download(), si, "state_i")
    assert_bits(d_sq.download(), sq, "state_q")
    assert_bits(np.concatenate([d_pi.download(), d_pq.download()]), pv, "prev")


def test_cfg4x8_full_call(gpu_ctx, oracle, built_lib):
    """bench.py's cfg4x8 launch exactly: 8 independent streams x 8,388,800
    pairs (32 x 262,150) in ONE batched frontend_dev call, each stream with its
    own non-zero carried state, against the oracle run block by block over the
    same samples (src/filter.cpp:139): every output and every state bitwise."""
    sdrhip = built_lib
    S, nblk, blk, D = 8, 32, 262150, 10
    n = nblk * blk
    nout, nb = n // D, blk // D
    h = load_golden("taps")["lpf_rf_mode0"]
    d_h = _dev(sdrhip, gpu_ctx, h)
    d_I, d_Q = _planar_batch(sdrhip, gpu_ctx, S, n, 4848)
    st0 = np.random.default_rng(8).uniform(-0.7, 0.7, (2, S, 100)).astype(np.float32)
    pv0 = np.random.default_rng(9).uniform(-0.7, 0.7, (2, S)).astype(np.float32)
    d_si, d_sq = _dev(sdrhip, gpu_ctx, st0[0]), _dev(sdrhip, gpu_ctx, st0[1])
    d_pi, d_pq = _dev(sdrhip, gpu_ctx, pv0[0]), _dev(sdrhip, gpu_ctx, pv0[1])
    d_out = sdrhip.DeviceArray(gpu_ctx, S * nout * 4)
    d_out.fill(0xFF)
    gpu_ctx.frontend_dev(D, d_I, d_Q, n, S, n, d_h, 101, d_si, d_sq, 100, d_pi, d_pq, d_out, nout)
    gpu_ctx.synchronize()
    got = d_out.download().reshape(S, nout)
    I, Q = d_I.download().reshape(S, n), d_Q.download().reshape(S, n)
    d_I.free()
    d_Q.free()
    ors = [dict(si=st0[0, s].copy(), sq=st0[1, s].copy(), prev=np.array([pv0[0, s], pv0[1, s]], np.float32))
           for s in range(S)]

    def run(s):
        o = ors[s]
        return np.concatenate([oracle.frontend(D, I[s, b * blk:(b + 1) * blk], Q[s, b * blk:(b + 1) * blk], h,
                                               o["si"], o["sq"], o["prev"]) for b in range(nblk)])

    with cf.ThreadPoolExecutor(S) as ex:
        want = list(ex.map(run, range(S)))
    for s in range(S):
        for b in range(0, nblk, 8):  # report a failing stream by its 8-block span
            assert_bits(got[s, b * nb:(b + 8) * nb], want[s][b * nb:(b + 8) * nb], f"stream {s} blocks {b}..{b + 7}")
    assert_bits(d_si.download().reshape(S, 100), np.stack([o["si"] for o in ors]), "state_i")
    assert_bits(d_sq.download().reshape(S, 100), np.stack([o["sq"] for o in ors]), "state_q")
    assert_bits(d_pi.download(), np.array([o["prev"][0] for o in ors], np.float32), "prev_i")
    assert_bits(d_pq.download(), np.array([o["prev"][1] for o in ors], np.float32), "prev_q")
    assert np.isfinite(got).all()


def test_cfg4_full_single_call(gpu_ctx, oracle, built_lib):
    """bench.py's cfg4 launch exactly: ONE stream x 67,110,400 pairs (256 x
    262,150) in a single frontend_dev call -- about 53 k tiles of one stream
    across the XCD-slab walk -- against the oracle run block by block over the
    same samples (src/filter.cpp:139 block-size independence), with a
    non-zero carried state; every output and the final state bitwise."""
    sdrhip = built_lib
    nblk, blk, D = 256, 262150, 10
    n = nblk * blk
    h = load_golden("taps")["lpf_rf_mode0"]
    d_h = _dev(sdrhip, gpu_ctx, h)
    d_I, d_Q = _planar_batch(sdrhip, gpu_ctx, 1, n, 4343)
    st0 = np.random.default_rng(7).uniform(-0.7, 0.7, (2, 100)).astype(np.float32)
    pv0 = np.array([-0.125, 0.75], np.float32)
    d_si, d_sq = _dev(sdrhip, gpu_ctx, st0[0]), _dev(sdrhip, gpu_ctx, st0[1])
    d_pi, d_pq = _dev(sdrhip, gpu_ctx, pv0[:1]), _dev(sdrhip, gpu_ctx, pv0[1:])
    d_out = sdrhip.DeviceArray(gpu_ctx, n // D * 4)
    gpu_ctx.frontend_dev(D, d_I, d_Q, n, 1, n, d_h, 101, d_si, d_sq, 100, d_pi, d_pq, d_out, n // D)
    gpu_ctx.synchronize()
    got = d_out.download()
    I, Q = d_I.download(), d_Q.download()
    d_I.free()
    d_Q.free()
    si, sq, pv = st0[0].copy(), st0[1].copy(), pv0.copy()
    nb = blk // D
    for b in range(nblk):
        want = oracle.frontend(D, I[b * blk:(b + 1) * blk], Q[b * blk:(b + 1) * blk], h, si, sq, pv)
        assert_bits(got[b * nb:(b + 1) * nb], want, f"one call vs oracle block {b}")
    assert_bits(d_si.download(), si, "state_i")
    assert_bits(d_sq.download(), sq, "state_q")
    assert_bits(np.concatenate([d_pi.download(), d_pq.download()]), pv, "prev")
    assert np.isfinite(got).all()


def test_cfg5_full_windows(gpu_ctx, oracle, built_lib):
    """BASELINE config 5 at full size: 2 x 1,048,576 samples through the exact
    1024-tap FIR, EVERY output against the oracle.  The record is cut into
    65,536-sample windows run in parallel: the first from the real carried
    state, each later one seeded with the 1,023 inputs before it -- the
    reference's own block rule (src/filter.cpp:82) makes that window equal to
    the same samples of one whole-record call."""
    sdrhip = built_lib
    n, T, W = 1048576, 1024, 65536
    h = oracle.taps_lpf(2.4e6, 100e3, T, 1)
    d_h = _dev(sdrhip, gpu_ctx, h)
    d_I, d_Q = _planar_batch(sdrhip, gpu_ctx, 1, n, 55)
    x = np.stack([d_I.download(), d_Q.download()])
    st0 = np.random.default_rng(4).uniform(-0.7, 0.7, (2, T - 1)).astype(np.float32)
    d_x, d_st = _dev(sdrhip, gpu_ctx, x), _dev(sdrhip, gpu_ctx, st0)
    d_y = sdrhip.DeviceArray(gpu_ctx, 2 * n * 4)
    d_y.fill(0xFF)
    gpu_ctx.fir_block_dev(d_x, n, 2, n, d_h, T, d_st, T - 1, d_y, n)
    gpu_ctx.synchronize()
    y = d_y.download().reshape(2, n)

    def window(job):
        c, a = job
        st = st0[c].copy() if a == 0 else x[c, a - (T - 1):a].copy()
        return oracle.fir_block(x[c, a:a + W], h, st)

    jobs = [(c, a) for c in range(2) for a in range(0, n, W)]
    with cf.ThreadPoolExecutor(16) as ex:
        want = list(ex.map(window, jobs))
    for (c, a), w in zip(jobs, want):
        assert_bits(y[c, a:a + W], w, f"channel {c} window at {a}")
    assert_bits(d_st.download().reshape(2, T - 1), x[:, n - (T - 1):], "state")


def test_cfg3_full_plan_two_steps(gpu_ctx, oracle, built_lib):
    """BASELINE config 3 exactly as bench.py launches it: 1,024 streams x
    65,600 samples through a resampler plan built from the real
    impulseResponseLPF(240e3*147, 16e3, 22197, 147) taps (151 per phase, S =
    150), two consecutive steps with the state carried.  EVERY stream's
    12,054 outputs and carried state bitwise against the oracle
    (src/filter.cpp:142-173) -- the workgroup item split at 1,024 streams."""
    sdrhip = built_lib
    S, n, up, down, T, ns = 1024, 65600, 147, 800, 151 * 147, 150
    ny = sdrhip.resample_out_len(up, down, n)
    assert ny == 12054
    h = oracle.taps_lpf(240e3 * 147, 16e3, T, 147)
    d_h = _dev(sdrhip, gpu_ctx, h)
    plan = gpu_ctx.resample_plan(up, down, d_h, T)
    d_st = _dev(sdrhip, gpu_ctx, np.zeros((S, ns), np.float32))
    d_y = sdrhip.DeviceArray(gpu_ctx, S * ny * 4)
    ors = [np.zeros(ns, np.float32) for _ in range(S)]
    try:
        for step, seed in enumerate((331, 332)):
            d_I, d_Q = _planar_batch(sdrhip, gpu_ctx, S, n, seed)
            d_Q.free()
            d_y.fill(0xFF)
            plan.resample_dev(d_I, n, S, n, d_st, ns, d_y, ny)
            gpu_ctx.synchronize()
            got = d_y.download().reshape(S, ny)
            x = d_I.download().reshape(S, n)
            with cf.ThreadPoolExecutor(16) as ex:  # C behind ctypes: the GIL is released
                want = np.stack(list(ex.map(lambda s: oracle.resample(up, down, x[s], h, ors[s]), range(S))))
            assert_bits(got, want, f"step {step}: all {S} streams")
            assert_bits(d_st.download().reshape(S, ns), np.stack(ors), f"step {step}: state (all streams)")
            d_I.free()
    finally:
        plan.close()


def test_cfg5h_full_f16_tolerance(gpu_ctx, oracle, built_lib):
    """BASELINE config 5's fp16 arm at full size (2 x 1,048,576 samples, the
    1024-tap LPF, fp16 storage, fp32 v_dot2 accumulation): every output within
    2^-9 * sum|h| * max|x| of the exact fp32 reference (src/filter.cpp:66-83),
    and within fp32 accumulation error of the exact sum over the fp16-rounded
    operands; the fp16 state is the last 1,023 inputs exactly."""
    from scipy.signal import oaconvolve

    sdrhip = built_lib
    n, T = 1048576, 1024
    ns = T - 1
    h = oracle.taps_lpf(2.4e6, 100e3, T, 1)
    d_h = _dev(sdrhip, gpu_ctx, h)
    d_I, d_Q = _planar_batch(sdrhip, gpu_ctx, 1, n, 56)
    x = np.stack([d_I.download(), d_Q.download()])
    d_I.free()
    d_Q.free()
    x16 = x.astype(np.float16)
    st0 = np.random.default_rng(5).uniform(-0.7, 0.7, (2, ns)).astype(np.float16)
    d_x, d_st = _dev(sdrhip, gpu_ctx, x16), _dev(sdrhip, gpu_ctx, st0)
    d_y = sdrhip.DeviceArray(gpu_ctx, 2 * n * 4)
    gpu_ctx.fir_block_f16_dev(d_x, n, 2, n, d_h, T, d_st, ns, d_y, n)
    gpu_ctx.synchronize()
    got = d_y.download().reshape(2, n).astype(np.float64)
    hh = h.astype(np.float16).astype(np.float64)
    for c in range(2):
        want = oracle.fir_block(x[c], h, st0[c].astype(np.float32))
        scale = float(np.abs(h).sum()) * float(np.abs(x[c]).max())
        err = np.abs(got[c] - want).max()
        assert err <= 2.0 ** -9 * scale, f"channel {c}: {err:.3g} > 2^-9 * {scale:.3g}"
        xs = np.concatenate([st0[c].astype(np.float64), x16[c].astype(np.float64)])
        exact = oaconvolve(xs, hh)[ns:ns + n]
        bound = T * 2.0 ** -23 * oaconvolve(np.abs(xs), np.abs(hh))[ns:ns + n] + 1e-9
        worst = np.max(np.abs(got[c] - exact) - bound)
        assert worst <= 0, f"channel {c}: off the fp16-operand sum by {worst:.3g} past the fp32 bound"
    assert np.array_equal(d_st.download(np.float16).reshape(2, ns), x16[:, n - ns:]), "fp16 state"
