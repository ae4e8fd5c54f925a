"""GPU parity: the HIP kernels, called through the C ABI, against the golden
fixtures of the compiled reference and against the oracle (the CPU
restatement pinned by those fixtures).

The bar is BIT-EXACT for every output and every carried state: the kernels
reproduce the reference's fp32 operation order (products and sums rounded
separately, taps in ascending order from 0.0f, double-precision envelope in
the discriminator), so no tolerance is needed.  For sizes where the oracle
would be too slow, size-independent properties are checked instead
(stream/shard permutation invariance, block-size independence).
"""
import math

import numpy as np
import pytest

from conftest import assert_bits, load_golden

pytestmark = pytest.mark.gpu


def _blocks(a, block, nblk):
    return [a[b * block:(b + 1) * block] for b in range(nblk)]


# ------------------------------------------------------------ golden, host API

@pytest.mark.parametrize("kernel", ["tile", "sc"])
@pytest.mark.parametrize("name", ["frontend_mode0", "frontend_mode1", "frontend_block100", "frontend_65540"])
def test_frontend_fused_golden(gpu_ctx, oracle, manifest, kswitch, name, kernel):
    """kernel: the fused f32 front end on fir_tile, or on fir_tile_sc (SDR_FIR_SC=1)."""
    kswitch("SDR_FIR_SC", "0" if kernel == "tile" else "1")
    g = load_golden(name)
    p = manifest["cases"][name]["params"]
    I, Q = oracle.u8_to_planar(g["iq_u8"])
    si, sq, prev = np.zeros(100, np.float32), np.zeros(100, np.float32), np.zeros(2, np.float32)
    for b, (xi, xq) in enumerate(zip(_blocks(I, p["block"], p["nblk"]), _blocks(Q, p["block"], p["nblk"]))):
        dm = gpu_ctx.frontend(p["D"], xi, xq, g["h"], si, sq, prev)
        assert_bits(dm, g["demod"][b], f"{name} demod[{b}]")
        assert_bits(np.concatenate([si, sq, prev]), g["states"][b], f"{name} states[{b}]")


@pytest.mark.parametrize("kernel", ["grp", "sc"])
@pytest.mark.parametrize("name", ["frontend_mode0", "frontend_mode1", "frontend_block100", "frontend_65540"])
def test_frontend_u8_golden(gpu_ctx, manifest, kswitch, name, kernel):
    """u8 wire front end on each kernel: fir_tile_grp (grp) and fir_tile_sc (sc)."""
    kswitch("SDR_FIR_SC_U8", "0" if kernel == "grp" else "1")
    g = load_golden(name)
    p = manifest["cases"][name]["params"]
    si, sq, prev = np.zeros(100, np.float32), np.zeros(100, np.float32), np.zeros(2, np.float32)
    for b, iq in enumerate(_blocks(g["iq_u8"], 2 * p["block"], p["nblk"])):
        dm = gpu_ctx.frontend_u8(p["D"], iq, g["h"], si, sq, prev)
        assert_bits(dm, g["demod"][b], f"{name} u8 demod[{b}]")
        assert_bits(np.concatenate([si, sq, prev]), g["states"][b], f"{name} u8 states[{b}]")


@pytest.mark.parametrize("name", ["frontend_mode0", "frontend_mode1", "frontend_65540"])
def test_fir_decim_and_demod_golden(gpu_ctx, oracle, manifest, name):
    """The unfused calls, exactly as src/project.cpp:86-90 makes them."""
    g = load_golden(name)
    p = manifest["cases"][name]["params"]
    I, Q = oracle.u8_to_planar(g["iq_u8"])
    si, sq, prev = np.zeros(100, np.float32), np.zeros(100, np.float32), np.zeros(2, np.float32)
    for b in range(p["nblk"]):
        sl = slice(b * p["block"], (b + 1) * p["block"])
        yi = gpu_ctx.fir_decim(p["D"], I[sl], g["h"], si)
        yq = gpu_ctx.fir_decim(p["D"], Q[sl], g["h"], sq)
        assert_bits(yi, g["yi"][b], f"{name} yi[{b}]")
        assert_bits(yq, g["yq"][b], f"{name} yq[{b}]")
        dm = gpu_ctx.fm_demod(yi, yq, prev)
        assert_bits(dm, g["demod"][b], f"{name} demod[{b}]")
        assert_bits(np.concatenate([si, sq, prev]), g["states"][b], f"{name} states[{b}]")


def test_demod_edges_golden(gpu_ctx, manifest):
    g = load_golden("demod_edges")
    prev = g["prev0"].copy()
    outs = []
    for i, (a, b) in enumerate(manifest["cases"]["demod_edges"]["params"]["segments"]):
        outs.append(gpu_ctx.fm_demod(g["I"][a:b], g["Q"][a:b], prev))
        assert_bits(prev, g["prevs"][i], f"prev[{i}]")
    assert_bits(np.concatenate(outs), g["out"], "demod edges")


@pytest.mark.parametrize("name", ["fir_block_pilot", "fir_block_stereo", "fir_block_1024"])
def test_fir_block_golden(gpu_ctx, manifest, name):
    g = load_golden(name)
    p = manifest["cases"][name]["params"]
    st = np.zeros(p["state"], np.float32)
    for b, x in enumerate(_blocks(g["x"], p["block"], p["nblk"])):
        assert_bits(gpu_ctx.fir_block(x, g["h"], st), g["y"][b], f"{name} y[{b}]")
        assert_bits(st, g["states"][b], f"{name} state[{b}]")


@pytest.mark.parametrize("name", ["resample_mode0", "resample_mode2", "resample_mode3", "resample_cfg3",
                                  "resample_3_5"])
def test_resample_golden(gpu_ctx, manifest, name):
    g = load_golden(name)
    p = manifest["cases"][name]["params"]
    st = np.zeros(p["state"], np.float32)
    for b, x in enumerate(_blocks(g["x"], p["block"], p["nblk"])):
        assert_bits(gpu_ctx.resample(p["up"], p["down"], x, g["h"], st), g["y"][b], f"{name} y[{b}]")
        assert_bits(st, g["states"][b], f"{name} state[{b}]")


# ---------------------------------------------------- oracle, other shapes

@pytest.mark.parametrize("D,ntaps,ns,n", [(10, 101, 100, 5120), (10, 101, 137, 5230), (5, 101, 100, 4100),
                                           (1, 101, 100, 3000), (8, 101, 100, 8192), (3, 17, 40, 999),
                                           (10, 64, 63, 640), (1, 1024, 1023, 4096), (4, 300, 320, 4000)])
def test_fir_decim_vs_oracle(gpu_ctx, oracle, D, ntaps, ns, n):
    """Tiled and generic kernels, odd state lengths, even/odd tap counts."""
    rng = np.random.default_rng(D * 1000 + ntaps)
    h = rng.standard_normal(ntaps).astype(np.float32) / ntaps
    s_g = rng.standard_normal(ns).astype(np.float32)
    s_o = s_g.copy()
    for blk in range(3):
        x = rng.standard_normal(n).astype(np.float32)
        assert_bits(gpu_ctx.fir_decim(D, x, h, s_g), oracle.fir_decim(D, x, h, s_o), f"D={D} T={ntaps} blk {blk}")
        assert_bits(s_g, s_o, "state")


@pytest.mark.parametrize("D,n,ns", [(10, 5130, 100), (10, 5130, 150), (10, 2000, 200), (5, 4105, 100),
                                    (5, 4105, 128), (10, 110, 100), (10, 200, 180), (10, 130, 120),
                                    (10, 65530, 100), (10, 65550, 300)])
@pytest.mark.parametrize("kernel", ["tile", "sc"])
def test_frontend_odd_shapes_vs_oracle(gpu_ctx, oracle, kswitch, D, n, ns, kernel):
    """Fused front end (f32 and u8 wire) where the tiled kernel's edge
    handling matters: n % 4 != 0 (a chunk straddles the block end), state
    lengths below and above the kernel's staged strip, blocks barely longer
    than the state (the last output's inputs reach into the old state)."""
    from sdrhip.synth import fm_iq_u8

    kswitch("SDR_FIR_SC", "0" if kernel == "tile" else "1")
    kswitch("SDR_FIR_SC_U8", "0" if kernel == "tile" else "1")
    h = load_golden("taps")["lpf_rf_mode0" if D == 10 else "lpf_rf_mode1"]
    iq = fm_iq_u8(n * 3, seed=D * 100 + n + ns)
    st = {k: [np.zeros(ns, np.float32), np.zeros(ns, np.float32), np.zeros(2, np.float32)]
          for k in ("f32", "u8", "oracle")}
    for b in range(3):
        blk = iq[2 * n * b:2 * n * (b + 1)]
        I, Q = oracle.u8_to_planar(blk)
        want = oracle.frontend(D, I, Q, h, *st["oracle"])
        assert_bits(gpu_ctx.frontend(D, I, Q, h, *st["f32"]), want, f"f32 block {b}")
        assert_bits(gpu_ctx.frontend_u8(D, blk, h, *st["u8"]), want, f"u8 block {b}")
        for k in ("f32", "u8"):
            for got, ref, what in zip(st[k], st["oracle"], ("state_i", "state_q", "prev")):
                assert_bits(got, ref, f"{k} {what} block {b}")


@pytest.mark.parametrize("up,down,ntaps,ns,n", [(147, 800, 22197, 150, 1600), (2, 3, 61, 30, 999),
                                                 (3, 8, 301, 150, 1600), (5, 2, 100, 20, 400)])
def test_resample_vs_oracle(gpu_ctx, oracle, up, down, ntaps, ns, n):
    rng = np.random.default_rng(up * 7 + down)
    h = rng.standard_normal(ntaps).astype(np.float32) / 20
    s_g = rng.standard_normal(ns).astype(np.float32)
    s_o = s_g.copy()
    for blk in range(2):
        x = rng.standard_normal(n).astype(np.float32)
        assert_bits(gpu_ctx.resample(up, down, x, h, s_g), oracle.resample(up, down, x, h, s_o), f"blk {blk}")
        assert_bits(s_g, s_o, "state")


RESAMPLE_CASES = [(147, 800, 151, 150, 1600), (147, 1280, 101, 100, 2560), (3, 7, 101, 100, 700),
                  (5, 2, 151, 150, 400), (147, 800, 151, 150, 65600), (147, 800, 101, 100, 8000),
                  (147, 1280, 101, 100, 12800), (7, 4, 151, 150, 4000), (64, 4, 101, 100, 640),
                  # resample_lp item 1 would start inside the carried state (C*down < 152)
                  (128, 4, 151, 150, 640)]
# resample_lp with its loader wave (the default) and without, then resample_rs,
# then the phase-major resample_pp
RESAMPLE_KERNELS = {"lpw": {"SDR_RESAMPLE_LOADER": "1"}, "lp": {"SDR_RESAMPLE_LOADER": "0"},
                    "rs": {"SDR_RESAMPLE_LP": "0"},
                    "pp": {"SDR_RESAMPLE_LP": "0", "SDR_RESAMPLE_RS": "0"}}


@pytest.mark.parametrize("kernel", list(RESAMPLE_KERNELS))
@pytest.mark.parametrize("up,down,cnt,ns,n", RESAMPLE_CASES)
def test_resample_batched_vs_oracle(gpu_ctx, oracle, built_lib, kswitch, kernel, up, down, cnt, ns, n):
    """Batched resampler (T = cnt*up) on each of its kernels -- lane-phase
    (taps in VGPRs), sliding-window and phase-major: several streams per
    launch, 16-B and dword staging (down % 4), small and large up (column
    subsets), items that start inside the carried state, ragged last
    batches, multi-block state carry.  The kernel is chosen per launch from
    SDR_RESAMPLE_{LP,RS,PP}; shapes a kernel does not cover fall through to
    the next one, so every case is checked under every setting."""
    for k, v in RESAMPLE_KERNELS[kernel].items():
        kswitch(k, v)
    sdrhip = built_lib
    nstreams = 5 if n < 10000 else 2
    rng = np.random.default_rng(up * 1000 + down)
    h = (rng.standard_normal(cnt * up) / cnt).astype(np.float32)
    ny = sdrhip.resample_out_len(up, down, n)
    states = [rng.standard_normal(ns).astype(np.float32) for _ in range(nstreams)]
    d_h = sdrhip.DeviceArray.from_numpy(gpu_ctx, h)
    d_st = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.stack(states))
    y_stride = ny + 3
    d_y = sdrhip.DeviceArray(gpu_ctx, nstreams * y_stride * 4)
    for blk in range(2):
        x = rng.standard_normal((nstreams, n)).astype(np.float32)
        d_x = sdrhip.DeviceArray.from_numpy(gpu_ctx, x)
        gpu_ctx.resample_dev(up, down, d_x, n, nstreams, n, d_h, len(h), d_st, ns, d_y, y_stride)
        gpu_ctx.synchronize()
        got = d_y.download().reshape(nstreams, y_stride)[:, :ny]
        for s in range(nstreams):
            assert_bits(got[s], oracle.resample(up, down, x[s], h, states[s]), f"stream {s} block {blk}")
        assert_bits(d_st.download().reshape(nstreams, ns), np.stack(states), f"state block {blk}")


@pytest.mark.parametrize("kernel", ["lpw", "lp", "rs"])
@pytest.mark.parametrize("up,down,cnt,ns,n", [(147, 800, 151, 150, 8000), (147, 1280, 101, 100, 12800)])
def test_resample_nonfinite_inputs(gpu_ctx, oracle, built_lib, kswitch, kernel, up, down, cnt, ns, n):
    """Inf and NaN inputs (and in the carried state): every output equals the
    reference's -- bitwise where it is a number or an infinity, NaN where the
    reference's is NaN.  resample_lp and resample_rs pad the window ends with
    zero taps and zeroed inputs (term +0), never 0 * Inf."""
    for k, v in RESAMPLE_KERNELS[kernel].items():
        kswitch(k, v)
    sdrhip = built_lib
    nstreams = 3
    rng = np.random.default_rng(7 + up)
    h = (rng.standard_normal(cnt * up) / cnt).astype(np.float32)
    ny = sdrhip.resample_out_len(up, down, n)
    states = [rng.standard_normal(ns).astype(np.float32) for _ in range(nstreams)]
    states[1][ns // 2] = np.inf
    d_h = sdrhip.DeviceArray.from_numpy(gpu_ctx, h)
    d_st = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.stack(states))
    d_y = sdrhip.DeviceArray(gpu_ctx, nstreams * ny * 4)
    x = rng.standard_normal((nstreams, n)).astype(np.float32)
    x[0, 1000] = np.nan
    x[0, 3001] = -np.inf
    x[2, n - 300] = np.inf
    d_x = sdrhip.DeviceArray.from_numpy(gpu_ctx, x)
    gpu_ctx.resample_dev(up, down, d_x, n, nstreams, n, d_h, len(h), d_st, ns, d_y, ny)
    gpu_ctx.synchronize()
    got = d_y.download().reshape(nstreams, ny)
    for s in range(nstreams):
        ref = np.asarray(oracle.resample(up, down, x[s], h, states[s]), dtype=np.float32)
        nan = np.isnan(ref)
        assert np.array_equal(np.isnan(got[s]), nan), f"stream {s}: NaN positions differ"
        assert_bits(got[s][~nan], ref[~nan], f"stream {s}")
        assert (~np.isfinite(ref)).any()  # the Inf / NaN reached some outputs


@pytest.mark.parametrize("up,down,cnt,nstreams,n", [(147, 800, 151, 130, 8000), (147, 800, 101, 64, 4000),
                                                     (441, 3200, 101, 70, 6400), (147, 1280, 101, 3, 25600)])
def test_resample_many_streams(gpu_ctx, oracle, built_lib, up, down, cnt, nstreams, n):
    """The default resampler over many streams per launch (64-130: several
    workgroups' item ranges, items starting inside the carried state, a
    ragged last batch) and over few long streams; three consecutive blocks,
    state carried; checked stream by stream against the oracle (a random
    sample of streams when there are many)."""
    sdrhip = built_lib
    rng = np.random.default_rng(up + down + nstreams)
    h = (rng.standard_normal(cnt * up) / cnt).astype(np.float32)
    ns = cnt - 1
    ny = sdrhip.resample_out_len(up, down, n)
    states = rng.standard_normal((nstreams, ns)).astype(np.float32)
    d_h = sdrhip.DeviceArray.from_numpy(gpu_ctx, h)
    d_st = sdrhip.DeviceArray.from_numpy(gpu_ctx, states)
    d_y = sdrhip.DeviceArray(gpu_ctx, nstreams * ny * 4)
    check = sorted(set([0, nstreams - 1] + list(rng.choice(nstreams, size=min(nstreams, 12), replace=False))))
    for blk in range(3):
        x = rng.standard_normal((nstreams, n)).astype(np.float32)
        d_x = sdrhip.DeviceArray.from_numpy(gpu_ctx, x)
        gpu_ctx.resample_dev(up, down, d_x, n, nstreams, n, d_h, len(h), d_st, ns, d_y, ny)
        gpu_ctx.synchronize()
        got = d_y.download().reshape(nstreams, ny)
        for s in check:
            ref_state = states[s].copy()
            assert_bits(got[s], oracle.resample(up, down, x[s], h, ref_state), f"stream {s} block {blk}")
        states = np.ascontiguousarray(x[:, n - ns:])
        assert_bits(d_st.download().reshape(nstreams, ns), states, f"state block {blk}")


@pytest.mark.parametrize("kernel", ["mfma", "dot2"])
@pytest.mark.parametrize("ntaps,n", [(1024, 65536), (64, 4096), (101, 5000), (1024, 3000), (256, 8200), (8, 704),
                                    (4096, 20000)])
def test_fir_block_f16_tolerance(gpu_ctx, oracle, built_lib, kswitch, ntaps, n, kernel):
    """BASELINE config 5's fp16 arm (fp16 storage, fp32 accumulation -- the
    Toeplitz-GEMM v_mfma_f32_32x32x16_f16 kernel for T % 8 == 0, else / under
    SDR_F16_MFMA=0 the v_dot2_f32_f16 kernel): within 2^-9 * sum|h| * max|x|
    of the exact fp32 reference, and within fp32 accumulation error of the
    exact sum over the fp16-rounded operands.  The carried fp16 state is the
    last ns inputs, exactly."""
    kswitch("SDR_F16_MFMA", "1" if kernel == "mfma" else "0")
    _f16_tolerance_check(gpu_ctx, oracle, built_lib, ntaps, n, 2, ntaps + n)


def _f16_tolerance_check(gpu_ctx, oracle, sdrhip, ntaps, n, nstreams, seed):
    rng = np.random.default_rng(seed)
    h = oracle.taps_lpf(2.4e6, 100e3, ntaps, 1)
    ns = ntaps - 1
    st_ref = [np.zeros(ns, np.float32) for _ in range(nstreams)]
    d_h = sdrhip.DeviceArray.from_numpy(gpu_ctx, h)
    sth = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.zeros(nstreams * ns, np.float16))
    y = sdrhip.DeviceArray(gpu_ctx, nstreams * n * 4)
    hh = h.astype(np.float16).astype(np.float64)
    prev16 = [np.zeros(ns, np.float64) for _ in range(nstreams)]
    for blk in range(2):
        x = rng.standard_normal((nstreams, n)).astype(np.float32)
        xs_ = (n + 7) // 8 * 8  # fp16 rows 16-B aligned (the call's precondition with several streams)
        xp = np.zeros((nstreams, xs_), np.float16)
        xp[:, :n] = x.astype(np.float16)
        xh = sdrhip.DeviceArray.from_numpy(gpu_ctx, xp)
        gpu_ctx.fir_block_f16_dev(xh, n, nstreams, xs_, d_h, ntaps, sth, ns, y, n)
        gpu_ctx.synchronize()
        got = y.download().reshape(nstreams, n)
        for s in range(nstreams):
            want = oracle.fir_block(x[s], h, st_ref[s])
            scale = np.abs(h).sum() * np.abs(x[s]).max()
            assert np.abs(got[s] - want).max() <= 2.0 ** -9 * scale, f"stream {s} block {blk} vs fp32"
            # exact sum over the fp16-rounded operands (fp64), fp32 accumulation bound
            xs = np.concatenate([prev16[s], x[s].astype(np.float16).astype(np.float64)])
            exact = np.convolve(xs, hh)[ns:ns + n]
            bound = ntaps * 2.0 ** -23 * np.convolve(np.abs(xs), np.abs(hh))[ns:ns + n] + 1e-30
            assert np.all(np.abs(got[s] - exact) <= bound), f"stream {s} block {blk} vs fp16-operand sum"
            prev16[s] = xs[-ns:]
        assert np.array_equal(sth.download(np.float16).reshape(nstreams, ns),
                              x[:, -ns:].astype(np.float16)), "fp16 state"


@pytest.mark.parametrize("kernel", ["mfma", "dot2"])
def test_fir_block_f16_padded_rows(gpu_ctx, oracle, built_lib, kswitch, kernel):
    """The fp16 arm on padded rows (x_stride, y_stride > n) over 3 streams, two
    blocks: each stream within the tolerance of its own exact fp32 filter, the
    padding never written, the fp16 state exact."""
    kswitch("SDR_F16_MFMA", "1" if kernel == "mfma" else "0")
    sdrhip = built_lib
    rng = np.random.default_rng(77)
    ntaps, n, nstreams = 1024, 20000, 3
    xs, ys = n + 72, n + 40  # x rows stay 16-B aligned (x_stride % 8 == 0)
    h = oracle.taps_lpf(2.4e6, 100e3, ntaps, 1)
    ns = ntaps - 1
    d_h = sdrhip.DeviceArray.from_numpy(gpu_ctx, h)
    sth = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.zeros(nstreams * ns, np.float16))
    sentinel = np.float32(-12345.0)
    y = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.full(nstreams * ys, sentinel, np.float32))
    st_ref = [np.zeros(ns, np.float32) for _ in range(nstreams)]
    for blk in range(2):
        x = rng.standard_normal((nstreams, n)).astype(np.float32)
        xp = np.zeros((nstreams, xs), np.float16)
        xp[:, :n] = x.astype(np.float16)
        d_x = sdrhip.DeviceArray.from_numpy(gpu_ctx, xp)
        gpu_ctx.fir_block_f16_dev(d_x, n, nstreams, xs, d_h, ntaps, sth, ns, y, ys)
        gpu_ctx.synchronize()
        got = y.download().reshape(nstreams, ys)
        assert np.all(got[:, n:] == sentinel), "padding written"
        for s in range(nstreams):
            want = oracle.fir_block(x[s], h, st_ref[s])
            scale = np.abs(h).sum() * np.abs(x[s]).max()
            assert np.abs(got[s, :n] - want).max() <= 2.0 ** -9 * scale, f"stream {s} block {blk}"
        assert np.array_equal(sth.download(np.float16).reshape(nstreams, ns),
                              x[:, -ns:].astype(np.float16)), "fp16 state"


@pytest.mark.parametrize("waves", ["8", "4"])
@pytest.mark.parametrize("ntaps,n,ns", [(1024, 65536, 1023), (64, 4096, 63), (4096, 20000, 4095), (8, 704, 7),
                                        (1024, 20000, 5000), (256, 8200, 255)])
def test_fir_block_f16_plan_equals_per_call(gpu_ctx, oracle, built_lib, kswitch, ntaps, n, ns, waves):
    """sdr_fir_f16_plan (the MFMA kernel's tap copies built once) against the
    per-call path that builds them in every workgroup: the same MFMA operands
    in the same order, so outputs and the carried fp16 state are BITWISE
    equal, two streams x two blocks; the per-call path itself is pinned to the
    fp32 reference by the tolerance tests above."""
    kswitch("SDR_F16_MFMA", 1)
    kswitch("SDR_F16_W8", 1 if waves == "8" else 0)
    sdrhip = built_lib
    rng = np.random.default_rng(ntaps + 7 * n)
    h = oracle.taps_lpf(2.4e6, 100e3, ntaps, 1)
    S = 2
    A = sdrhip.DeviceArray
    d_h = A.from_numpy(gpu_ctx, h)
    st0 = rng.standard_normal((S, ns)).astype(np.float16)
    sth = {k: A.from_numpy(gpu_ctx, st0.reshape(-1)) for k in ("call", "plan")}
    y = {k: A(gpu_ctx, S * n * 4) for k in ("call", "plan")}
    plan = gpu_ctx.fir_f16_plan(d_h, ntaps)
    try:
        for blk in range(2):
            xh = A.from_numpy(gpu_ctx, rng.standard_normal((S, n)).astype(np.float16))
            gpu_ctx.fir_block_f16_dev(xh, n, S, n, d_h, ntaps, sth["call"], ns, y["call"], n)
            plan.fir_block_f16_dev(xh, n, S, n, sth["plan"], ns, y["plan"], n)
            gpu_ctx.synchronize()
            assert_bits(y["plan"].download(), y["call"].download(), f"block {blk} outputs")
            assert np.array_equal(sth["plan"].download(np.uint16), sth["call"].download(np.uint16)), "fp16 state"
    finally:
        plan.close()


@pytest.mark.parametrize("waves", ["8", "4"])
@pytest.mark.parametrize("head", ["1", "0"])
@pytest.mark.parametrize("ns", [1500, 5000])
def test_fir_block_f16_long_state(gpu_ctx, oracle, built_lib, kswitch, ns, head, waves):
    """The MFMA fp16 arm with a carried state longer than T-1 (the first
    workgroup stages positions [-T, 0) of it and rewrites all ns, past its
    register slots through its loop), under both state-staging orders
    (SDR_F16_HEAD) and both workgroup shapes (SDR_F16_W8: 8 waves of one tile,
    4 of two), two blocks: within the tolerance of the exact fp32 filter, the
    state exact."""
    kswitch("SDR_F16_MFMA", "1")
    kswitch("SDR_F16_HEAD", head)
    kswitch("SDR_F16_W8", "1" if waves == "8" else "0")
    sdrhip = built_lib
    rng = np.random.default_rng(ns)
    ntaps, n, nstreams = 1024, 20000, 2
    h = oracle.taps_lpf(2.4e6, 100e3, ntaps, 1)
    d_h = sdrhip.DeviceArray.from_numpy(gpu_ctx, h)
    st0 = rng.standard_normal((nstreams, ns)).astype(np.float16)
    sth = sdrhip.DeviceArray.from_numpy(gpu_ctx, st0.reshape(-1))
    st_ref = [st0[s].astype(np.float32) for s in range(nstreams)]
    y = sdrhip.DeviceArray(gpu_ctx, nstreams * n * 4)
    for blk in range(2):
        x = rng.standard_normal((nstreams, n)).astype(np.float16).astype(np.float32)
        xh = sdrhip.DeviceArray.from_numpy(gpu_ctx, x.astype(np.float16))
        gpu_ctx.fir_block_f16_dev(xh, n, nstreams, n, d_h, ntaps, sth, ns, y, n)
        gpu_ctx.synchronize()
        got = y.download().reshape(nstreams, n)
        for s in range(nstreams):
            want = oracle.fir_block(x[s], h, st_ref[s])
            scale = np.abs(h).sum() * max(np.abs(x[s]).max(), 4.0)
            assert np.abs(got[s] - want).max() <= 2.0 ** -9 * scale, f"stream {s} block {blk}"
        assert np.array_equal(sth.download(np.float16).reshape(nstreams, ns),
                              x[:, -ns:].astype(np.float16)), "fp16 state"


# ------------------------------------------------------- batched device API

def _fm_streams(nstreams, n, seed=5):
    from sdrhip.synth import fm_iq_u8

    return np.stack([fm_iq_u8(n, seed=seed + s) for s in range(nstreams)])


@pytest.mark.parametrize("src", ["f32", "f32sc", "u8", "u8sc"])
@pytest.mark.parametrize("D,n", [(10, 65540), (10, 5120), (5, 40960)])
def test_frontend_batched_vs_oracle(gpu_ctx, oracle, built_lib, kswitch, src, D, n):
    """nstreams independent streams x 3 consecutive blocks through the
    device-resident batched call; every stream checked against the oracle.
    f32sc: the f32 call on fir_tile_sc (SDR_FIR_SC=1)."""
    sdrhip = built_lib
    kswitch("SDR_FIR_SC", "1" if src == "f32sc" else "0")
    kswitch("SDR_FIR_SC_U8", "1" if src == "u8sc" else "0")
    src = src[:-2] if src.endswith("sc") else src
    nstreams, nblk = 6, 3
    h = load_golden("taps")["lpf_rf_mode0" if D == 10 else "lpf_rf_mode1"]
    iq = _fm_streams(nstreams, n * nblk)
    nout = n // D
    d_h = sdrhip.DeviceArray.from_numpy(gpu_ctx, h)
    d_si = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.zeros((nstreams, 100), np.float32))
    d_sq = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.zeros((nstreams, 100), np.float32))
    d_pi = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.zeros(nstreams, np.float32))
    d_pq = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.zeros(nstreams, np.float32))
    out_stride = (nout + 3) // 4 * 4 + 4  # padded rows
    d_out = sdrhip.DeviceArray(gpu_ctx, nstreams * out_stride * 4)
    ors = [dict(si=np.zeros(100, np.float32), sq=np.zeros(100, np.float32), prev=np.zeros(2, np.float32))
           for _ in range(nstreams)]
    for b in range(nblk):
        blk = iq[:, 2 * n * b:2 * n * (b + 1)]
        if src == "u8":
            d_iq = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.ascontiguousarray(blk))
            gpu_ctx.frontend_u8_dev(D, d_iq, n, nstreams, 2 * n, d_h, len(h), d_si, d_sq, 100, d_pi, d_pq, d_out,
                                    out_stride)
        else:
            I = np.stack([oracle.u8_to_planar(blk[s])[0] for s in range(nstreams)])
            Q = np.stack([oracle.u8_to_planar(blk[s])[1] for s in range(nstreams)])
            d_I = sdrhip.DeviceArray.from_numpy(gpu_ctx, I)
            d_Q = sdrhip.DeviceArray.from_numpy(gpu_ctx, Q)
            gpu_ctx.frontend_dev(D, d_I, d_Q, n, nstreams, n, d_h, len(h), d_si, d_sq, 100, d_pi, d_pq, d_out,
                                 out_stride)
        gpu_ctx.synchronize()
        got = d_out.download().reshape(nstreams, out_stride)[:, :nout]
        for s in range(nstreams):
            Is, Qs = oracle.u8_to_planar(blk[s])
            want = oracle.frontend(D, Is, Qs, h, ors[s]["si"], ors[s]["sq"], ors[s]["prev"])
            assert_bits(got[s], want, f"stream {s} block {b}")
        assert_bits(d_si.download().reshape(nstreams, 100), np.stack([o["si"] for o in ors]), "state_i")
        assert_bits(d_sq.download().reshape(nstreams, 100), np.stack([o["sq"] for o in ors]), "state_q")
        assert_bits(d_pi.download(), np.array([o["prev"][0] for o in ors], np.float32), "prev_i")
        assert_bits(d_pq.download(), np.array([o["prev"][1] for o in ors], np.float32), "prev_q")


@pytest.mark.parametrize("src", ["f32", "u8"])
@pytest.mark.parametrize("D,n", [(10, 65540), (5, 40960)])
def test_frontend_fma_tolerance(gpu_ctx, oracle, built_lib, src, D, n):
    """SDR_ARITH_FMA: one fused multiply-add per tap, same taps and order.  Not
    the reference's bits; bar: demod within 1e-5 of the exact
    oracle where I^2+Q^2 >= 1e-3, carried prev_* within 4e-6*sum|h|*max|x|,
    state exact.  Three consecutive blocks, so the FMA prev_* feeds the next."""
    sdrhip = built_lib
    nstreams, nblk = 4, 3
    h = load_golden("taps")["lpf_rf_mode0" if D == 10 else "lpf_rf_mode1"]
    fir_tol = 4e-6 * np.abs(h).sum() * 1.0  # |x| <= 1 (u8 wire scale)
    iq = _fm_streams(nstreams, n * nblk, seed=40)
    nout = n // D
    d_h = sdrhip.DeviceArray.from_numpy(gpu_ctx, h)
    z = lambda k: sdrhip.DeviceArray.from_numpy(gpu_ctx, np.zeros(k, np.float32))  # noqa: E731
    d_si, d_sq, d_pi, d_pq = z(nstreams * 100), z(nstreams * 100), z(nstreams), z(nstreams)
    d_out = sdrhip.DeviceArray(gpu_ctx, nstreams * nout * 4)
    ors = [dict(si=np.zeros(100, np.float32), sq=np.zeros(100, np.float32), prev=np.zeros(2, np.float32))
           for _ in range(nstreams)]
    gpu_ctx.set_arith(sdrhip.ARITH_FMA)
    try:
        worst = 0.0
        for b in range(nblk):
            blk = iq[:, 2 * n * b:2 * n * (b + 1)]
            if src == "u8":
                d_iq = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.ascontiguousarray(blk))
                gpu_ctx.frontend_u8_dev(D, d_iq, n, nstreams, 2 * n, d_h, len(h), d_si, d_sq, 100, d_pi, d_pq, d_out,
                                        nout)
            else:
                I = np.stack([oracle.u8_to_planar(blk[s])[0] for s in range(nstreams)])
                Q = np.stack([oracle.u8_to_planar(blk[s])[1] for s in range(nstreams)])
                gpu_ctx.frontend_dev(D, sdrhip.DeviceArray.from_numpy(gpu_ctx, I),
                                     sdrhip.DeviceArray.from_numpy(gpu_ctx, Q), n, nstreams, n, d_h, len(h), d_si,
                                     d_sq, 100, d_pi, d_pq, d_out, nout)
            gpu_ctx.synchronize()
            got = d_out.download().reshape(nstreams, nout)
            for s in range(nstreams):
                Is, Qs = oracle.u8_to_planar(blk[s])
                yi = oracle.fir_decim(D, Is, h, ors[s]["si"])
                yq = oracle.fir_decim(D, Qs, h, ors[s]["sq"])
                env = yi.astype(np.float64) ** 2 + yq.astype(np.float64) ** 2
                want = oracle.fm_demod(yi, yq, ors[s]["prev"])
                # the bar holds where the discriminator is conditioned: a block's
                # first outputs see the zero initial state (I^2+Q^2 ~ 1e-6)
                ok = env >= 1e-3
                assert ok.mean() > 0.99
                err = np.abs(got[s].astype(np.float64) - want)[ok]
                assert np.isfinite(got[s]).all()
                assert err.max() <= 1e-5, f"stream {s} block {b}: demod max err {err.max():.3g}"
                worst = max(worst, err.max())
            assert_bits(d_si.download().reshape(nstreams, 100), np.stack([o["si"] for o in ors]), "state_i")
            assert_bits(d_sq.download().reshape(nstreams, 100), np.stack([o["sq"] for o in ors]), "state_q")
            pi = d_pi.download()
            assert np.abs(pi - np.array([o["prev"][0] for o in ors])).max() <= fir_tol, "prev_i"
            pq = d_pq.download()
            assert np.abs(pq - np.array([o["prev"][1] for o in ors])).max() <= fir_tol, "prev_q"
        print(f"fma {src} D={D}: worst demod |err| vs exact {worst:.3g}")
    finally:
        gpu_ctx.set_arith(sdrhip.ARITH_EXACT)


def test_fir_decim_batched_misaligned_stride(gpu_ctx, oracle, built_lib):
    """A stride that breaks 16-B row alignment takes the generic kernel: same bits."""
    sdrhip = built_lib
    rng = np.random.default_rng(3)
    nstreams, n, stride = 3, 5120, 5123
    h = load_golden("taps")["lpf_rf_mode0"]
    x = rng.standard_normal((nstreams, stride)).astype(np.float32)
    st = rng.standard_normal((nstreams, 100)).astype(np.float32)
    d_x = sdrhip.DeviceArray.from_numpy(gpu_ctx, x)
    d_h = sdrhip.DeviceArray.from_numpy(gpu_ctx, h)
    d_s = sdrhip.DeviceArray.from_numpy(gpu_ctx, st)
    d_y = sdrhip.DeviceArray(gpu_ctx, nstreams * 513 * 4)
    gpu_ctx.fir_decim_dev(10, d_x, n, nstreams, stride, d_h, 101, d_s, 100, d_y, 513)
    gpu_ctx.synchronize()
    y = d_y.download().reshape(nstreams, 513)[:, :512]
    for s in range(nstreams):
        so = st[s].copy()
        assert_bits(y[s], oracle.fir_decim(10, x[s, :n], h, so), f"stream {s}")
        assert_bits(d_s.download().reshape(nstreams, 100)[s], so, "state")


def test_u8_to_planar_dev(gpu_ctx, oracle, built_lib):
    sdrhip = built_lib
    iq = _fm_streams(2, 10007 + 1, seed=9)[:, :2 * 10000]
    d_iq = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.ascontiguousarray(iq))
    d_I = sdrhip.DeviceArray(gpu_ctx, 2 * 10000 * 4)
    d_Q = sdrhip.DeviceArray(gpu_ctx, 2 * 10000 * 4)
    gpu_ctx.u8_to_planar_dev(d_iq, 10000, 2, 20000, d_I, d_Q, 10000)
    gpu_ctx.synchronize()
    for s in range(2):
        I, Q = oracle.u8_to_planar(iq[s])
        assert_bits(d_I.download().reshape(2, 10000)[s], I)
        assert_bits(d_Q.download().reshape(2, 10000)[s], Q)


# ------------------------------------------- full BASELINE sizes: properties

def test_full_size_stream_permutation_and_spotcheck(gpu_ctx, oracle, built_lib):
    """BASELINE config 2 at full size (1024 x 65,540-pair blocks, device
    synthetic input): (a) running the streams in a different order/grouping
    gives identical bits per stream (no cross-stream leakage, the property
    multi-GPU sharding relies on); (b) a sample of streams equals the oracle."""
    sdrhip = built_lib
    nstreams, n, D = 1024, 65540, 10
    nout = n // D
    h = load_golden("taps")["lpf_rf_mode0"]
    d_iq = sdrhip.DeviceArray(gpu_ctx, nstreams * 2 * n)
    gpu_ctx.synth_fm_u8_dev(d_iq, n, nstreams, 2 * n, seed=77)
    d_h = sdrhip.DeviceArray.from_numpy(gpu_ctx, h)

    def run(streams):
        k = len(streams)
        d_si = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.zeros((k, 100), np.float32))
        d_sq = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.zeros((k, 100), np.float32))
        d_pi = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.zeros(k, np.float32))
        d_pq = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.zeros(k, np.float32))
        d_out = sdrhip.DeviceArray(gpu_ctx, k * nout * 4 + 16)
        # contiguous runs of streams are one batched launch each
        s0 = streams[0]
        assert list(streams) == list(range(s0, s0 + k))
        gpu_ctx.frontend_u8_dev(D, d_iq.ptr + s0 * 2 * n, n, k, 2 * n, d_h, 101, d_si, d_sq, 100, d_pi, d_pq,
                                d_out, nout)
        gpu_ctx.synchronize()
        return d_out.download(count=k * nout).reshape(k, nout)

    full = run(list(range(nstreams)))
    half = np.concatenate([run(list(range(512, 1024))), run(list(range(0, 512)))])
    assert_bits(np.concatenate([half[512:], half[:512]]), full, "regrouped streams")
    iq_host = d_iq.download(np.uint8).reshape(nstreams, 2 * n)
    for s in (0, 1, 511, 777, 1023):
        I, Q = oracle.u8_to_planar(iq_host[s])
        want = oracle.frontend(D, I, Q, h, np.zeros(100, np.float32), np.zeros(100, np.float32),
                               np.zeros(2, np.float32))
        assert_bits(full[s], want, f"stream {s}")


def test_block_size_independence_gpu(gpu_ctx, oracle):
    """One stream as one 655,400-pair block == the same samples as 10 blocks."""
    from sdrhip.synth import fm_planar

    I, Q = fm_planar(655400, seed=11)
    h = load_golden("taps")["lpf_rf_mode0"]
    z = lambda k: np.zeros(k, np.float32)  # noqa: E731
    whole = gpu_ctx.frontend(10, I, Q, h, z(100), z(100), z(2))
    si, sq, pv = z(100), z(100), z(2)
    parts = [gpu_ctx.frontend(10, I[a:a + 65540], Q[a:a + 65540], h, si, sq, pv) for a in range(0, 655400, 65540)]
    assert_bits(np.concatenate(parts), whole, "blocked vs whole")


# ----------------------------------------------------------- preconditions

def test_preconditions_are_errors(gpu_ctx, built_lib):
    sdrhip = built_lib
    h = np.ones(101, np.float32)
    with pytest.raises(sdrhip.SdrError) as e:  # reference: heap overflow at filter.cpp:132
        gpu_ctx.fir_decim(10, np.zeros(65536, np.float32), h, np.zeros(100, np.float32))
    assert e.value.code == sdrhip.SDR_EINVAL and "multiple" in str(e.value)
    with pytest.raises(sdrhip.SdrError):  # state shorter than taps-1: reads before state
        gpu_ctx.fir_block(np.zeros(1000, np.float32), h, np.zeros(50, np.float32))
    with pytest.raises(sdrhip.SdrError):  # block shorter than the state: state.assign UB
        gpu_ctx.fir_decim(10, np.zeros(50, np.float32), h, np.zeros(100, np.float32))
    with pytest.raises(sdrhip.SdrError):  # resampler y overflow (n*L % M != 0)
        gpu_ctx.resample(147, 800, np.zeros(65536, np.float32), np.ones(22197, np.float32),
                         np.zeros(150, np.float32))
    with pytest.raises(sdrhip.SdrError):  # empty demod block: reference reads I[-1]
        gpu_ctx.fm_demod(np.zeros(0, np.float32), np.zeros(0, np.float32), np.zeros(2, np.float32))


@pytest.mark.parametrize("mix,n", [(False, 12000), (True, 12000), (False, 1003), (True, 5)])
def test_pll_many_streams_vs_oracle(gpu_ctx, oracle, built_lib, mix, n):
    """fmPLL (src/filter.cpp:174-228), one lane per stream, against the
    oracle on 192 streams x 2 blocks x 12,000 samples (~18M double-precision
    atan2/cos/sin evaluations): every NCO sample and all six state floats
    bit-equal.  Pilots: 19 kHz tones at 240 kHz with random phase, frequency
    offset, amplitude and noise, plus exact zeros (the `PLLin == 0` branch).
    n = 1003 and 5 take the kernel's ragged tail (its chunks are 8 samples)."""
    sdrhip = built_lib
    rng = np.random.default_rng(19000 + mix + n)
    S, Fs = 192, 240e3
    t = np.arange(2 * n)
    f = 19e3 + rng.uniform(-40, 40, S)[:, None]
    x = (rng.uniform(0.01, 0.3, S)[:, None] * np.cos(2 * np.pi * f / Fs * t + rng.uniform(0, 6.3, S)[:, None])
         + rng.normal(0, 0.01, (S, 2 * n))).astype(np.float32)
    x[:, ::997] = 0.0
    mixin = rng.standard_normal((S, 2 * n)).astype(np.float32)
    pll = np.tile(np.array([1, 0, 0, 0, 0, 1], np.float32), S)
    A = sdrhip.DeviceArray
    d_pll = A.from_numpy(gpu_ctx, pll)
    d_out = A(gpu_ctx, S * n * 4)
    ost = [np.array([1, 0, 0, 0, 0, 1], np.float32) for _ in range(S)]
    for b in range(2):
        blk = np.ascontiguousarray(x[:, b * n:(b + 1) * n])
        mb = np.ascontiguousarray(mixin[:, b * n:(b + 1) * n])
        d_x, d_m = A.from_numpy(gpu_ctx, blk), A.from_numpy(gpu_ctx, mb)
        gpu_ctx.fm_pll_dev(d_x, n, S, n, 19e3, Fs, 2.0, 0.0, 0.01, d_pll, d_m if mix else None, n, d_out, n)
        gpu_ctx.synchronize()
        got = d_out.download().reshape(S, n)
        dev_st = d_pll.download().reshape(S, 6)
        for s in range(S):
            nco = oracle.fm_pll(blk[s], 19e3, Fs, 2.0, 0.0, 0.01, ost[s])
            want = oracle.pointwise_mul(nco, mb[s]) if mix else nco
            assert_bits(got[s], want, f"stream {s} block {b}")
            assert_bits(dev_st[s], ost[s], f"pll state stream {s} block {b}")


@pytest.mark.parametrize("trig0,phase0", [(0.0, 0.0), (3.0e6, 0.0), (1.6e7, 0.0), (16773000.0, 0.0),
                                          (16777216.0, 0.0), (16777216.0, 2.5e7)])
def test_pll_fast_vs_library(gpu_ctx, oracle, built_lib, trig0, phase0, kswitch):
    """The PLL kernel's certified short-chain path (csrc/pll_fast.hpp, the
    default) against its library-routine path (SDR_PLL_FAST=0) on 512 streams
    x 8,192 samples, bitwise, and 8 streams of it against the oracle.  trig0
    starts the oscillator's trigOffset late (oscillator arguments up to ~8e6
    rad: the reduction's large-argument range); 16,773,000 crosses fp32's
    integer limit 2^24 mid-block and 2^24 starts there -- trigOffset++ stops
    advancing (src/filter.cpp:212), and the certified path keeps running;
    phase0 = 2.5e7 starts phaseEst past 2^24 as well (the loop's phase keeps
    growing there)."""
    sdrhip = built_lib
    rng = np.random.default_rng(int(trig0) + 5)
    S, n, Fs = 512, 8192, 240e3
    t = np.arange(n)
    f = 19e3 + rng.uniform(-40, 40, S)[:, None]
    x = (rng.uniform(0.01, 0.3, S)[:, None] * np.cos(2 * np.pi * f / Fs * t + rng.uniform(0, 6.3, S)[:, None])
         + rng.normal(0, 0.01, (S, n))).astype(np.float32)
    x[:, ::1013] = 0.0
    st0 = np.tile(np.array([1, 0, 0, phase0, trig0, 1], np.float32), S)
    A = sdrhip.DeviceArray
    d_x = A.from_numpy(gpu_ctx, x)
    res = {}
    for fast in ("1", "0"):
        kswitch("SDR_PLL_FAST", fast)
        d_pll = A.from_numpy(gpu_ctx, st0)
        d_out = A(gpu_ctx, S * n * 4)
        gpu_ctx.fm_pll_dev(d_x, n, S, n, 19e3, Fs, 2.0, 0.0, 0.01, d_pll, None, n, d_out, n)
        gpu_ctx.synchronize()
        res[fast] = (d_out.download().reshape(S, n), d_pll.download().reshape(S, 6))
    assert_bits(res["1"][0], res["0"][0], "nco fast vs library")
    assert_bits(res["1"][1], res["0"][1], "pll state fast vs library")
    for s in range(0, S, 64):
        ost = st0[6 * s:6 * s + 6].copy()
        nco = oracle.fm_pll(x[s], 19e3, Fs, 2.0, 0.0, 0.01, ost)
        assert_bits(res["1"][0][s], nco, f"stream {s} vs oracle")
        assert_bits(res["1"][1][s], ost, f"stream {s} state vs oracle")


@pytest.mark.parametrize("guard,n", [("1", 4096), ("0", 4096), ("1", 4093)])
def test_pll_fast_vs_library_wild_inputs(gpu_ctx, oracle, built_lib, kswitch, guard, n):
    """The certified path (its rotation phase detector, the 1,024-ulp window
    and the chunk guards) on inputs far from a pilot: magnitudes 2^-40..2^40
    with random signs, 2 % exact zeros, 1 % tiny or subnormal samples
    (2^-149..2^-60), constant and all-zero streams; every
    result bitwise equal to the library path, 4 streams to the oracle.
    guard: the chunks' input checks from the parallel pre-pass (1, default)
    or inside the recurrence (SDR_PLL_GUARD=0); n = 4093 leaves a ragged tail."""
    sdrhip = built_lib
    kswitch("SDR_PLL_GUARD", guard)
    rng = np.random.default_rng(11)
    S, Fs = 256, 240e3
    x = (rng.choice([-1.0, 1.0], (S, n)) * np.exp2(rng.uniform(-40, 40, (S, n)))).astype(np.float32)
    x[rng.uniform(size=(S, n)) < 0.02] = 0.0
    # tiny and subnormal samples (2^-149 .. 2^-60): outside pllfast::input_ok,
    # their chunks must re-run on the library path
    tiny = rng.uniform(size=(S, n)) < 0.01
    x[tiny] = (rng.choice([-1.0, 1.0], tiny.sum()) * np.exp2(rng.uniform(-149, -60, tiny.sum()))).astype(np.float32)
    x[1] = 0.0
    x[2] = 0.25
    x[3] = -1e-3
    st0 = np.tile(np.array([1, 0, 0, 0, 0, 1], np.float32), S)
    A = sdrhip.DeviceArray
    d_x = A.from_numpy(gpu_ctx, x)
    res = {}
    for fast in ("1", "0"):
        kswitch("SDR_PLL_FAST", fast)
        d_pll = A.from_numpy(gpu_ctx, st0)
        d_out = A(gpu_ctx, S * n * 4)
        gpu_ctx.fm_pll_dev(d_x, n, S, n, 19e3, Fs, 2.0, 0.0, 0.01, d_pll, None, n, d_out, n)
        gpu_ctx.synchronize()
        res[fast] = (d_out.download().reshape(S, n), d_pll.download().reshape(S, 6))
    assert_bits(res["1"][0], res["0"][0], "nco fast vs library")
    assert_bits(res["1"][1], res["0"][1], "pll state fast vs library")
    for s in (0, 1, 2, 3):
        ost = st0[6 * s:6 * s + 6].copy()
        nco = oracle.fm_pll(x[s], 19e3, Fs, 2.0, 0.0, 0.01, ost)
        assert_bits(res["1"][0][s], nco, f"stream {s} vs oracle")
        assert_bits(res["1"][1][s], ost, f"stream {s} state vs oracle")


@pytest.mark.parametrize("up,down,cnt,ns,n", [(147, 800, 151, 150, 65600), (147, 800, 101, 100, 8000),
                                             (147, 1280, 101, 100, 12800), (3, 5, 101, 100, 5000)])
def test_resample_plan_vs_oracle(gpu_ctx, oracle, built_lib, up, down, cnt, ns, n):
    """sdr_resample_plan_*: the lane-phase tables built once at plan creation,
    then three consecutive blocks through the plan -- outputs and carried
    state bitwise against the oracle.  (3, 5) is a shape the lane-phase
    kernel does not take: the plan falls back to the per-call path."""
    sdrhip = built_lib
    nstreams = 3
    rng = np.random.default_rng(up + down + cnt)
    h = (rng.standard_normal(cnt * up) / cnt).astype(np.float32)
    ny = sdrhip.resample_out_len(up, down, n)
    states = [rng.standard_normal(ns).astype(np.float32) for _ in range(nstreams)]
    d_h = sdrhip.DeviceArray.from_numpy(gpu_ctx, h)
    d_st = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.stack(states))
    d_y = sdrhip.DeviceArray(gpu_ctx, nstreams * ny * 4)
    plan = gpu_ctx.resample_plan(up, down, d_h, len(h))
    try:
        for blk in range(3):
            x = rng.standard_normal((nstreams, n)).astype(np.float32)
            d_x = sdrhip.DeviceArray.from_numpy(gpu_ctx, x)
            plan.resample_dev(d_x, n, nstreams, n, d_st, ns, d_y, ny)
            gpu_ctx.synchronize()
            got = d_y.download().reshape(nstreams, ny)
            for s in range(nstreams):
                assert_bits(got[s], oracle.resample(up, down, x[s], h, states[s]), f"stream {s} block {blk}")
            assert_bits(d_st.download().reshape(nstreams, ns), np.stack(states), f"state block {blk}")
    finally:
        plan.close()


# ------------------------------------------------ non-finite inputs

def _rows(a, stride):
    """[S][n] -> [S][stride] zero-padded rows (stride > n: padded or misaligned rows)."""
    out = np.zeros((a.shape[0], stride), np.float32)
    out[:, :a.shape[1]] = a
    return out


@pytest.mark.parametrize("kernel", ["sc", "tile", "generic"])
def test_frontend_nonfinite_inputs(gpu_ctx, built_lib, kswitch, kernel):
    """The fused front end (src/filter.cpp:123-140 x2 + 85-102) on the
    compiled reference's non-finite fixture: Inf, -Inf and NaN in I, in Q, in
    the carried state and prev_*, at a stream's first tile, mid-block, in the
    last 3 samples and in the second block's first tile, and finite inputs
    whose sums overflow to +-Inf (Inf envelopes, Inf - Inf).  7 streams in one
    batched launch, two blocks of 5,130 pairs (n % 4 = 2: the straddling
    chunk); fir_tile_sc (default), fir_tile, and the generic kernel (rows not
    16-B aligned).  Outputs and every carried word bitwise where the
    reference's is a number or an infinity, NaN where it is NaN."""
    from conftest import assert_bits_nan

    sdrhip = built_lib
    kswitch("SDR_FIR_SC", 0 if kernel == "tile" else 1)
    g = load_golden("nonfinite_frontend")
    S, nblk, nout = g["demod"].shape
    block = g["I"].shape[1] // nblk
    stride = block + (1 if kernel == "generic" else 2)
    A = sdrhip.DeviceArray
    d_h = A.from_numpy(gpu_ctx, g["h"])
    d_si, d_sq = A.from_numpy(gpu_ctx, g["state_i0"]), A.from_numpy(gpu_ctx, g["state_q0"])
    d_pi = A.from_numpy(gpu_ctx, np.ascontiguousarray(g["prev0"][:, 0]))
    d_pq = A.from_numpy(gpu_ctx, np.ascontiguousarray(g["prev0"][:, 1]))
    d_out = A(gpu_ctx, S * nout * 4)
    for b in range(nblk):
        sl = slice(b * block, (b + 1) * block)
        d_I = A.from_numpy(gpu_ctx, _rows(g["I"][:, sl], stride))
        d_Q = A.from_numpy(gpu_ctx, _rows(g["Q"][:, sl], stride))
        gpu_ctx.frontend_dev(10, d_I, d_Q, block, S, stride, d_h, 101, d_si, d_sq, 100, d_pi, d_pq, d_out, nout)
        gpu_ctx.synchronize()
        got = d_out.download().reshape(S, nout)
        for s in range(S):
            assert_bits_nan(got[s], g["demod"][s, b], f"{kernel} stream {s} block {b}")
        st = g["states"][:, b]
        assert_bits_nan(d_si.download().reshape(S, 100), st[:, :100], f"{kernel} state_i block {b}")
        assert_bits_nan(d_sq.download().reshape(S, 100), st[:, 100:200], f"{kernel} state_q block {b}")
        assert_bits_nan(d_pi.download(), st[:, 200], f"{kernel} prev_i block {b}")
        assert_bits_nan(d_pq.download(), st[:, 201], f"{kernel} prev_q block {b}")


# kernel: which path runs the fixture (rows 16-B aligned or not, switches)
NONFINITE_FIR = [("nonfinite_fir_101", "tileD1"), ("nonfinite_fir_101", "generic"),
                 ("nonfinite_fir_1024", "long"), ("nonfinite_fir_1024", "long_sgpr"),
                 ("nonfinite_fir_1024", "long_commit0"),
                 ("nonfinite_fir_100", "generic"), ("nonfinite_decim_101", "grp"),
                 ("nonfinite_decim_101", "generic")]


@pytest.mark.parametrize("name,kernel", NONFINITE_FIR)
def test_fir_block_nonfinite_inputs(gpu_ctx, built_lib, manifest, kswitch, name, kernel):
    """blockConvolveFIR (src/filter.cpp:66-83) and the single-channel
    downsampleBlockConvolveFIR (:123-140) on the reference's non-finite
    fixtures: Inf / NaN in samples and carried state (first sample, mid-block,
    the block's last sample carried on, the state's newest word) and sums
    overflowing to +-Inf, 4 streams x 2 blocks in one batched launch each, on
    every kernel the shape can take: fir_tile D = 1 (101 taps), fir_long with
    LDS or SGPR taps (1024), the persistent fir_tile_grp (D = 10), and
    fir_generic (100 taps, or rows not 16-B aligned)."""
    from conftest import assert_bits_nan

    sdrhip = built_lib
    kswitch("SDR_LONG_VTAP", 0 if kernel == "long_sgpr" else 1)
    kswitch("SDR_LONG_COMMIT", 0 if kernel == "long_commit0" else 1)
    g = load_golden(name)
    p = manifest["cases"][name]["params"]
    S, D, block, ns, T = p["streams"], p["D"], p["block"], p["state"], p["ntaps"]
    nout = block // D
    stride = block + (1 if kernel == "generic" else 4)
    A = sdrhip.DeviceArray
    d_h = A.from_numpy(gpu_ctx, g["h"])
    d_st = A.from_numpy(gpu_ctx, g["state0"])
    d_y = A(gpu_ctx, S * nout * 4)
    for b in range(p["nblk"]):
        d_x = A.from_numpy(gpu_ctx, _rows(g["x"][:, b * block:(b + 1) * block], stride))
        gpu_ctx.fir_decim_dev(D, d_x, block, S, stride, d_h, T, d_st, ns, d_y, nout)
        gpu_ctx.synchronize()
        got = d_y.download().reshape(S, nout)
        for s in range(S):
            assert_bits_nan(got[s], g["y"][s, b], f"{name} {kernel} stream {s} block {b}")
        assert_bits_nan(d_st.download().reshape(S, ns), g["states"][:, b], f"{name} {kernel} state block {b}")


def test_demod_nonfinite_inputs(gpu_ctx, built_lib, manifest):
    """fmDemodArctan (src/filter.cpp:85-102) alone on the reference's
    non-finite fixture: Inf / NaN in I, Q and the carried prev_*, envelopes
    that overflow the float (2e19^2 * 2) but not the double, a zero envelope
    between non-finite neighbours -- the `param == 0` rule (:89-92) and the
    IEEE divide meet Inf; three calls carry prev_* on."""
    from conftest import assert_bits_nan

    sdrhip = built_lib
    g = load_golden("nonfinite_demod")
    A = sdrhip.DeviceArray
    d_pi, d_pq = A.from_numpy(gpu_ctx, g["prev0"][:1]), A.from_numpy(gpu_ctx, g["prev0"][1:])
    outs = []
    for i, (a, b) in enumerate(manifest["cases"]["nonfinite_demod"]["params"]["segments"]):
        d_I, d_Q = A.from_numpy(gpu_ctx, g["I"][a:b]), A.from_numpy(gpu_ctx, g["Q"][a:b])
        d_o = A(gpu_ctx, (b - a) * 4)
        gpu_ctx.fm_demod_dev(d_I, d_Q, b - a, 1, b - a, d_pi, d_pq, d_o, b - a)
        gpu_ctx.synchronize()
        outs.append(d_o.download())
        prev = np.concatenate([d_pi.download(), d_pq.download()])
        assert_bits_nan(prev, g["prevs"][i], f"prev after segment {i}")
        # the same segment through the host one-block call (filter.h contract)
        pv = (g["prev0"] if i == 0 else g["prevs"][i - 1]).copy()
        assert_bits_nan(gpu_ctx.fm_demod(g["I"][a:b], g["Q"][a:b], pv), outs[-1], f"host call segment {i}")
    assert_bits_nan(np.concatenate(outs), g["out"], "demod")


@pytest.mark.parametrize("commit", [1, 0])
@pytest.mark.parametrize("ntaps,ns,n", [(64, 63, 5000), (64, 63, 900), (1024, 1023, 5000), (1024, 1500, 5000),
                                        (1056, 1055, 5000)])
def test_fir_long_state_commit(gpu_ctx, oracle, built_lib, kswitch, ntaps, ns, n, commit):
    """blockConvolveFIR's state update (src/filter.cpp:82) under both commit
    paths of fir_long: the stream's first workgroup writing the new state in
    the filter's own launch (T <= 1,025: it is the old state's only reader),
    or the separate long_commit launch (SDR_LONG_COMMIT=0, and always for
    T = 1,056, whose second workgroup also reads the state) -- 3 streams x 3
    blocks on padded rows, outputs and every state bitwise the oracle's; n = 900
    is one workgroup per stream (it reads and rewrites the state alone)."""
    sdrhip = built_lib
    kswitch("SDR_LONG_COMMIT", commit)
    S, stride = 3, n + 4
    rng = np.random.default_rng(ntaps + ns)
    h = (rng.standard_normal(ntaps) / ntaps).astype(np.float32)
    st = rng.standard_normal((S, ns)).astype(np.float32)
    ost = [st[s].copy() for s in range(S)]
    A = sdrhip.DeviceArray
    d_h, d_st, d_y = A.from_numpy(gpu_ctx, h), A.from_numpy(gpu_ctx, st), A(gpu_ctx, S * n * 4)
    for b in range(3):
        x = rng.standard_normal((S, n)).astype(np.float32)
        d_x = A.from_numpy(gpu_ctx, _rows(x, stride))
        gpu_ctx.fir_block_dev(d_x, n, S, stride, d_h, ntaps, d_st, ns, d_y, n)
        gpu_ctx.synchronize()
        got = d_y.download().reshape(S, n)
        for s in range(S):
            assert_bits(got[s], oracle.fir_block(x[s], h, ost[s]), f"stream {s} block {b}")
        assert_bits(d_st.download().reshape(S, ns), np.stack(ost), f"state block {b}")


def test_fir_long_8192_taps_both_tap_modes(gpu_ctx, oracle, built_lib, kswitch):
    """fir_long at its largest tap count (8,192): the LDS-tap kernel would
    halve the workgroups per CU there, so the launcher takes the SGPR-tap
    kernel; under either switch setting the outputs and state are
    bitwise the oracle's (src/filter.cpp:66-83), 2 streams x 2 blocks."""
    sdrhip = built_lib
    T, ns, n, S = 8192, 8191, 20000, 2
    rng = np.random.default_rng(8192)
    h = (rng.standard_normal(T) / T).astype(np.float32)
    A = sdrhip.DeviceArray
    d_h = A.from_numpy(gpu_ctx, h)
    for vtap in (1, 0):
        kswitch("SDR_LONG_VTAP", vtap)
        st = rng.standard_normal((S, ns)).astype(np.float32)
        d_st = A.from_numpy(gpu_ctx, st)
        ost = [st[s].copy() for s in range(S)]
        d_y = A(gpu_ctx, S * n * 4)
        for b in range(2):
            x = rng.standard_normal((S, n)).astype(np.float32)
            gpu_ctx.fir_block_dev(A.from_numpy(gpu_ctx, x), n, S, n, d_h, T, d_st, ns, d_y, n)
            gpu_ctx.synchronize()
            got = d_y.download().reshape(S, n)
            for s in range(S):
                assert_bits(got[s], oracle.fir_block(x[s], h, ost[s]), f"vtap {vtap} stream {s} block {b}")
            assert_bits(d_st.download().reshape(S, ns), np.stack(ost), f"vtap {vtap} state block {b}")


# ------------------------------------------------ seeded random shape sweep
# Shapes drawn once from a fixed seed (the same list every run): decimation
# 1-12, tap counts 1-320 odd and even, state lengths from T-1 to T+63, block
# lengths from one output to ~20 k samples, three consecutive blocks each so
# the carried state is exercised -- every kernel choice the dispatcher makes
# (tiled, split-channel, generic, long) meets shapes no hand-written case
# picked.  Bitwise against the oracle, outputs and state.  Shapes the
# reference cannot run (block shorter than the state, n*up/down fractional)
# are refused by the library and are kept out of the draw.
_RNG = np.random.default_rng(20261018)
_DECIM = []
for _ in range(24):
    _D = int(_RNG.integers(1, 13))
    _T = int(_RNG.choice([int(_RNG.integers(1, 40)), int(_RNG.integers(40, 321)), 101, 64, 128]))
    _ns = _T - 1 + int(_RNG.integers(0, 64))
    _n = _D * int(_RNG.choice([1, int(_RNG.integers(2, 300)), int(_RNG.integers(300, 2000))]))
    _ns = max(_ns, 0)
    _n = max(_n, (_ns + _D - 1) // _D * _D)  # block >= state (filter.cpp:139's precondition, refused otherwise)
    _DECIM.append((_D, _T, _ns, _n))
_RES = []
for _ in range(12):
    _up, _down = int(_RNG.integers(1, 12)), int(_RNG.integers(1, 40))
    _T = _up * int(_RNG.integers(2, 120)) + int(_RNG.integers(0, _up))
    _ns = (_T + _up - 1) // _up - 1 + int(_RNG.integers(0, 8))
    _q = _down // math.gcd(_up, _down)  # n*up/down whole (filter.cpp:149-162's loop bound, refused otherwise)
    _n = _q * max(1, int(_RNG.integers(1, 6000)) // _q)
    _n = max(_n, (_ns + _q - 1) // _q * _q)
    _RES.append((_up, _down, _T, max(_ns, 1), _n))

_FRONT = []
for _ in range(12):
    _D = int(_RNG.choice([1, 2, 4, 5, 8, 10, 10, 12]))
    _T = int(_RNG.choice([101, 101, int(_RNG.integers(2, 200))]))
    _ns = _T - 1 + int(_RNG.integers(0, 40))
    _n = _D * max(int(_RNG.integers(1, 3000)), (_ns + _D - 1) // _D)
    _FRONT.append((_D, _T, _ns, _n))


@pytest.mark.gpu
@pytest.mark.parametrize("D,ntaps,ns,n", _FRONT, ids=[f"D{d}-T{t}-ns{s}-n{n}" for d, t, s, n in _FRONT])
def test_frontend_random_shapes(gpu_ctx, oracle, D, ntaps, ns, n):
    """The fused front end (FIR + decimate on I and Q, then the
    discriminator), f32 planar and u8 wire input, three blocks each."""
    from sdrhip.synth import fm_iq_u8

    rng = np.random.default_rng(D * 131 + ntaps * 7 + n)
    h = (rng.standard_normal(ntaps) / ntaps).astype(np.float32)
    iq = fm_iq_u8(n * 3, seed=int(rng.integers(1 << 30)))
    st = {k: [np.zeros(ns, np.float32), np.zeros(ns, np.float32), np.zeros(2, np.float32)]
          for k in ("f32", "u8", "oracle")}
    for b in range(3):
        blk = iq[2 * n * b:2 * n * (b + 1)]
        I, Q = oracle.u8_to_planar(blk)
        want = oracle.frontend(D, I, Q, h, *st["oracle"])
        assert_bits(gpu_ctx.frontend(D, I, Q, h, *st["f32"]), want, f"f32 block {b}")
        assert_bits(gpu_ctx.frontend_u8(D, blk, h, *st["u8"]), want, f"u8 block {b}")
        for k in ("f32", "u8"):
            for got, ref, what in zip(st[k], st["oracle"], ("state_i", "state_q", "prev")):
                assert_bits(got, ref, f"{k} {what} block {b}")


@pytest.mark.gpu
@pytest.mark.parametrize("D,ntaps,ns,n", _DECIM, ids=[f"D{d}-T{t}-ns{s}-n{n}" for d, t, s, n in _DECIM])
def test_fir_decim_random_shapes(gpu_ctx, oracle, D, ntaps, ns, n):
    rng = np.random.default_rng(D * 7919 + ntaps * 31 + n)
    h = (rng.standard_normal(ntaps) / max(ntaps, 1)).astype(np.float32)
    s_g = rng.standard_normal(ns).astype(np.float32)
    s_o = s_g.copy()
    for blk in range(3):
        x = rng.standard_normal(n).astype(np.float32)
        assert_bits(gpu_ctx.fir_decim(D, x, h, s_g), oracle.fir_decim(D, x, h, s_o), f"block {blk}")
        assert_bits(s_g, s_o, f"state after block {blk}")


@pytest.mark.gpu
@pytest.mark.parametrize("up,down,ntaps,ns,n", _RES, ids=[f"L{u}-M{d}-T{t}-ns{s}-n{n}" for u, d, t, s, n in _RES])
def test_resample_random_shapes(gpu_ctx, oracle, up, down, ntaps, ns, n):
    rng = np.random.default_rng(up * 104729 + down * 31 + ntaps)
    h = (rng.standard_normal(ntaps) / 20).astype(np.float32)
    s_g = rng.standard_normal(ns).astype(np.float32)
    s_o = s_g.copy()
    for blk in range(3):
        x = rng.standard_normal(n).astype(np.float32)
        assert_bits(gpu_ctx.resample(up, down, x, h, s_g), oracle.resample(up, down, x, h, s_o), f"block {blk}")
        assert_bits(s_g, s_o, f"state after block {blk}")


_BATCH = []
for _ in range(12):
    _D = int(_RNG.choice([1, 2, 4, 5, 10, 10, 8]))
    _T = int(_RNG.choice([101, int(_RNG.integers(2, 160))]))
    _ns = _T - 1 + int(_RNG.integers(0, 20))
    _n = _D * max(int(_RNG.integers(1, 2500)), (_ns + _D - 1) // _D)
    _BATCH.append((_D, _T, _ns, _n, int(_RNG.integers(1, 8)), int(_RNG.integers(0, 8)), int(_RNG.integers(0, 6))))


@pytest.mark.gpu
@pytest.mark.parametrize("D,ntaps,ns,n,nstreams,xpad,ypad", _BATCH,
                         ids=[f"D{d}-T{t}-ns{s}-n{n}-S{k}-px{p}-py{q}" for d, t, s, n, k, p, q in _BATCH])
def test_batched_random_shapes(gpu_ctx, oracle, built_lib, D, ntaps, ns, n, nstreams, xpad, ypad):
    """The device-resident batched calls on random shapes: nstreams rows
    with padded strides (aligned or not -- the dispatcher's fast or generic
    path), FIR + decimate on f32 rows and the fused u8 front end, three
    blocks, every stream and state bitwise against the oracle."""
    sdrhip = built_lib
    rng = np.random.default_rng(D * 17 + ntaps * 3 + n + nstreams)
    h = (rng.standard_normal(ntaps) / ntaps).astype(np.float32)
    nout = n // D
    xs, ys = n + xpad, nout + ypad
    d_h = sdrhip.DeviceArray.from_numpy(gpu_ctx, h)
    # FIR + decimate, f32 rows
    st = rng.standard_normal((nstreams, ns)).astype(np.float32)
    ref_st = st.copy()
    d_s = sdrhip.DeviceArray.from_numpy(gpu_ctx, st)
    d_y = sdrhip.DeviceArray(gpu_ctx, nstreams * ys * 4)
    for b in range(3):
        x = rng.standard_normal((nstreams, xs)).astype(np.float32)
        d_x = sdrhip.DeviceArray.from_numpy(gpu_ctx, x)
        gpu_ctx.fir_decim_dev(D, d_x, n, nstreams, xs, d_h, ntaps, d_s, ns, d_y, ys)
        gpu_ctx.synchronize()
        y = d_y.download().reshape(nstreams, ys)[:, :nout]
        for s in range(nstreams):
            assert_bits(y[s], oracle.fir_decim(D, x[s, :n], h, ref_st[s]), f"fir stream {s} block {b}")
        assert_bits(d_s.download().reshape(nstreams, ns), ref_st, f"fir state block {b}")
    # fused u8 front end (IQ rows of 2n bytes + an even pad)
    iqs = 2 * n + 2 * xpad
    iq = _fm_streams(nstreams, (iqs // 2) * 3 + 1, seed=int(rng.integers(1 << 30)))
    z = lambda *shape: sdrhip.DeviceArray.from_numpy(gpu_ctx, np.zeros(shape, np.float32))  # noqa: E731
    d_si, d_sq, d_pi, d_pq = z(nstreams, ns), z(nstreams, ns), z(nstreams), z(nstreams)
    ors = [dict(si=np.zeros(ns, np.float32), sq=np.zeros(ns, np.float32), prev=np.zeros(2, np.float32))
           for _ in range(nstreams)]
    for b in range(3):
        blk = np.ascontiguousarray(iq[:, iqs * b:iqs * (b + 1)])
        d_iq = sdrhip.DeviceArray.from_numpy(gpu_ctx, blk)
        gpu_ctx.frontend_u8_dev(D, d_iq, n, nstreams, iqs, d_h, ntaps, d_si, d_sq, ns, d_pi, d_pq, d_y, ys)
        gpu_ctx.synchronize()
        got = d_y.download().reshape(nstreams, ys)[:, :nout]
        for s in range(nstreams):
            Is, Qs = oracle.u8_to_planar(blk[s, :2 * n])
            want = oracle.frontend(D, Is, Qs, h, ors[s]["si"], ors[s]["sq"], ors[s]["prev"])
            assert_bits(got[s], want, f"u8 stream {s} block {b}")
        assert_bits(d_si.download().reshape(nstreams, ns), np.stack([o["si"] for o in ors]), f"state_i block {b}")
        assert_bits(d_sq.download().reshape(nstreams, ns), np.stack([o["sq"] for o in ors]), f"state_q block {b}")
        assert_bits(d_pi.download(), np.array([o["prev"][0] for o in ors], np.float32), f"prev_i block {b}")
        assert_bits(d_pq.download(), np.array([o["prev"][1] for o in ors], np.float32), f"prev_q block {b}")


_F16 = []
for _ in range(10):
    _T = int(_RNG.choice([8 * int(_RNG.integers(1, 257)), int(_RNG.integers(2, 600))]))
    _F16.append((_T, int(_RNG.integers(max(_T, 8), 40000)), int(_RNG.integers(1, 4))))


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", ["mfma", "dot2"])
@pytest.mark.parametrize("ntaps,n,nstreams", _F16, ids=[f"T{t}-n{n}-S{k}" for t, n, k in _F16])
def test_fir_block_f16_random_shapes(gpu_ctx, oracle, built_lib, kswitch, ntaps, n, nstreams, kernel):
    """The fp16 arm's tolerance contract (as test_fir_block_f16_tolerance) on
    seeded random shapes: tap counts on and off the MFMA kernel's T % 8 grid,
    1-3 streams, blocks from the tap count to 40 k."""
    kswitch("SDR_F16_MFMA", "1" if kernel == "mfma" else "0")
    _f16_tolerance_check(gpu_ctx, oracle, built_lib, ntaps, n, nstreams, ntaps * 7 + n)


_RESB = []
for _ in range(8):
    _up = int(_RNG.choice([int(_RNG.integers(1, 12)), int(_RNG.integers(12, 449))]))
    _down = int(_RNG.choice([4 * int(_RNG.integers(1, 330)), int(_RNG.integers(1, 1300))]))
    _cnt = int(_RNG.choice([101, 151, int(_RNG.integers(2, 60))]))
    _ns = _cnt - 1 + int(_RNG.integers(0, 8))
    _q = _down // math.gcd(_up, _down)
    _n = _q * max(1, int(_RNG.integers(1, 9000)) // _q)
    _n = max(_n, (_ns + _q - 1) // _q * _q)
    _RESB.append((_up, _down, _cnt, _ns, _n, int(_RNG.integers(1, 6)), int(_RNG.integers(0, 5))))


@pytest.mark.gpu
@pytest.mark.parametrize("kernel", list(RESAMPLE_KERNELS))
@pytest.mark.parametrize("up,down,cnt,ns,n,nstreams,xpad", _RESB,
                         ids=[f"L{u}-M{d}-C{c}-ns{s}-n{n}-S{k}-px{p}" for u, d, c, s, n, k, p in _RESB])
def test_resample_batched_random_shapes(gpu_ctx, oracle, built_lib, kswitch, kernel, up, down, cnt, ns, n,
                                        nstreams, xpad):
    """The batched resampler on seeded random shapes (T = cnt * up, lane-phase
    shapes and others, padded input rows) under every kernel setting, three
    blocks, every stream and state bitwise against the oracle."""
    for k, v in RESAMPLE_KERNELS[kernel].items():
        kswitch(k, v)
    sdrhip = built_lib
    rng = np.random.default_rng(up * 1009 + down * 7 + cnt + n)
    h = (rng.standard_normal(cnt * up) / cnt).astype(np.float32)
    ny = sdrhip.resample_out_len(up, down, n)
    states = [rng.standard_normal(ns).astype(np.float32) for _ in range(nstreams)]
    d_h = sdrhip.DeviceArray.from_numpy(gpu_ctx, h)
    d_st = sdrhip.DeviceArray.from_numpy(gpu_ctx, np.stack(states))
    xs, ys = n + xpad, ny + 1
    d_y = sdrhip.DeviceArray(gpu_ctx, nstreams * ys * 4)
    for blk in range(3):
        x = rng.standard_normal((nstreams, xs)).astype(np.float32)
        d_x = sdrhip.DeviceArray.from_numpy(gpu_ctx, x)
        gpu_ctx.resample_dev(up, down, d_x, n, nstreams, xs, d_h, len(h), d_st, ns, d_y, ys)
        gpu_ctx.synchronize()
        got = d_y.download().reshape(nstreams, ys)[:, :ny]
        for s in range(nstreams):
            assert_bits(got[s], oracle.resample(up, down, x[s, :n], h, states[s]), f"stream {s} block {blk}")
        assert_bits(d_st.download().reshape(nstreams, ns), np.stack(states), f"state block {blk}")
