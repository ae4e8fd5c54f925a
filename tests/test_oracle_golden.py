"""Pins the CPU restatement (oracle/sdr_oracle.c) to the reference.

Every golden fixture in tests/golden/ was produced by the reference's own
src/filter.cpp compiled from /root/reference (tests/golden/make_golden.py).
The oracle must reproduce each one bit for bit; only then is it trusted as
the checker for the GPU kernels at sizes no fixture covers.
"""
import hashlib
import os

import numpy as np
import pytest

from conftest import GOLDEN, assert_bits, assert_bits_nan, load_golden


def test_manifest_hashes(manifest):
    for name, case in manifest["cases"].items():
        with open(os.path.join(GOLDEN, name + ".npz"), "rb") as f:
            assert hashlib.sha256(f.read()).hexdigest() == case["sha256"], name


def test_taps(oracle, manifest):
    g = load_golden("taps")
    params = manifest["cases"]["taps"]["params"]
    for k, (Fs, Fc, T, U) in params["lpf"].items():
        assert_bits(oracle.taps_lpf(Fs, Fc, int(T), int(U)), g["lpf_" + k], f"lpf {k}")
    for k, (Fs, Fb, Fe, T, U) in params["bpf"].items():
        assert_bits(oracle.taps_bpf(Fs, Fb, Fe, int(T), int(U)), g["bpf_" + k], f"bpf {k}")


@pytest.mark.parametrize("name", ["frontend_mode0", "frontend_mode1", "frontend_block100", "frontend_65540"])
def test_frontend(oracle, manifest, name):
    g = load_golden(name)
    p = manifest["cases"][name]["params"]
    D, block, nblk = p["D"], p["block"], p["nblk"]
    I, Q = oracle.u8_to_planar(g["iq_u8"])
    si, sq = np.zeros(100, np.float32), np.zeros(100, np.float32)
    prev = np.zeros(2, np.float32)
    for b in range(nblk):
        sl = slice(b * block, (b + 1) * block)
        yi = oracle.fir_decim(D, I[sl], g["h"], si)
        yq = oracle.fir_decim(D, Q[sl], g["h"], sq)
        dm = oracle.fm_demod(yi, yq, prev)
        assert_bits(yi, g["yi"][b], f"{name} yi[{b}]")
        assert_bits(yq, g["yq"][b], f"{name} yq[{b}]")
        assert_bits(dm, g["demod"][b], f"{name} demod[{b}]")
        assert_bits(np.concatenate([si, sq, prev]), g["states"][b], f"{name} state[{b}]")


def test_demod_edges(oracle, manifest):
    g = load_golden("demod_edges")
    prev = g["prev0"].copy()
    outs = []
    for i, (a, b) in enumerate(manifest["cases"]["demod_edges"]["params"]["segments"]):
        outs.append(oracle.fm_demod(g["I"][a:b], g["Q"][a:b], prev))
        assert_bits(prev, g["prevs"][i], f"prev after segment {i}")
    assert_bits(np.concatenate(outs), g["out"], "demod edges")


@pytest.mark.parametrize("name", ["fir_block_pilot", "fir_block_stereo", "fir_block_1024"])
def test_fir_block(oracle, manifest, name):
    g = load_golden(name)
    p = manifest["cases"][name]["params"]
    st = np.zeros(p["state"], np.float32)
    for b in range(p["nblk"]):
        y = oracle.fir_block(g["x"][b * p["block"]:(b + 1) * p["block"]], g["h"], st)
        assert_bits(y, g["y"][b], f"{name} y[{b}]")
        assert_bits(st, g["states"][b], f"{name} state[{b}]")


@pytest.mark.parametrize("name", ["resample_mode0", "resample_mode2", "resample_mode3", "resample_cfg3",
                                  "resample_3_5"])
def test_resample(oracle, manifest, name):
    g = load_golden(name)
    p = manifest["cases"][name]["params"]
    st = np.zeros(p["state"], np.float32)
    for b in range(p["nblk"]):
        y = oracle.resample(p["up"], p["down"], g["x"][b * p["block"]:(b + 1) * p["block"]], g["h"], st)
        assert_bits(y, g["y"][b], f"{name} y[{b}]")
        assert_bits(st, g["states"][b], f"{name} state[{b}]")


def test_host_glue(oracle):
    g = load_golden("host_glue")
    x = g["x"]
    pll = np.array([1, 0, 0, 0, 0, 1], np.float32)
    for b in range(2):
        nco = oracle.fm_pll(g["pilot"][b * 1024:(b + 1) * 1024], 19e3, 240e3, 2.0, 0.0, 0.01, pll)
        assert_bits(nco, g["nco"][b], f"pll nco[{b}]")
        assert_bits(pll, g["pll_states"][b], f"pll state[{b}]")
    dst = np.zeros(50, np.float32)
    assert_bits(oracle.delay_block(x[:1024], dst), g["delay"][0], "delay 0")
    assert_bits(oracle.delay_block(x[1024:], dst), g["delay"][1], "delay 1")
    assert_bits(dst, g["delay_state"], "delay state")
    y = x[::-1].copy()
    assert_bits(oracle.pointwise_mul(x, y[:2000]), g["mul"], "mul")
    assert_bits(oracle.pointwise_add(x, y), g["add"], "add")
    assert_bits(oracle.pointwise_sub(x, y), g["sub"], "sub")
    assert_bits(oracle.interleave(x[:100], y[:100]), g["inter"], "interleave")
    taps = load_golden("taps")["bpf_pilot_mode0"]
    assert_bits(oracle.convolve_full(x[:300], taps), g["conv"], "convolveFIR")
    assert_bits(oracle.downsample(x[:303], 10), g["down"], "downsample")
    assert_bits(oracle.upsample(x[:40], 3), g["up"], "upsample")


def test_preconditions(oracle):
    h = np.ones(101, np.float32)
    with pytest.raises(ValueError):  # n % D != 0: the reference overflows y (filter.cpp:127-132)
        oracle.fir_decim(10, np.zeros(65536, np.float32), h, np.zeros(100, np.float32))
    with pytest.raises(ValueError):  # state shorter than taps-1
        oracle.fir_block(np.zeros(1000, np.float32), h, np.zeros(50, np.float32))
    with pytest.raises(ValueError):  # (n*L) % M != 0: the reference overflows y (filter.cpp:149-162)
        oracle.resample(147, 800, np.zeros(65536, np.float32), np.ones(22197, np.float32), np.zeros(150, np.float32))


def test_block_size_independence(oracle):
    """The reference property the GPU tiling relies on: one
    whole-stream call == the same samples in consecutive blocks, bitwise."""
    from sdrhip.synth import fm_planar

    I, _ = fm_planar(5120 * 4, seed=7)
    h = load_golden("taps")["lpf_rf_mode0"]
    whole = oracle.fir_decim(10, I, h, np.zeros(100, np.float32))
    st = np.zeros(100, np.float32)
    parts = [oracle.fir_decim(10, I[a:a + 1280], h, st) for a in range(0, len(I), 1280)]
    assert_bits(np.concatenate(parts), whole, "blocked vs whole")


@pytest.mark.skipif(not os.path.exists(os.path.join(os.path.dirname(GOLDEN), "..", "oracle", "_ref", "libref_filter.so")),
                    reason="compiled reference (oracle/_ref) not present")
def test_oracle_vs_compiled_reference_random(oracle):
    """Beyond the fixtures: random inputs, oracle vs the compiled reference."""
    from oracle import Reference

    ref = Reference()
    rng = np.random.default_rng(99)
    h = rng.standard_normal(57).astype(np.float32)
    for D in (1, 3, 10):
        x = rng.standard_normal(570 * D).astype(np.float32)
        s1 = rng.standard_normal(60).astype(np.float32)
        s2 = s1.copy()
        assert_bits(oracle.fir_decim(D, x, h, s1), ref.fir_decim(D, x, h, s2), f"D={D}")
        assert_bits(s1, s2)
    x = rng.standard_normal(1600).astype(np.float32)
    hh = rng.standard_normal(301).astype(np.float32)
    s1 = rng.standard_normal(150).astype(np.float32)
    s2 = s1.copy()
    assert_bits(oracle.resample(3, 8, x, hh, s1), ref.resample(3, 8, x, hh, s2), "resample 3/8")


def test_nonfinite_frontend(oracle):
    """Inf / NaN in samples, carried state and prev_*, sums overflowing to
    Inf: the oracle propagates them as the compiled reference did."""
    g = load_golden("nonfinite_frontend")
    S, nblk, block = g["demod"].shape[0], g["demod"].shape[1], g["I"].shape[1] // g["demod"].shape[1]
    for s in range(S):
        si, sq, prev = g["state_i0"][s].copy(), g["state_q0"][s].copy(), g["prev0"][s].copy()
        for b in range(nblk):
            sl = slice(b * block, (b + 1) * block)
            yi = oracle.fir_decim(10, g["I"][s, sl], g["h"], si)
            yq = oracle.fir_decim(10, g["Q"][s, sl], g["h"], sq)
            assert_bits_nan(oracle.fm_demod(yi, yq, prev), g["demod"][s, b], f"stream {s} block {b}")
            assert_bits_nan(np.concatenate([si, sq, prev]), g["states"][s, b], f"stream {s} state {b}")
    assert np.isnan(g["demod"]).any() and np.isinf(g["demod"]).any()


@pytest.mark.parametrize("name", ["nonfinite_fir_101", "nonfinite_fir_1024", "nonfinite_fir_100",
                                  "nonfinite_decim_101"])
def test_nonfinite_fir(oracle, manifest, name):
    g = load_golden(name)
    p = manifest["cases"][name]["params"]
    for s in range(p["streams"]):
        st = g["state0"][s].copy()
        for b in range(p["nblk"]):
            xb = g["x"][s, b * p["block"]:(b + 1) * p["block"]]
            y = oracle.fir_block(xb, g["h"], st) if p["D"] == 1 else oracle.fir_decim(p["D"], xb, g["h"], st)
            assert_bits_nan(y, g["y"][s, b], f"{name} stream {s} block {b}")
            assert_bits_nan(st, g["states"][s, b], f"{name} stream {s} state {b}")


def test_nonfinite_demod(oracle, manifest):
    g = load_golden("nonfinite_demod")
    prev = g["prev0"].copy()
    outs = []
    for i, (a, b) in enumerate(manifest["cases"]["nonfinite_demod"]["params"]["segments"]):
        outs.append(oracle.fm_demod(g["I"][a:b], g["Q"][a:b], prev))
        assert_bits_nan(prev, g["prevs"][i], f"prev after segment {i}")
    assert_bits_nan(np.concatenate(outs), g["out"], "demod")
