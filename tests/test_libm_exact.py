"""CPU proof that csrc/libm_exact.hpp gives glibc's floats.

The reference's fmPLL stores (float) of glibc's double atan2 / sincos / cos
on float arguments (src/filter.cpp:199-221; the compiled reference calls
glibc's atan2, sincos and cos).  libm_exact.hpp is what the device PLL and NCO
kernels evaluate (csrc/stereo.hip); its host build here runs the same source
with the same IEEE operations.  tests/test_gpu_libm.py checks that the device
computes the same bits.

* sin / cos: the committed fixture (tests/golden/libm_sincos.npz) comes from a
  sweep over EVERY finite float with zero mismatches; here a slice of 128
  chunks (2^27 arguments) is re-swept, its hashes must equal the fixture's,
  and the fixture's near-midpoint arguments must evaluate to glibc's floats
  (SDR_LIBM_FULL=1 re-sweeps all 4,096 chunks: about 2 minutes on 8 cores).
* atan2: a fresh seeded sample of 2^26 pairs against glibc, and the
  committed near-midpoint pairs of the 2^34-pair sweep.
"""
from __future__ import annotations

import ctypes as C
import json
import os
import subprocess

import numpy as np
import pytest

from conftest import GOLDEN, REPO, load_golden

CSRC = os.path.join(REPO, "3dy4-real-time-software-defined-radio-_amd", "csrc")
# chunk = bits >> 20: around 1.0 (0x3f8), PLL-sized arguments up to 2^26 (0x4c8),
# beyond (Payne-Hanek on the fast path), tiny and subnormal, and negatives
SLICES = [(0, 8), (960, 1000), (1016, 1048), (1180, 1240), (2048, 2056), (3064, 3084)]


@pytest.fixture(scope="module")
def sweep(tmp_path_factory):
    exe = tmp_path_factory.mktemp("libm") / "libm_sweep"
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", "-I", CSRC, "-o", str(exe),
                    os.path.join(REPO, "tests", "libm_sweep.cpp")], check=True)
    return str(exe)


@pytest.fixture(scope="module")
def libm():
    m = C.CDLL("libm.so.6")
    for f in ("sin", "cos"):
        getattr(m, f).restype = C.c_double
        getattr(m, f).argtypes = [C.c_double]
    m.atan2.restype = C.c_double
    m.atan2.argtypes = [C.c_double, C.c_double]
    return m


def _f(bits) -> np.ndarray:
    return np.asarray(bits, np.uint32).view(np.float32)


def _bits(x) -> int:
    return int(np.array([x], np.float32).view(np.uint32)[0])


def _eval(sweep, tmp_path, fn, a, b=None):
    rec = np.zeros((len(a), 3), np.uint32)
    rec[:, 0] = fn
    rec[:, 1] = a
    rec[:, 2] = 0 if b is None else b
    src, dst = tmp_path / "in.bin", tmp_path / "out.bin"
    rec.tofile(src)
    subprocess.run([sweep, "eval", str(src), str(dst)], check=True)
    return np.fromfile(dst, np.uint32)


def test_sincos_fixture_provenance():
    g = load_golden("libm_sincos")
    meta = json.loads(str(g["meta"]))
    # the committed sweep covered every finite float and found no mismatch
    assert meta["args"] == 2 ** 32 - 2 ** 24, meta
    assert meta["sin_mismatch"] == 0 and meta["cos_mismatch"] == 0, meta
    assert meta["sincos_vs_sin_cos"] == 0, meta  # glibc's sincos == its sin and cos
    # the PLL kernel's certified fast sine / cosine (pll_fast.hpp, window kCertWSc) on its whole domain
    assert meta["fast_certified_mismatch"] == 0, meta
    assert g["hash"].shape == (4096,) and g["hash"].dtype == np.uint64


@pytest.mark.parametrize("lo,hi", SLICES)
def test_sincos_slice(sweep, tmp_path, lo, hi):
    pre = str(tmp_path / "s")
    r = json.loads(subprocess.run([sweep, "sincos", str(lo), str(hi), "8", pre], check=True, capture_output=True,
                                  text=True).stdout)
    assert r["sin_mismatch"] == 0 and r["cos_mismatch"] == 0, r
    assert r["sincos_vs_sin_cos"] == 0 and r["fast_certified_mismatch"] == 0, r
    h = np.fromfile(pre + ".hash", np.uint64)
    want = load_golden("libm_sincos")["hash"]
    assert np.array_equal(h[lo:hi], want[lo:hi]), "this host's glibc differs from the fixture's"


@pytest.mark.skipif(os.environ.get("SDR_LIBM_FULL") != "1", reason="SDR_LIBM_FULL=1: every finite float (~2 min)")
def test_sincos_every_float(sweep, tmp_path):
    pre = str(tmp_path / "all")
    r = json.loads(subprocess.run([sweep, "sincos", "0", "4096", str(os.cpu_count() or 8), pre], check=True,
                                  capture_output=True, text=True).stdout)
    assert r["args"] == 2 ** 32 - 2 ** 24
    assert r["sin_mismatch"] == 0 and r["cos_mismatch"] == 0 and r["sincos_vs_sin_cos"] == 0, r
    assert r["fast_certified_mismatch"] == 0, r
    assert np.array_equal(np.fromfile(pre + ".hash", np.uint64), load_golden("libm_sincos")["hash"])


def test_sincos_near_midpoint_fixture(sweep, tmp_path, libm):
    near = load_golden("libm_sincos")["near"]
    assert len(near) > 20
    # this host's glibc still gives the committed floats
    for u, s, c, _ in near:
        x = float(_f([u])[0])
        assert _bits(np.float32(libm.sin(x))) == s and _bits(np.float32(libm.cos(x))) == c, hex(u)
    got_s = _eval(sweep, tmp_path, 0, near[:, 0])
    got_c = _eval(sweep, tmp_path, 1, near[:, 0])
    assert np.array_equal(got_s, near[:, 1]) and np.array_equal(got_c, near[:, 2])


def test_atan2_sample(sweep):
    r = json.loads(subprocess.run([sweep, "atan2", "77", "26", "8"], check=True, capture_output=True,
                                  text=True).stdout)
    assert r["pairs"] == 2 ** 26 and r["atan2_mismatch"] == 0, r
    assert r["fast_uncertified"] < 0.05 * r["pairs"], r  # the short path is the common one


def test_atan2_near_midpoint_fixture(sweep, tmp_path, libm):
    g = load_golden("libm_atan2")
    meta = json.loads(str(g["meta"]))
    assert meta["pairs"] == 2 ** 34 and meta["atan2_mismatch"] == 0, meta
    near = g["near"]
    assert len(near) > 50
    y, x = _f(near[:, 0]), _f(near[:, 1])
    for i in range(len(near)):
        assert _bits(np.float32(libm.atan2(float(y[i]), float(x[i])))) == near[i, 2], i
    assert np.array_equal(_eval(sweep, tmp_path, 2, near[:, 0], near[:, 1]), near[:, 2])
