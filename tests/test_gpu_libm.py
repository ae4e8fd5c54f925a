"""GPU proof that the device PLL / NCO transcendental routines
(csrc/libm_exact.hpp, called by csrc/stereo.hip) give glibc's floats -- the
floats the reference's fmPLL stores (src/filter.cpp:199-221).

* sin / cos on EVERY finite float: the device's per-chunk hashes of its
  (sin, cos) floats over all 2^32 bit patterns equal the hashes of glibc's
  floats committed in tests/golden/libm_sincos.npz (the CPU sweep that made
  them found libm_exact == glibc on every argument).
* ROCm's own double sin / cos (what the PLL's fallback and the NCO ran until
  round 6) over the same 2^32 patterns: every argument where its float differs
  from the device routine's is listed, and on each one the device routine
  agrees with this box's glibc and ROCm's does not.
* the committed near-midpoint arguments of sin / cos and pairs of atan2: the
  device gives glibc's floats.
* atan2 screened on the device: 2^36 seeded pairs; every pair whose exact
  value lies within 4 double ulps of a float midpoint (the only pairs two
  ~1-ulp libraries can round apart) is checked against this box's glibc; the
  rest are decided by the error bounds (libm_exact.hpp header).
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import pytest

from conftest import load_golden

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def libm():
    m = C.CDLL("libm.so.6")
    for f in ("sin", "cos"):
        getattr(m, f).restype = C.c_double
        getattr(m, f).argtypes = [C.c_double]
    m.atan2.restype = C.c_double
    m.atan2.argtypes = [C.c_double, C.c_double]
    return m


def _bits(x) -> int:
    return int(np.array([x], np.float32).view(np.uint32)[0])


def _f(u) -> float:
    return float(np.array([u], np.uint32).view(np.float32)[0])


def _hashes(sdrhip, ctx, mode):
    d_h = sdrhip.DeviceArray(ctx, 4096 * 8)
    d_h.fill(0)
    for lo in range(0, 4096, 512):  # 2^29 arguments per launch
        ctx.libm_sincos_hash_dev(mode, lo, lo + 512, d_h)
    ctx.synchronize()
    return d_h.download(np.uint64)


def test_device_sincos_every_float(gpu_ctx, built_lib):
    want = load_golden("libm_sincos")["hash"]
    got = _hashes(built_lib, gpu_ctx, 0)
    bad = np.flatnonzero(got != want)
    assert len(bad) == 0, f"{len(bad)} of 4096 chunks differ from glibc's floats, first chunk {bad[:8]}"


def test_rocm_library_vs_glibc(gpu_ctx, built_lib, libm, record_property):
    """Where ROCm's double sin / cos round to another float than the device
    routine, the device routine is glibc's and ROCm's is not."""
    sdrhip = built_lib
    cap = 1 << 20
    d_n = sdrhip.DeviceArray(gpu_ctx, 8)
    d_n.fill(0)
    d_a = sdrhip.DeviceArray(gpu_ctx, 2 * cap * 4)
    for lo in range(0, 4096, 512):
        gpu_ctx.libm_sincos_diff_dev(lo, lo + 512, d_n, d_a, cap)
    gpu_ctx.synchronize()
    n = int(d_n.download(np.uint64)[0])
    assert n <= cap, n
    rec = d_a.download(np.uint32, count=2 * n).reshape(n, 2)
    record_property("rocm_sincos_float_differs", n)
    print(f"ROCm double sin/cos round to a different float than glibc on {n} of 4,278,190,080 arguments")
    if n:
        k = min(n, 4096)  # the first 4,096 listed (glibc runs per argument on the host)
        d_x = sdrhip.DeviceArray.from_numpy(gpu_ctx, rec[:k, 0].copy())
        d_o = sdrhip.DeviceArray(gpu_ctx, 4 * k)
        out = {}
        for fn in (0, 1, 3, 4):
            gpu_ctx.libm_eval_dev(fn, d_x, None, k, d_o)
            gpu_ctx.synchronize()
            out[fn] = d_o.download(np.uint32)
        for i, (u, flags) in enumerate(rec[:k]):
            x = _f(u)
            gs, gc = _bits(np.float32(libm.sin(x))), _bits(np.float32(libm.cos(x)))
            assert out[0][i] == gs and out[1][i] == gc, f"device routine != glibc at x={x!r}"
            assert (flags & 1) == 0 or out[3][i] != gs, f"ROCm sin listed but equal to glibc at {x!r}"
            assert (flags & 2) == 0 or out[4][i] != gc, f"ROCm cos listed but equal to glibc at {x!r}"


def test_device_libm_near_midpoint_fixtures(gpu_ctx, built_lib):
    sdrhip = built_lib
    near = load_golden("libm_sincos")["near"]
    d_a = sdrhip.DeviceArray.from_numpy(gpu_ctx, near[:, 0].copy())
    d_o = sdrhip.DeviceArray(gpu_ctx, 4 * len(near))
    for fn, col in ((0, 1), (1, 2)):
        gpu_ctx.libm_eval_dev(fn, d_a, None, len(near), d_o)
        gpu_ctx.synchronize()
        got = d_o.download(np.uint32)
        assert np.array_equal(got, near[:, col]), f"fn {fn}: {np.count_nonzero(got != near[:, col])} differ"
    at = load_golden("libm_atan2")["near"]
    d_y = sdrhip.DeviceArray.from_numpy(gpu_ctx, at[:, 0].copy())
    d_x = sdrhip.DeviceArray.from_numpy(gpu_ctx, at[:, 1].copy())
    d_o = sdrhip.DeviceArray(gpu_ctx, 4 * len(at))
    gpu_ctx.libm_eval_dev(2, d_y, d_x, len(at), d_o)
    gpu_ctx.synchronize()
    got = d_o.download(np.uint32)
    assert np.array_equal(got, at[:, 2]), f"atan2: {np.count_nonzero(got != at[:, 2])} of {len(at)} differ"
    # the platform library on the same pairs (informational: how often it rounds apart)
    gpu_ctx.libm_eval_dev(5, d_y, d_x, len(at), d_o)
    gpu_ctx.synchronize()
    print(f"ROCm atan2 differs from glibc on {np.count_nonzero(d_o.download(np.uint32) != at[:, 2])} "
          f"of {len(at)} near-midpoint pairs")


def test_device_atan2_screen(gpu_ctx, built_lib, libm, record_property):
    sdrhip = built_lib
    seed, total, batch = 0x5D0A7A25, 1 << 36, 1 << 32
    cand_cap, out_cap = 1 << 27, 1 << 16
    d_c = sdrhip.DeviceArray(gpu_ctx, cand_cap * 4)
    d_o = sdrhip.DeviceArray(gpu_ctx, out_cap * 16)
    d_n = sdrhip.DeviceArray(gpu_ctx, 16)
    checked = ncand = 0
    for first in range(0, total, batch):
        d_n.fill(0)
        gpu_ctx.libm_atan2_screen_dev(seed, first, batch, d_c, cand_cap, d_o, out_cap, d_n)
        gpu_ctx.synchronize()
        nc, nn = (int(v) for v in d_n.download(np.uint64))
        assert nc <= cand_cap and nn <= out_cap, (nc, nn)
        ncand += nc
        rec = d_o.download(np.uint32, count=4 * nn).reshape(nn, 4)
        for y, x, f, _ in rec:
            g = _bits(np.float32(libm.atan2(_f(y), _f(x))))
            assert f == g, f"atan2({_f(y)!r}, {_f(x)!r}): device {_f(f)!r}, glibc {_f(g)!r}"
        checked += nn
    record_property("atan2_screen", {"pairs": total, "uncertified": ncand, "near_midpoint_checked": checked})
    print(f"atan2 screen: {total} pairs, {ncand} through the double-double path, {checked} near-midpoint "
          f"pairs checked against glibc")
    assert checked > 100
