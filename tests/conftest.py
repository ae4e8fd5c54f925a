"""Shared test plumbing.

Markers: ``gpu`` -- needs an MI355X (runs through libsdrhip.so); everything
else runs on CPU in a few minutes.  The oracle (oracle/, test infrastructure)
is imported only here and in the tests, as the checker.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "3dy4-real-time-software-defined-radio-_amd")
ORACLE_DIR = os.path.join(REPO, "oracle")
GOLDEN = os.path.join(REPO, "tests", "golden")
for p in (PKG, ORACLE_DIR):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (gfx950) GPU")


def _make(directory: str, *targets: str):
    subprocess.run(["make", "-s", "-C", directory, *targets], check=True, stdout=subprocess.DEVNULL)


@pytest.fixture(scope="session")
def oracle():
    from oracle import ORACLE_SO, Oracle

    if not os.path.exists(ORACLE_SO):
        _make(ORACLE_DIR)
    return Oracle()


@pytest.fixture(scope="session")
def built_lib():
    """libsdrhip.so + libdy4filter_hip.so + sdr_project, built in-tree if missing."""
    if not all(os.path.exists(os.path.join(PKG, f)) for f in ("libsdrhip.so", "libdy4filter_hip.so", "sdr_project")):
        _make(PKG, "-j4")
    import sdrhip

    return sdrhip


@pytest.fixture
def kswitch(built_lib):
    """kswitch(name, value): pick a kernel through sdr_set_switch (process-wide,
    include/sdr_hip.h) for one test; every switch it touched is restored after."""
    old = {}

    def set_(name, value):
        if name not in old:
            old[name] = built_lib.get_switch(name)
        built_lib.set_switch(name, int(value))

    yield set_
    for k, v in old.items():
        built_lib.set_switch(k, v)


@pytest.fixture(scope="session")
def manifest():
    with open(os.path.join(GOLDEN, "MANIFEST.json")) as f:
        return json.load(f)


def load_golden(name: str) -> dict:
    with np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False) as z:
        return {k: z[k] for k in z.files}


@pytest.fixture(scope="session")
def golden():
    return load_golden


@pytest.fixture(scope="session")
def gpu_ctx(built_lib):
    sdrhip = built_lib
    if sdrhip.device_count() < 1:
        pytest.fail("no GPU visible to libsdrhip.so (gpu-marked test run on a machine without an MI355X)")
    ctx = sdrhip.Context(0)
    yield ctx
    ctx.close()


@pytest.fixture(scope="session")
def harness(built_lib, tmp_path_factory):
    """tests/dropin_harness.cpp compiled against the drop-in library."""
    out = tmp_path_factory.mktemp("harness") / "dropin_harness"
    subprocess.run(["g++", "-O2", "-std=c++17", "-I", os.path.join(REPO, "include"),
                    os.path.join(REPO, "tests", "dropin_harness.cpp"), "-o", str(out),
                    "-L", PKG, "-ldy4filter_hip", "-lsdrhip", f"-Wl,-rpath,{PKG}", "-pthread"], check=True)
    return str(out)


def bits_equal(a, b) -> bool:
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    return a.shape == b.shape and np.array_equal(a.view(np.uint32), b.view(np.uint32))


def assert_bits(a, b, what=""):
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    assert a.shape == b.shape, f"{what}: shape {a.shape} != {b.shape}"
    if not np.array_equal(a.view(np.uint32), b.view(np.uint32)):
        bad = np.flatnonzero(a.view(np.uint32) != b.view(np.uint32))
        i = bad[0]
        raise AssertionError(f"{what}: {len(bad)} of {a.size} elements differ in bits; first at {i}: "
                             f"{a.flat[i]!r} vs {b.flat[i]!r}; max |diff| {np.nanmax(np.abs(a - b)):.3g}")


def assert_bits_nan(a, b, what=""):
    """Bitwise where `b` (the reference) is a number or an infinity, NaN exactly
    where it is NaN (payloads may differ: x86 and gfx950 quiet NaNs differ)."""
    a = np.ascontiguousarray(a, dtype=np.float32)
    b = np.ascontiguousarray(b, dtype=np.float32)
    assert a.shape == b.shape, f"{what}: shape {a.shape} != {b.shape}"
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        bad = np.flatnonzero(na != nb)
        raise AssertionError(f"{what}: NaN positions differ at {len(bad)} of {a.size} elements; first at {bad[0]}: "
                             f"{a.flat[bad[0]]!r} vs {b.flat[bad[0]]!r}")
    assert_bits(a[~nb], b[~nb], what)
