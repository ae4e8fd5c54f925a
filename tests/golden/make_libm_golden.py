#!/usr/bin/env python3
"""Fixtures for the device transcendental routines (csrc/libm_exact.hpp).

The reference's fmPLL stores (float) of glibc's double atan2 / sincos / cos on
float arguments (src/filter.cpp:199-221).  This script runs tests/libm_sweep.cpp
(g++, this container's glibc 2.35 -- the same image as the GPU box) and writes:

  libm_sincos.npz  every finite float (4,278,190,080 arguments):
                     hash[4096]  per-chunk u64 hashes of glibc's (sin, cos)
                                 floats (chunk = bits >> 20) -- the device
                                 test's reference for all 2^32 patterns;
                     near[k, 4]  every argument whose glibc double lies within
                                 4 double ulps of a float rounding midpoint:
                                 (argument bits, glibc sin float bits, glibc
                                 cos float bits, 1 = sin near | 2 = cos near);
                     meta        the sweep's JSON line (mismatches of
                                 libm_exact against glibc, and of the PLL's
                                 certified fast sine / cosine on |x| < 2^26:
                                 must be 0).
  libm_atan2.npz   2^34 seeded pairs (tests/libm_sweep.cpp's four families):
                     near[m, 3]  every pair whose glibc double lies within 4
                                 ulps of a float midpoint: (y, x, glibc float);
                     meta        the sweep's JSON line.

Run in the build container (takes about 12 minutes on 8 cores):
    python tests/golden/make_libm_golden.py
"""
from __future__ import annotations

import json
import os
import platform
import subprocess
import sys
import tempfile

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(os.path.dirname(HERE))
CSRC = os.path.join(ROOT, "3dy4-real-time-software-defined-radio-_amd", "csrc")
ATAN2_SEED = 20261018
ATAN2_LOG2 = 34


def build(tmp: str) -> str:
    exe = os.path.join(tmp, "libm_sweep")
    subprocess.run(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-pthread", "-I", CSRC, "-o", exe,
                    os.path.join(ROOT, "tests", "libm_sweep.cpp")], check=True)
    return exe


def main(threads: int = os.cpu_count() or 8, only: str = ""):
    libc = platform.libc_ver()
    with tempfile.TemporaryDirectory() as tmp:
        exe = build(tmp)
        if only != "atan2":
            sincos(exe, tmp, threads, libc)
        if only != "sincos":
            atan2(exe, tmp, threads, libc)


def sincos(exe, tmp, threads, libc):
    pre = os.path.join(tmp, "sc")
    line = subprocess.run([exe, "sincos", "0", "4096", str(threads), pre], check=True, capture_output=True,
                          text=True).stdout.strip()
    meta = json.loads(line)
    assert meta["sin_mismatch"] == 0 and meta["cos_mismatch"] == 0 and meta["sincos_vs_sin_cos"] == 0, meta
    assert meta["fast_certified_mismatch"] == 0, meta
    meta["glibc"] = "-".join(libc)
    h = np.fromfile(pre + ".hash", np.uint64)
    near = np.fromfile(pre + ".near", np.uint32).reshape(-1, 4)
    np.savez_compressed(os.path.join(HERE, "libm_sincos.npz"), hash=h, near=near,
                        meta=np.array(json.dumps(meta)))
    print("sincos", meta)


def atan2(exe, tmp, threads, libc):
    out = os.path.join(tmp, "at")
    line = subprocess.run([exe, "atan2", str(ATAN2_SEED), str(ATAN2_LOG2), str(threads), out], check=True,
                          capture_output=True, text=True).stdout.strip()
    meta = json.loads(line)
    assert meta["atan2_mismatch"] == 0, meta
    meta.update(glibc="-".join(libc), seed=ATAN2_SEED, log2_pairs=ATAN2_LOG2)
    near = np.fromfile(out, np.uint32).reshape(-1, 3)
    near = near[np.lexsort((near[:, 1], near[:, 0]))]
    np.savez_compressed(os.path.join(HERE, "libm_atan2.npz"), near=near, meta=np.array(json.dumps(meta)))
    print("atan2", meta)


if __name__ == "__main__":
    # usage: make_libm_golden.py [threads] [sincos|atan2]  (both by default)
    main(int(sys.argv[1]) if len(sys.argv) > 1 else (os.cpu_count() or 8), sys.argv[2] if len(sys.argv) > 2 else "")
