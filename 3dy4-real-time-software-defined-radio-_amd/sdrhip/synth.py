"""Seeded synthetic RF input.

Baseband FM at the mode-0 rate (Fs = 2.4 MS/s, src/project.cpp:180): message
0.8*sin(2*pi*1 kHz*t) + 0.1*sin(2*pi*19 kHz*t) (a tone plus a stereo pilot),
75 kHz peak deviation, carrier amplitude 0.7, AWGN sigma 0.02 per rail,
quantised to the RTL-SDR wire format: interleaved unsigned 8-bit I/Q,
u8 = clip(round(128*x + 128)).  The reference turns those bytes into floats
with (u - 128) / 128.0 (src/iofunc.cpp:117-119) and de-interleaves them
(src/project.cpp:78-81); ``planar_from_u8`` does the same.

The constant-envelope carrier keeps I^2+Q^2 well away from zero, where the
discriminator (src/filter.cpp:85-102) is well conditioned.
"""
from __future__ import annotations

import numpy as np

FS_MODE0 = 2.4e6


def fm_iq_u8(npairs: int, seed: int = 1234, fs: float = FS_MODE0, t0: int = 0,
             amp: float = 0.7, dev: float = 75e3, sigma: float = 0.02) -> np.ndarray:
    """Interleaved u8 IQ (length 2*npairs) of a noisy FM carrier."""
    rng = np.random.default_rng(seed)
    n = np.arange(t0, t0 + npairs, dtype=np.float64)
    t = n / fs
    # closed-form phase of the integrated message (no cumsum drift)
    w1, w2 = 2 * np.pi * 1e3, 2 * np.pi * 19e3
    phase = 2 * np.pi * dev * (0.8 * (1 - np.cos(w1 * t)) / w1 + 0.1 * (1 - np.cos(w2 * t)) / w2)
    i = amp * np.cos(phase) + sigma * rng.standard_normal(npairs)
    q = amp * np.sin(phase) + sigma * rng.standard_normal(npairs)
    out = np.empty(2 * npairs, np.float64)
    out[0::2] = i
    out[1::2] = q
    return np.clip(np.rint(128.0 * out + 128.0), 0, 255).astype(np.uint8)


def planar_from_u8(iq: np.ndarray):
    """(I, Q) float32 exactly as float((u-128)/128.0) + de-interleave."""
    v = ((iq.astype(np.int32) - 128).astype(np.float64) / 128.0).astype(np.float32)
    return np.ascontiguousarray(v[0::2]), np.ascontiguousarray(v[1::2])


def fm_planar(npairs: int, seed: int = 1234, **kw):
    return planar_from_u8(fm_iq_u8(npairs, seed=seed, **kw))
