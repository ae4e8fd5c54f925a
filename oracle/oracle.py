"""ctypes front for the TEST-ONLY checkers in oracle/.

* ``Oracle``    -- liboracle.so, the C restatement of src/filter.cpp
                   (oracle/sdr_oracle.c).
* ``Reference`` -- oracle/_ref/libref_filter.so, the reference's own
                   src/filter.cpp compiled from /root/reference by
                   ``make -C oracle ref`` (only present where it was built).

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg import
this module.  The product path (the HIP library and its bindings) never does.
Both classes expose the same numpy-level methods, mirroring the reference's
std::vector API: outputs are returned, in/out state arrays are updated in
place (they must be contiguous float32 numpy arrays).
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
ORACLE_SO = os.path.join(HERE, "liboracle.so")
REF_SO = os.path.join(HERE, "_ref", "libref_filter.so")

_fp = C.POINTER(C.c_float)
_u8p = C.POINTER(C.c_ubyte)
_L = C.c_long


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def _p(a: np.ndarray):
    return a.ctypes.data_as(_fp)


def _check_state(s):
    if not (isinstance(s, np.ndarray) and s.dtype == np.float32 and s.flags.c_contiguous):
        raise TypeError("state must be a contiguous float32 numpy array (updated in place)")


class _Lib:
    """Shared numpy wrappers; subclasses bind symbol names."""

    prefix = ""

    def __init__(self, path: str):
        if not os.path.exists(path):
            raise FileNotFoundError(f"{path} not built (run `make -C oracle` / `make -C oracle ref`)")
        self.path = path
        self.lib = C.CDLL(path)
        for name in ("taps_lpf", "taps_bpf", "convolve_full", "fir_block", "fir_decim", "resample",
                     "fm_demod", "downsample", "upsample", "fm_pll", "delay_block", "pointwise_mul",
                     "pointwise_add", "pointwise_sub", "interleave"):
            getattr(self.lib, self.prefix + name).restype = _L

    def _fn(self, name):
        return getattr(self.lib, self.prefix + name)

    # -- taps (src/filter.cpp:14-49)
    def taps_lpf(self, Fs, Fc, ntaps, up=1):
        h = np.zeros(ntaps, np.float32)
        self._fn("taps_lpf")(C.c_float(Fs), C.c_float(Fc), C.c_ushort(ntaps), C.c_int(up), _p(h))
        return h

    def taps_bpf(self, Fs, Fb, Fe, ntaps, up=1):
        h = np.zeros(ntaps, np.float32)
        self._fn("taps_bpf")(C.c_float(Fs), C.c_float(Fb), C.c_float(Fe), C.c_ushort(ntaps), C.c_int(up), _p(h))
        return h

    # -- convolutions (src/filter.cpp:53-83, 123-173)
    def convolve_full(self, x, h):
        x, h = _f32(x), _f32(h)
        y = np.zeros(len(x) + len(h) - 1, np.float32)
        self._fn("convolve_full")(_p(x), _L(len(x)), _p(h), C.c_int(len(h)), _p(y))
        return y

    def fir_block(self, x, h, state):
        x, h = _f32(x), _f32(h)
        _check_state(state)
        y = np.zeros(len(x), np.float32)
        rc = self._fn("fir_block")(_p(x), _L(len(x)), _p(h), C.c_int(len(h)), _p(state), C.c_int(len(state)), _p(y))
        if rc < 0:
            raise ValueError("fir_block precondition")
        return y

    def fir_decim(self, D, x, h, state):
        x, h = _f32(x), _f32(h)
        _check_state(state)
        y = np.zeros(len(x) // D, np.float32)
        rc = self._fn("fir_decim")(C.c_int(D), _p(x), _L(len(x)), _p(h), C.c_int(len(h)), _p(state),
                                   C.c_int(len(state)), _p(y))
        if rc < 0:
            raise ValueError("fir_decim precondition")
        return y

    def resample(self, up, down, x, h, state):
        x, h = _f32(x), _f32(h)
        _check_state(state)
        ny = int(np.float32(np.float32(len(x)) / np.float32(down)) * np.float32(up))
        y = np.zeros(max(ny, 1), np.float32)
        rc = self._fn("resample")(C.c_int(up), C.c_int(down), _p(x), _L(len(x)), _p(h), C.c_int(len(h)),
                                  _p(state), C.c_int(len(state)), _p(y))
        if rc < 0:
            raise ValueError("resample precondition")
        return y[:ny]

    def fm_demod(self, I, Q, prev):
        """prev: float32 array [prev_I, prev_Q], updated in place."""
        I, Q = _f32(I), _f32(Q)
        _check_state(prev)
        out = np.zeros(len(I), np.float32)
        pi, pq = C.c_float(prev[0]), C.c_float(prev[1])
        self._fn("fm_demod")(_p(I), _p(Q), _L(len(I)), C.byref(pi), C.byref(pq), _p(out))
        prev[0], prev[1] = pi.value, pq.value
        return out

    def downsample(self, x, factor):
        x = _f32(x)
        out = np.zeros(-(-len(x) // factor) if len(x) else 1, np.float32)
        m = self._fn("downsample")(_p(x), _L(len(x)), _L(factor), _p(out))
        return out[:m]

    def upsample(self, x, factor):
        x = _f32(x)
        out = np.zeros(max(len(x) * max(factor, 1), 1), np.float32)
        m = self._fn("upsample")(_p(x), _L(len(x)), _L(factor), _p(out))
        return out[:m]

    def fm_pll(self, x, freq, Fs, nco_scale, phase_adjust, norm_bw, pll):
        """pll: float32[6] {feedbackI, feedbackQ, integrator, phaseEst, trigOffset, nco_state}, in place."""
        x = _f32(x)
        _check_state(pll)
        out = np.zeros(len(x), np.float32)
        self._fn("fm_pll")(_p(x), _L(len(x)), C.c_float(freq), C.c_float(Fs), C.c_float(nco_scale),
                           C.c_float(phase_adjust), C.c_float(norm_bw), _p(out), _p(pll))
        return out

    def delay_block(self, x, state):
        x = _f32(x)
        _check_state(state)
        out = np.zeros(len(x), np.float32)
        self._fn("delay_block")(_p(x), _L(len(x)), _p(state), C.c_int(len(state)), _p(out))
        return out

    def _pw(self, name, a, b, n):
        a, b = _f32(a), _f32(b)
        out = np.zeros(max(n, 1), np.float32)
        m = self._fn(name)(_p(a), _L(len(a)), _p(b), _L(len(b)), _p(out))
        return out[:m]

    def pointwise_mul(self, a, b):
        return self._pw("pointwise_mul", a, b, min(len(a), len(b)))

    def pointwise_add(self, a, b):
        return self._pw("pointwise_add", a, b, len(a))

    def pointwise_sub(self, a, b):
        return self._pw("pointwise_sub", a, b, len(a))

    def interleave(self, l, r):
        l, r = _f32(l), _f32(r)
        out = np.zeros(max(len(l) + len(r), 1), np.float32)
        m = self._fn("interleave")(_p(l), _L(len(l)), _p(r), _L(len(r)), _p(out))
        return out[:m]

    # -- the front end as src/project.cpp:86-90 sequences it
    def frontend(self, D, I, Q, h, state_i, state_q, prev):
        yi = self.fir_decim(D, I, h, state_i)
        yq = self.fir_decim(D, Q, h, state_q)
        return self.fm_demod(yi, yq, prev)


class Oracle(_Lib):
    """The C restatement (oracle/sdr_oracle.c)."""

    prefix = "or_"

    def __init__(self, path: str = ORACLE_SO):
        super().__init__(path)
        self.lib.or_resample_len.restype = _L
        self.lib.or_u8_to_planar.restype = _L
        self.lib.or_pcm_s16.restype = _L

    def resample_len(self, up, down, nx):
        return int(self.lib.or_resample_len(C.c_int(up), C.c_int(down), _L(nx)))

    def u8_to_planar(self, iq):
        iq = np.ascontiguousarray(iq, dtype=np.uint8)
        n = len(iq) // 2
        I = np.zeros(n, np.float32)
        Q = np.zeros(n, np.float32)
        self.lib.or_u8_to_planar(iq.ctypes.data_as(_u8p), _L(n), _p(I), _p(Q))
        return I, Q

    def pcm_s16(self, x):
        """src/project.cpp:311-314: NaN -> 0, else (short)(x * 16384)."""
        x = _f32(x)
        out = np.zeros(max(len(x), 1), np.int16)
        self._fn("pcm_s16")(_p(x), _L(len(x)), out.ctypes.data_as(C.c_void_p))
        return out[:len(x)]

    def mono(self, D, iq, h_rf, st_i, st_q, prev, delay_state, up, down, h_audio, st_audio):
        """src/project.cpp:72-118 + 304-314 for one mono block: u8 IQ -> s16 PCM."""
        I, Q = self.u8_to_planar(iq)
        demod = self.frontend(D, I, Q, h_rf, st_i, st_q, prev)
        delayed = self.delay_block(demod, delay_state)
        audio = self.resample(up, down, delayed, h_audio, st_audio)
        return self.pcm_s16(audio)


    def stereo(self, D, iq, h_rf, st, up, down, h_audio, h_pilot, h_stereo, audio_fs):
        """src/project.cpp:72-132 + 304-314 for one stereo block: u8 IQ ->
        interleaved s16 L/R.  st: dict of float32 state arrays (i, q, prev[2],
        delay, audio, pilot, stereo, stereo_lp, pll[6]), updated in place."""
        I, Q = self.u8_to_planar(iq)
        demod = self.frontend(D, I, Q, h_rf, st["i"], st["q"], st["prev"])
        mono = self.resample(up, down, self.delay_block(demod, st["delay"]), h_audio, st["audio"])
        pilot = self.fir_block(demod, h_pilot, st["pilot"])
        sband = self.fir_block(demod, h_stereo, st["stereo"])
        nco = self.fm_pll(pilot, 19e3, audio_fs, 2.0, 0.0, 0.01, st["pll"])  # src/project.cpp:100-104,123
        slp = self.resample(up, down, self.pointwise_mul(nco, sband), h_audio, st["stereo_lp"])
        left, right = self.pointwise_add(mono, slp), self.pointwise_sub(mono, slp)
        return self.pcm_s16(self.interleave(left, right))


class Reference(_Lib):
    """The reference's own src/filter.cpp, compiled (oracle/_ref)."""

    prefix = "ref_"

    def __init__(self, path: str = REF_SO):
        super().__init__(path)
        self.lib.ref_front_new.restype = C.c_void_p
        self.lib.ref_front_new.argtypes = [_fp, C.c_int, C.c_int]
        self.lib.ref_front_free.argtypes = [C.c_void_p]
        self.lib.ref_front_run.restype = _L
        self.lib.ref_front_run.argtypes = [C.c_void_p, C.c_int, _fp, _fp, _L, _fp]

    def frontend_runner(self, h, ns):
        """Persistent-state front end (timed by the CPU baseline)."""
        h = _f32(h)
        handle = self.lib.ref_front_new(_p(h), len(h), ns)
        lib = self.lib

        class _Runner:
            def run(self, D, I, Q, demod=None):
                return lib.ref_front_run(handle, D, _p(I), _p(Q), len(I), _p(demod) if demod is not None else None)

            def close(self):
                lib.ref_front_free(handle)

        return _Runner()


def available_reference() -> bool:
    return os.path.exists(REF_SO)
