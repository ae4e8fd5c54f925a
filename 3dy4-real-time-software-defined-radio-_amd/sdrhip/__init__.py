"""Python binding of libsdrhip.so (the C ABI in include/sdr_hip.h).

This is the host-side face of the MI355X RF front end for tests, the
benchmark and Python callers; C/C++ callers use the C ABI or the drop-in
filter.h implementation (host/filter_hip.cpp) directly.

Two layers, mirroring the C ABI:

* ``Context`` host-array methods (``fir_decim``, ``fir_block``,
  ``resample``, ``fm_demod``, ``frontend``, ``frontend_u8``) -- numpy in,
  numpy out, one block of one stream, state arrays updated in place: the
  reference's filter.h contract (src/filter.cpp).
* ``Context`` ``*_dev`` methods -- device-resident and batched: arguments are
  device pointers (ints) or objects exposing ``data_ptr()`` (torch tensors
  on the GPU).  They enqueue on the context's stream and return at once.

There is no CPU fallback anywhere: if the shared library is missing or no
GPU is present, constructing a Context raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG_DIR = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
# SDRHIP_LIB: another build of the same C ABI (A/B timing of kernel
# revisions, scripts/build_ab.sh); the in-tree library otherwise.
LIB_PATH = os.environ.get("SDRHIP_LIB") or os.path.join(PKG_DIR, "libsdrhip.so")
DROPIN_PATH = os.path.join(PKG_DIR, "libdy4filter_hip.so")
REPO_DIR = os.path.dirname(PKG_DIR)
HEADER_PATH = os.path.join(REPO_DIR, "include", "sdr_hip.h")

SDR_OK, SDR_EINVAL, SDR_EHIP, SDR_ENOMEM, SDR_ENODEV = 0, -1, -2, -3, -4
ARITH_EXACT, ARITH_FMA = 0, 1  # sdr_ctx_set_arith modes
FORK_AUTO, FORK_SERIAL, FORK_SIDE = -1, 0, 1  # sdr_ctx_set_stereo_fork modes

_lib = None

_vp = C.c_void_p
_fp = C.POINTER(C.c_float)
_ll = C.c_longlong
_i = C.c_int

# name -> argtypes (restype int unless listed in _RESTYPE)
_SIGS = {
    "sdr_version": [],
    "sdr_abi_version": [],
    "sdr_strerror": [_i],
    "sdr_device_count": [C.POINTER(_i)],
    "sdr_set_switch": [C.c_char_p, _i],
    "sdr_get_switch": [C.c_char_p, C.POINTER(_i)],
    "sdr_ctx_create": [_i, C.POINTER(_vp)],
    "sdr_ctx_destroy": [_vp],
    "sdr_ctx_set_stream": [_vp, _vp],
    "sdr_ctx_get_stream": [_vp],
    "sdr_ctx_synchronize": [_vp],
    "sdr_ctx_set_arith": [_vp, _i],
    "sdr_ctx_set_stereo_fork": [_vp, _i],
    "sdr_ctx_pin_scratch": [_vp, _i],
    "sdr_ctx_last_error": [_vp],
    "sdr_dev_alloc": [_vp, C.c_size_t, C.POINTER(_vp)],
    "sdr_dev_free": [_vp, _vp],
    "sdr_copy_h2d": [_vp, _vp, _vp, C.c_size_t],
    "sdr_copy_d2h": [_vp, _vp, _vp, C.c_size_t],
    "sdr_dev_memset": [_vp, _vp, _i, C.c_size_t],
    "sdr_host_alloc": [_vp, C.c_size_t, C.POINTER(_vp)],
    "sdr_host_free": [_vp, _vp],
    "sdr_copy_h2d_async": [_vp, _vp, _vp, C.c_size_t],
    "sdr_copy_d2h_async": [_vp, _vp, _vp, C.c_size_t],
    "sdr_event_create": [_vp, C.POINTER(_vp)],
    "sdr_event_record": [_vp, _vp],
    "sdr_event_synchronize": [_vp, _vp],
    "sdr_event_destroy": [_vp, _vp],
    "sdr_ctx_wait_event": [_vp, _vp],
    "sdr_graph_begin": [_vp],
    "sdr_graph_end": [_vp, C.POINTER(_vp)],
    "sdr_graph_launch": [_vp, _vp],
    "sdr_graph_destroy": [_vp, _vp],
    "sdr_resample_out_len": [_i, _i, _ll],
    "sdr_taps_lpf": [C.c_float, C.c_float, _i, _i, _vp],
    "sdr_taps_bpf": [C.c_float, C.c_float, C.c_float, _i, _i, _vp],
    "sdr_fir_block_f32": [_vp, _vp, _ll, _vp, _i, _vp, _i, _vp],
    "sdr_fir_decim_f32": [_vp, _i, _vp, _ll, _vp, _i, _vp, _i, _vp],
    "sdr_resample_f32": [_vp, _i, _i, _vp, _ll, _vp, _i, _vp, _i, _vp, _ll],
    "sdr_fm_demod_f32": [_vp, _vp, _vp, _ll, _vp, _vp, _vp],
    "sdr_frontend_f32": [_vp, _i, _vp, _vp, _ll, _vp, _i, _vp, _vp, _i, _vp, _vp, _vp],
    "sdr_frontend_u8": [_vp, _i, _vp, _ll, _vp, _i, _vp, _vp, _i, _vp, _vp, _vp],
    "sdr_fir_decim_f32_dev": [_vp, _i, _vp, _ll, _i, _ll, _vp, _i, _vp, _i, _vp, _ll],
    "sdr_fir_block_f32_dev": [_vp, _vp, _ll, _i, _ll, _vp, _i, _vp, _i, _vp, _ll],
    "sdr_fm_demod_f32_dev": [_vp, _vp, _vp, _ll, _i, _ll, _vp, _vp, _vp, _ll],
    "sdr_frontend_f32_dev": [_vp, _i, _vp, _vp, _ll, _i, _ll, _vp, _i, _vp, _vp, _i, _vp, _vp, _vp, _ll],
    "sdr_frontend_u8_dev": [_vp, _i, _vp, _ll, _i, _ll, _vp, _i, _vp, _vp, _i, _vp, _vp, _vp, _ll],
    "sdr_resample_f32_dev": [_vp, _i, _i, _vp, _ll, _i, _ll, _vp, _i, _vp, _i, _vp, _ll],
    "sdr_resample_plan_create": [_vp, _i, _i, _vp, _i, C.POINTER(_vp)],
    "sdr_resample_plan_f32_dev": [_vp, _vp, _vp, _ll, _i, _ll, _vp, _i, _vp, _ll],
    "sdr_resample_plan_destroy": [_vp, _vp],
    "sdr_fir_block_f16_dev": [_vp, _vp, _ll, _i, _ll, _vp, _i, _vp, _i, _vp, _ll],
    "sdr_fir_f16_plan_create": [_vp, _vp, _i, C.POINTER(_vp)],
    "sdr_fir_block_f16_plan_dev": [_vp, _vp, _vp, _ll, _i, _ll, _vp, _i, _vp, _ll],
    "sdr_fir_f16_plan_destroy": [_vp, _vp],
    "sdr_f32_to_f16_dev": [_vp, _vp, _ll, _vp],
    "sdr_fir_block_f16_kernel": [_i],
    "sdr_delay_f32_dev": [_vp, _vp, _ll, _i, _ll, _vp, _i, _vp, _ll],
    "sdr_pcm_s16_dev": [_vp, _vp, _ll, _i, _ll, _vp, _ll],
    "sdr_mono_pcm_u8_dev": [_vp, _i, _vp, _ll, _i, _ll, _vp, _i, _vp, _vp, _i, _vp, _vp, _vp, _i, _i, _i, _vp, _i,
                            _vp, _i, _vp, _ll],
    "sdr_fm_pll_dev": [_vp, _vp, _ll, _i, _ll, C.c_float, C.c_float, C.c_float, C.c_float, C.c_float, _vp, _vp,
                       _ll, _vp, _ll],
    "sdr_stereo_pcm_dev": [_vp, _vp, _vp, _ll, _i, _ll, _vp, _ll],
    "sdr_stereo_pcm_u8_dev": [_vp, _i, _vp, _ll, _i, _ll, _i, _i, C.c_float, _vp, _vp, _vp, _ll],
    "sdr_stereo_work_create": [_vp, _i, _ll, _i, _i, _i, C.POINTER(_vp)],
    "sdr_stereo_work_destroy": [_vp, _vp],
    "sdr_stereo_front_u8_dev": [_vp, _vp, _ll, _vp, _vp, _vp],
    "sdr_stereo_back_dev": [_vp, C.c_float, _vp, _vp, _vp, _vp, _ll],
    "sdr_stereo_pll_dev": [_vp, C.c_float, _vp, _vp],
    "sdr_stereo_post_dev": [_vp, _vp, _vp, _vp, _vp, _ll],
    "sdr_synth_fm_u8_dev": [_vp, _vp, _ll, _i, _ll, C.c_ulonglong],
    "sdr_u8_to_planar_dev": [_vp, _vp, _ll, _i, _ll, _vp, _vp, _ll],
    "sdr_mono_work_create": [_vp, _i, _ll, _i, _i, _i, _i, _vp, _i, _i, _vp, _i, _i, C.POINTER(_vp)],
    "sdr_mono_work_destroy": [_vp, _vp],
    "sdr_mono_front_u8_dev": [_vp, _vp, _ll, _vp, _i, _vp, _vp, _i, _vp, _vp, _vp],
    "sdr_mono_back_dev": [_vp, _vp, _i, _vp, _i, _vp, _vp, _vp, _ll],
    "sdr_libm_sincos_hash_dev": [_vp, _i, C.c_uint, C.c_uint, _vp],
    "sdr_libm_sincos_diff_dev": [_vp, C.c_uint, C.c_uint, _vp, _vp, _ll],
    "sdr_libm_eval_dev": [_vp, _i, _vp, _vp, _ll, _vp],
    "sdr_libm_atan2_screen_dev": [_vp, C.c_ulonglong, C.c_ulonglong, C.c_ulonglong, _vp, _ll, _vp, _ll, _vp],
}
_RESTYPE = {"sdr_version": C.c_char_p, "sdr_strerror": C.c_char_p, "sdr_ctx_last_error": C.c_char_p,
            "sdr_ctx_get_stream": _vp, "sdr_resample_out_len": _ll}

EXPORTED = tuple(_SIGS)


class StereoTaps(C.Structure):
    """include/sdr_hip.h sdr_stereo_taps (device pointers)."""
    _fields_ = [("h_rf", _vp), ("rf_taps", _i), ("h_audio", _vp), ("audio_taps", _i), ("h_pilot", _vp),
                ("h_stereo", _vp), ("bpf_taps", _i)]


class StereoState(C.Structure):
    """include/sdr_hip.h sdr_stereo_state (device pointers, one row per stream)."""
    _fields_ = [("state_i", _vp), ("state_q", _vp), ("ns_rf", _i), ("prev_i", _vp), ("prev_q", _vp),
                ("delay_state", _vp), ("ns_delay", _i), ("state_audio", _vp), ("stereo_lp_state", _vp),
                ("ns_audio", _i), ("pilot_state", _vp), ("stereo_state", _vp), ("ns_bpf", _i), ("pll", _vp)]


class SdrError(RuntimeError):
    def __init__(self, code: int, where: str, detail: str = ""):
        self.code = code
        super().__init__(f"{where}: {lib().sdr_strerror(code).decode()} ({detail})")


ABI_VERSION = 3  # include/sdr_hip.h SDR_ABI_VERSION this binding was written for


def lib() -> C.CDLL:
    """Load libsdrhip.so (raises if it was not built -- no fallback -- or if
    its ABI version is not the one this binding was written for)."""
    global _lib
    if _lib is None:
        if not os.path.exists(LIB_PATH):
            raise ImportError(f"{LIB_PATH} missing: build it (python -c 'import __graft_entry__ as g; g.build()')")
        L = C.CDLL(LIB_PATH)
        # an explicitly named library (SDRHIP_LIB: a same-box A/B build of an
        # older tree) may predate entry points; the shipped one may not
        ab = bool(os.environ.get("SDRHIP_LIB"))
        if hasattr(L, "sdr_abi_version"):
            L.sdr_abi_version.restype = _i
            if L.sdr_abi_version() != ABI_VERSION and not ab:
                raise ImportError(f"{LIB_PATH} has ABI {L.sdr_abi_version()}, this binding needs {ABI_VERSION}: rebuild")
        elif not ab:
            raise ImportError(f"{LIB_PATH} has no sdr_abi_version (an older build): rebuild")
        for name, args in _SIGS.items():
            if ab and not hasattr(L, name):
                continue
            f = getattr(L, name)
            f.argtypes = args
            f.restype = _RESTYPE.get(name, _i)
        _lib = L
    return _lib


def version() -> str:
    return lib().sdr_version().decode()


SWITCHES = ("SDR_FIR_SC", "SDR_FIR_SC_U8", "SDR_RESAMPLE_LP", "SDR_RESAMPLE_LOADER", "SDR_RESAMPLE_RS",
            "SDR_RESAMPLE_PP", "SDR_LONG_VTAP", "SDR_F16_MFMA", "SDR_F16_HEAD", "SDR_F16_W8", "SDR_PLL_FAST",
            "SDR_PLL_GUARD", "SDR_LONG_COMMIT")


def set_switch(name: str, value: int) -> None:
    """sdr_set_switch: pick one of several bit-identical kernels, process-wide
    (include/sdr_hip.h); applies to launches enqueued after the call."""
    if lib().sdr_set_switch(name.encode(), int(value)) != SDR_OK:
        raise ValueError(f"unknown kernel switch {name!r}")


def get_switch(name: str) -> int:
    v = _i(0)
    if lib().sdr_get_switch(name.encode(), C.byref(v)) != SDR_OK:
        raise ValueError(f"unknown kernel switch {name!r}")
    return v.value


class switches:
    """Context manager: set kernel switches for a block, restore them after."""

    def __init__(self, **values):
        self._new = {k: int(v) for k, v in values.items()}
        self._old = {}

    def __enter__(self):
        for k, v in self._new.items():
            self._old[k] = get_switch(k)
            set_switch(k, v)
        return self

    def __exit__(self, *exc):
        for k, v in self._old.items():
            set_switch(k, v)


def device_count() -> int:
    n = _i(0)
    lib().sdr_device_count(C.byref(n))
    return n.value


def resample_out_len(up: int, down: int, n: int) -> int:
    """(size_t)((n / (float)down) * up) -- src/filter.cpp:149."""
    return int(lib().sdr_resample_out_len(up, down, n))


def taps_lpf(Fs: float, Fc: float, ntaps: int, up: int = 1) -> np.ndarray:
    """impulseResponseLPF (src/filter.cpp:14-29), bit-identical."""
    h = np.empty(ntaps, np.float32)
    if lib().sdr_taps_lpf(Fs, Fc, ntaps, up, h.ctypes.data) != SDR_OK:
        raise ValueError("bad tap design arguments")
    return h


def taps_bpf(Fs: float, Fb: float, Fe: float, ntaps: int, up: int = 1) -> np.ndarray:
    """impulseResponseBPF (src/filter.cpp:31-49), bit-identical."""
    h = np.empty(ntaps, np.float32)
    if lib().sdr_taps_bpf(Fs, Fb, Fe, ntaps, up, h.ctypes.data) != SDR_OK:
        raise ValueError("bad tap design arguments")
    return h


def _ptr(x) -> int:
    if x is None:
        return 0
    if isinstance(x, int):
        return x
    if hasattr(x, "data_ptr"):
        return int(x.data_ptr())
    if isinstance(x, np.ndarray):
        return int(x.ctypes.data)
    raise TypeError(f"cannot take a device pointer of {type(x)!r}")


def _f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def _inplace(a, what):
    if not (isinstance(a, np.ndarray) and a.dtype == np.float32 and a.flags.c_contiguous and a.flags.writeable):
        raise TypeError(f"{what} must be a writeable contiguous float32 numpy array (updated in place)")
    return a


class Graph:
    """An instantiated capture (sdr_graph): launch() replays it."""

    def __init__(self, ctx: "Context", g):
        self._ctx, self._g = ctx, g

    def launch(self):
        self._ctx._check(lib().sdr_graph_launch(self._ctx._c, self._g), "graph_launch")

    def close(self):
        if self._g and self._ctx._c:
            lib().sdr_graph_destroy(self._ctx._c, self._g)
        self._g = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class ResamplePlan:
    """sdr_resample_plan: resample_dev with the tap tables built once."""

    def __init__(self, ctx: "Context", p):
        self._ctx, self._p = ctx, p

    def resample_dev(self, x, n, nstreams, x_stride, state, ns, y, y_stride):
        self._ctx._check(lib().sdr_resample_plan_f32_dev(self._ctx._c, self._p, _ptr(x), n, nstreams, x_stride,
                                                         _ptr(state), ns, _ptr(y), y_stride), "resample_plan_dev")

    def close(self):
        if self._p:
            lib().sdr_resample_plan_destroy(self._ctx._c, self._p)
            self._p = _vp()


class F16Plan:
    """sdr_fir_f16_plan: fir_block_f16_dev with the MFMA kernel's tap copies built once."""

    def __init__(self, ctx: "Context", p):
        self._ctx, self._p = ctx, p

    def fir_block_f16_dev(self, x, n, nstreams, x_stride, state, ns, y, y_stride):
        self._ctx._check(lib().sdr_fir_block_f16_plan_dev(self._ctx._c, self._p, _ptr(x), n, nstreams, x_stride,
                                                          _ptr(state), ns, _ptr(y), y_stride), "fir_block_f16_plan_dev")

    def close(self):
        if self._p:
            lib().sdr_fir_f16_plan_destroy(self._ctx._c, self._p)
            self._p = _vp()


class Event:
    """sdr_event: marks the work enqueued on a context's stream so far."""

    def __init__(self, ctx: "Context"):
        self._ctx, self._e = ctx, _vp()
        ctx._check(lib().sdr_event_create(ctx._c, C.byref(self._e)), "event_create")

    def record(self, ctx: "Context"):
        ctx._check(lib().sdr_event_record(ctx._c, self._e), "event_record")

    def wait(self, ctx: "Context"):
        """ctx's stream waits (on the device) for the recorded work (sdr_ctx_wait_event)."""
        ctx._check(lib().sdr_ctx_wait_event(ctx._c, self._e), "ctx_wait_event")

    def synchronize(self):
        self._ctx._check(lib().sdr_event_synchronize(self._ctx._c, self._e), "event_synchronize")

    def close(self):
        if self._e and self._ctx._c:
            lib().sdr_event_destroy(self._ctx._c, self._e)
        self._e = _vp()


class StereoWork:
    """sdr_stereo_work: intermediates of one block for stereo_front/back."""

    def __init__(self, ctx: "Context", w):
        self._ctx, self._w = ctx, w

    def close(self):
        if self._w and self._ctx._c:
            lib().sdr_stereo_work_destroy(self._ctx._c, self._w)
        self._w = _vp()


class MonoWork:
    """sdr_mono_work: one block's demodulated row for mono_front/back."""

    def __init__(self, ctx: "Context", w):
        self._ctx, self._w = ctx, w

    def close(self):
        if self._w and self._ctx._c:
            lib().sdr_mono_work_destroy(self._ctx._c, self._w)
        self._w = _vp()


class Context:
    """One GPU + one HIP stream + scratch buffers (sdr_ctx)."""

    def __init__(self, device: int = 0):
        self._c = _vp()
        rc = lib().sdr_ctx_create(device, C.byref(self._c))
        if rc != SDR_OK:
            raise SdrError(rc, f"sdr_ctx_create({device})")
        self.device = device

    # -- lifetime / stream
    def close(self):
        if self._c:
            lib().sdr_ctx_destroy(self._c)
            self._c = _vp()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def __enter__(self):
        return self

    def __exit__(self, *exc):
        self.close()

    def set_arith(self, mode: int):
        """FIR arithmetic of the fused front end: ARITH_EXACT (the reference's
        bits, default) or ARITH_FMA (one fused multiply-add per tap)."""
        self._check(lib().sdr_ctx_set_arith(self._c, mode), "set_arith")

    def set_stereo_fork(self, mode: int):
        """stereo_pcm_u8_dev's launch order: FORK_AUTO (side branch on a
        second stream at <= CUs/4 PLL waves), FORK_SERIAL or FORK_SIDE."""
        self._check(lib().sdr_ctx_set_stereo_fork(self._c, mode), "set_stereo_fork")

    def pin_scratch(self, pinned: bool = True):
        """Refuse scratch growth (SDR_EINVAL) while pinned: for graphs the
        caller captures itself on this context's stream (sdr_ctx_pin_scratch)."""
        self._check(lib().sdr_ctx_pin_scratch(self._c, int(bool(pinned))), "pin_scratch")

    def set_stream(self, hip_stream: int | None):
        """Use an external hipStream_t (e.g. torch.cuda.current_stream().cuda_stream)."""
        self._check(lib().sdr_ctx_set_stream(self._c, hip_stream or None), "set_stream")

    @property
    def stream(self) -> int:
        return lib().sdr_ctx_get_stream(self._c) or 0

    def synchronize(self):
        self._check(lib().sdr_ctx_synchronize(self._c), "synchronize")

    # -- HIP-graph capture of this context's stream (sdr_graph_*)
    def capture(self, fn) -> "Graph":
        """Record the stream-ordered calls `fn()` makes on this context into
        a HIP graph (nothing runs while recording); Graph.launch() replays
        them on the context's stream."""
        self._check(lib().sdr_graph_begin(self._c), "graph_begin")
        g = _vp()
        try:
            fn()
        finally:
            rc = lib().sdr_graph_end(self._c, C.byref(g))
        self._check(rc, "graph_end")
        return Graph(self, g)

    def last_error(self) -> str:
        return lib().sdr_ctx_last_error(self._c).decode()

    def _check(self, rc: int, where: str):
        if rc != SDR_OK:
            raise SdrError(rc, where, self.last_error())

    # -- host arrays, one block (filter.h contract) ----------------------
    def fir_block(self, x, h, state):
        """blockConvolveFIR (src/filter.cpp:66-83)."""
        x, h, state = _f32(x), _f32(h), _inplace(state, "state")
        y = np.empty(len(x), np.float32)
        self._check(lib().sdr_fir_block_f32(self._c, _ptr(x), len(x), _ptr(h), len(h), _ptr(state), len(state),
                                            _ptr(y)), "fir_block")
        return y

    def fir_decim(self, D, x, h, state):
        """downsampleBlockConvolveFIR (src/filter.cpp:123-140)."""
        x, h, state = _f32(x), _f32(h), _inplace(state, "state")
        y = np.empty(max(len(x) // max(D, 1), 1), np.float32)
        self._check(lib().sdr_fir_decim_f32(self._c, D, _ptr(x), len(x), _ptr(h), len(h), _ptr(state),
                                            len(state), _ptr(y)), "fir_decim")
        return y[:len(x) // D]

    def resample(self, up, down, x, h, state):
        """resampleBlockConvolveFIR (src/filter.cpp:142-173)."""
        x, h, state = _f32(x), _f32(h), _inplace(state, "state")
        ny = resample_out_len(up, down, len(x))
        y = np.empty(max(ny, 1), np.float32)
        self._check(lib().sdr_resample_f32(self._c, up, down, _ptr(x), len(x), _ptr(h), len(h), _ptr(state),
                                           len(state), _ptr(y), max(ny, 0)), "resample")
        return y[:ny]

    def fm_demod(self, I, Q, prev):
        """fmDemodArctan (src/filter.cpp:85-102); prev = float32[2] {prev_I, prev_Q}, in place."""
        I, Q, prev = _f32(I), _f32(Q), _inplace(prev, "prev")
        out = np.empty(max(len(I), 1), np.float32)
        pv = prev.ctypes.data
        self._check(lib().sdr_fm_demod_f32(self._c, _ptr(I), _ptr(Q), len(I), pv, pv + 4, _ptr(out)), "fm_demod")
        return out[:len(I)]

    def frontend(self, D, I, Q, h, state_i, state_q, prev):
        """Fused src/project.cpp:86-90 in one launch; returns the demodulated block."""
        I, Q, h = _f32(I), _f32(Q), _f32(h)
        _inplace(state_i, "state_i"), _inplace(state_q, "state_q"), _inplace(prev, "prev")
        out = np.empty(max(len(I) // max(D, 1), 1), np.float32)
        pv = prev.ctypes.data
        self._check(lib().sdr_frontend_f32(self._c, D, _ptr(I), _ptr(Q), len(I), _ptr(h), len(h), _ptr(state_i),
                                           _ptr(state_q), len(state_i), pv, pv + 4, _ptr(out)), "frontend")
        return out[:len(I) // D]

    def frontend_u8(self, D, iq, h, state_i, state_q, prev):
        """Fused front end straight from interleaved u8 IQ (src/iofunc.cpp:117-119 folded in)."""
        iq = np.ascontiguousarray(iq, dtype=np.uint8)
        h = _f32(h)
        _inplace(state_i, "state_i"), _inplace(state_q, "state_q"), _inplace(prev, "prev")
        npairs = len(iq) // 2
        out = np.empty(max(npairs // max(D, 1), 1), np.float32)
        pv = prev.ctypes.data
        self._check(lib().sdr_frontend_u8(self._c, D, _ptr(iq), npairs, _ptr(h), len(h), _ptr(state_i),
                                          _ptr(state_q), len(state_i), pv, pv + 4, _ptr(out)), "frontend_u8")
        return out[:npairs // D]

    # -- device pointers, batched ------------------------------------------
    def fir_decim_dev(self, D, x, n, nstreams, x_stride, h, ntaps, state, ns, y, y_stride):
        self._check(lib().sdr_fir_decim_f32_dev(self._c, D, _ptr(x), n, nstreams, x_stride, _ptr(h), ntaps,
                                                _ptr(state), ns, _ptr(y), y_stride), "fir_decim_dev")

    def fir_block_dev(self, x, n, nstreams, x_stride, h, ntaps, state, ns, y, y_stride):
        self._check(lib().sdr_fir_block_f32_dev(self._c, _ptr(x), n, nstreams, x_stride, _ptr(h), ntaps,
                                                _ptr(state), ns, _ptr(y), y_stride), "fir_block_dev")

    def fm_demod_dev(self, I, Q, n, nstreams, stride, prev_i, prev_q, out, out_stride):
        self._check(lib().sdr_fm_demod_f32_dev(self._c, _ptr(I), _ptr(Q), n, nstreams, stride, _ptr(prev_i),
                                               _ptr(prev_q), _ptr(out), out_stride), "fm_demod_dev")

    def frontend_dev(self, D, I, Q, n, nstreams, x_stride, h, ntaps, state_i, state_q, ns, prev_i, prev_q, out,
                     out_stride):
        self._check(lib().sdr_frontend_f32_dev(self._c, D, _ptr(I), _ptr(Q), n, nstreams, x_stride, _ptr(h), ntaps,
                                               _ptr(state_i), _ptr(state_q), ns, _ptr(prev_i), _ptr(prev_q),
                                               _ptr(out), out_stride), "frontend_dev")

    def frontend_u8_dev(self, D, iq, npairs, nstreams, iq_stride, h, ntaps, state_i, state_q, ns, prev_i, prev_q,
                        out, out_stride):
        self._check(lib().sdr_frontend_u8_dev(self._c, D, _ptr(iq), npairs, nstreams, iq_stride, _ptr(h), ntaps,
                                              _ptr(state_i), _ptr(state_q), ns, _ptr(prev_i), _ptr(prev_q),
                                              _ptr(out), out_stride), "frontend_u8_dev")

    def resample_dev(self, up, down, x, n, nstreams, x_stride, h, ntaps, state, ns, y, y_stride):
        self._check(lib().sdr_resample_f32_dev(self._c, up, down, _ptr(x), n, nstreams, x_stride, _ptr(h), ntaps,
                                               _ptr(state), ns, _ptr(y), y_stride), "resample_dev")

    def resample_plan(self, up, down, h, ntaps) -> "ResamplePlan":
        """sdr_resample_plan_create: the lane-phase kernel's tables built once from device taps h."""
        p = _vp()
        self._check(lib().sdr_resample_plan_create(self._c, up, down, _ptr(h), ntaps, C.byref(p)), "resample_plan")
        return ResamplePlan(self, p)

    def fir_block_f16_dev(self, x, n, nstreams, x_stride, h, ntaps, state, ns, y, y_stride):
        """fp16-storage arm of blockConvolveFIR (tolerance, not bit-exact)."""
        self._check(lib().sdr_fir_block_f16_dev(self._c, _ptr(x), n, nstreams, x_stride, _ptr(h), ntaps,
                                                _ptr(state), ns, _ptr(y), y_stride), "fir_block_f16_dev")

    def fir_f16_plan(self, h, ntaps) -> "F16Plan":
        """sdr_fir_f16_plan_create: the fp16 MFMA kernel's tap copies built once from device taps h."""
        p = _vp()
        self._check(lib().sdr_fir_f16_plan_create(self._c, _ptr(h), ntaps, C.byref(p)), "fir_f16_plan")
        return F16Plan(self, p)

    def f32_to_f16_dev(self, x, count, y):
        self._check(lib().sdr_f32_to_f16_dev(self._c, _ptr(x), count, _ptr(y)), "f32_to_f16_dev")

    def delay_dev(self, x, n, nstreams, x_stride, state, ns, y, y_stride):
        self._check(lib().sdr_delay_f32_dev(self._c, _ptr(x), n, nstreams, x_stride, _ptr(state), ns, _ptr(y),
                                            y_stride), "delay_dev")

    def pcm_s16_dev(self, x, n, nstreams, x_stride, pcm, pcm_stride):
        self._check(lib().sdr_pcm_s16_dev(self._c, _ptr(x), n, nstreams, x_stride, _ptr(pcm), pcm_stride),
                    "pcm_s16_dev")

    def mono_pcm_u8_dev(self, D, iq, npairs, nstreams, iq_stride, h_rf, rf_taps, st_i, st_q, ns_rf, prev_i, prev_q,
                        delay_state, ns_delay, up, down, h_audio, audio_taps, st_audio, ns_audio, pcm, pcm_stride):
        """src/project.cpp's mono path for one block of every stream: u8 IQ -> s16 PCM, on the device."""
        self._check(lib().sdr_mono_pcm_u8_dev(self._c, D, _ptr(iq), npairs, nstreams, iq_stride, _ptr(h_rf), rf_taps,
                                              _ptr(st_i), _ptr(st_q), ns_rf, _ptr(prev_i), _ptr(prev_q),
                                              _ptr(delay_state), ns_delay, up, down, _ptr(h_audio), audio_taps,
                                              _ptr(st_audio), ns_audio, _ptr(pcm), pcm_stride), "mono_pcm_u8_dev")

    def fm_pll_dev(self, x, n, nstreams, x_stride, freq, Fs, nco_scale, phase_adjust, norm_bw, pll, mix, mix_stride,
                   out, out_stride):
        """fmPLL, one lane per stream; mix given: fused with the x2 stereo mixer."""
        self._check(lib().sdr_fm_pll_dev(self._c, _ptr(x), n, nstreams, x_stride, freq, Fs, nco_scale, phase_adjust,
                                         norm_bw, _ptr(pll), _ptr(mix), mix_stride, _ptr(out), out_stride),
                    "fm_pll_dev")

    def stereo_pcm_dev(self, mono, stereo, n, nstreams, stride, pcm, pcm_stride):
        self._check(lib().sdr_stereo_pcm_dev(self._c, _ptr(mono), _ptr(stereo), n, nstreams, stride, _ptr(pcm),
                                             pcm_stride), "stereo_pcm_dev")

    def stereo_pcm_u8_dev(self, D, iq, npairs, nstreams, iq_stride, up, down, audio_fs, taps, state, pcm,
                          pcm_stride):
        """src/project.cpp's stereo path for one block of every stream: u8 IQ -> interleaved s16 L/R."""
        self._check(lib().sdr_stereo_pcm_u8_dev(self._c, D, _ptr(iq), npairs, nstreams, iq_stride, up, down,
                                                audio_fs, C.addressof(taps), C.addressof(state), _ptr(pcm),
                                                pcm_stride), "stereo_pcm_u8_dev")

    def stereo_work(self, D, npairs, up, down, nstreams) -> "StereoWork":
        """sdr_stereo_work: one block's intermediates for the two-stage stereo calls."""
        w = _vp()
        self._check(lib().sdr_stereo_work_create(self._c, D, npairs, up, down, nstreams, C.byref(w)),
                    "stereo_work_create")
        return StereoWork(self, w)

    def stereo_front_u8_dev(self, iq, iq_stride, taps, state, work):
        """Front stage of the stereo path (src/project.cpp:72-121) into `work`."""
        self._check(lib().sdr_stereo_front_u8_dev(self._c, _ptr(iq), iq_stride, C.addressof(taps),
                                                  C.addressof(state), work._w), "stereo_front_u8_dev")

    def stereo_back_dev(self, audio_fs, taps, state, work, pcm, pcm_stride):
        """Back stage (PLL recurrence onwards, :123-132 + 304-314) from `work` to s16 L/R."""
        self._check(lib().sdr_stereo_back_dev(self._c, audio_fs, C.addressof(taps), C.addressof(state), work._w,
                                              _ptr(pcm), pcm_stride), "stereo_back_dev")

    def stereo_pll_dev(self, audio_fs, state, work):
        """The back stage's recurrence half (:123-126): the block's oscillator arguments into `work`."""
        self._check(lib().sdr_stereo_pll_dev(self._c, audio_fs, C.addressof(state), work._w), "stereo_pll_dev")

    def stereo_post_dev(self, taps, state, work, pcm, pcm_stride):
        """The back stage's post half (:127-132 + 304-314): NCO x stereo band, resampler, s16 L/R."""
        self._check(lib().sdr_stereo_post_dev(self._c, C.addressof(taps), C.addressof(state), work._w, _ptr(pcm),
                                              pcm_stride), "stereo_post_dev")

    def mono_work(self, D, npairs, up, down, nstreams, ns_delay, h_rf, rf_taps, ns_rf, h_audio, audio_taps,
                  ns_audio) -> "MonoWork":
        """sdr_mono_work: one block's row for the two-stage mono calls (shape, taps and state lengths fixed)."""
        w = _vp()
        self._check(lib().sdr_mono_work_create(self._c, D, npairs, up, down, nstreams, ns_delay, _ptr(h_rf), rf_taps,
                                               ns_rf, _ptr(h_audio), audio_taps, ns_audio, C.byref(w)),
                    "mono_work_create")
        return MonoWork(self, w)

    def mono_front_u8_dev(self, iq, iq_stride, h_rf, rf_taps, state_i, state_q, ns_rf, prev_i, prev_q, work):
        """Front stage of the mono path (src/project.cpp:72-93) into `work`."""
        self._check(lib().sdr_mono_front_u8_dev(self._c, _ptr(iq), iq_stride, _ptr(h_rf), rf_taps, _ptr(state_i),
                                                _ptr(state_q), ns_rf, _ptr(prev_i), _ptr(prev_q), work._w),
                    "mono_front_u8_dev")

    def mono_back_dev(self, h_audio, audio_taps, state_audio, ns_audio, delay_state, work, pcm, pcm_stride):
        """Back stage (delay, audio filter, s16: :114-118 + 304-314) from `work`."""
        self._check(lib().sdr_mono_back_dev(self._c, _ptr(h_audio), audio_taps, _ptr(state_audio), ns_audio,
                                            _ptr(delay_state), work._w, _ptr(pcm), pcm_stride), "mono_back_dev")

    def synth_fm_u8_dev(self, iq, npairs, nstreams, iq_stride, seed=1234):
        self._check(lib().sdr_synth_fm_u8_dev(self._c, _ptr(iq), npairs, nstreams, iq_stride, seed), "synth")

    # -- the device transcendental routines of the PLL / NCO (libm_exact.hpp), in bulk
    def libm_sincos_hash_dev(self, mode, chunk_lo, chunk_hi, hash_):
        self._check(lib().sdr_libm_sincos_hash_dev(self._c, mode, chunk_lo, chunk_hi, _ptr(hash_)),
                    "sdr_libm_sincos_hash_dev")

    def libm_sincos_diff_dev(self, chunk_lo, chunk_hi, count, args, cap):
        self._check(lib().sdr_libm_sincos_diff_dev(self._c, chunk_lo, chunk_hi, _ptr(count), _ptr(args), cap),
                    "sdr_libm_sincos_diff_dev")

    def libm_eval_dev(self, fn, a, b, n, out):
        self._check(lib().sdr_libm_eval_dev(self._c, fn, _ptr(a), _ptr(b) if b is not None else None, n, _ptr(out)),
                    "sdr_libm_eval_dev")

    def libm_atan2_screen_dev(self, seed, first, count, cand, cand_cap, out, out_cap, counters):
        self._check(lib().sdr_libm_atan2_screen_dev(self._c, seed, first, count, _ptr(cand), cand_cap, _ptr(out),
                                                    out_cap, _ptr(counters)), "sdr_libm_atan2_screen_dev")

    def u8_to_planar_dev(self, iq, npairs, nstreams, iq_stride, I, Q, x_stride):
        self._check(lib().sdr_u8_to_planar_dev(self._c, _ptr(iq), npairs, nstreams, iq_stride, _ptr(I), _ptr(Q),
                                               x_stride), "u8_to_planar_dev")


def header_symbols(path: str = HEADER_PATH) -> list[str]:
    """Function names declared in include/sdr_hip.h."""
    import re

    text = open(path).read()
    return sorted(set(re.findall(r"\b(sdr_[a-z0-9_]+)\s*\(", text)))


class DeviceArray:
    """A device buffer owned through the C ABI (no torch needed)."""

    def __init__(self, ctx: Context, nbytes: int):
        self.ctx = ctx
        self.nbytes = int(nbytes)
        p = _vp()
        ctx._check(lib().sdr_dev_alloc(ctx._c, max(self.nbytes, 16), C.byref(p)), "dev_alloc")
        self.ptr = int(p.value)

    @classmethod
    def from_numpy(cls, ctx: Context, a: np.ndarray) -> "DeviceArray":
        a = np.ascontiguousarray(a)
        d = cls(ctx, a.nbytes)
        d.upload(a)
        return d

    def upload(self, a: np.ndarray, offset: int = 0):
        a = np.ascontiguousarray(a)
        assert offset + a.nbytes <= self.nbytes
        self.ctx._check(lib().sdr_copy_h2d(self.ctx._c, self.ptr + offset, a.ctypes.data, a.nbytes), "copy_h2d")

    def download(self, dtype=np.float32, count: int | None = None, offset: int = 0) -> np.ndarray:
        dt = np.dtype(dtype)
        if count is None:
            count = (self.nbytes - offset) // dt.itemsize
        out = np.empty(count, dt)
        self.ctx._check(lib().sdr_copy_d2h(self.ctx._c, out.ctypes.data, self.ptr + offset, out.nbytes), "copy_d2h")
        return out

    def fill(self, byte: int = 0):
        self.ctx._check(lib().sdr_dev_memset(self.ctx._c, self.ptr, byte, self.nbytes), "memset")

    def data_ptr(self) -> int:
        return self.ptr

    def free(self):
        if self.ptr:
            lib().sdr_dev_free(self.ctx._c, self.ptr)
            self.ptr = 0

    def __del__(self):
        try:
            self.free()
        except Exception:
            pass
