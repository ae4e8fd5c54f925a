// capi.hip -- the C ABI of libsdrhip.so (include/sdr_hip.h): contexts,
// argument validation (every precondition the reference leaves as UB is an
// SDR_EINVAL here), the host-pointer synchronous wrappers used by the
// drop-in filter.h implementation, and the device-resident batched calls.
#include <hip/hip_runtime.h>

#include <atomic>
#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstring>
#include <mutex>
#include <string>
#include <utility>
#include <vector>

#include "sdr_common.hpp"
#include "sdr_hip.h"

struct sdr_ctx {
  int device = 0;
  hipStream_t own = nullptr;
  hipStream_t cur = nullptr;
  // the stereo pipeline's fork/join: a second stream for the branches that
  // do not wait for the PLL recurrence, and the two events that join them
  // (created on first use)
  hipStream_t side = nullptr;
  hipEvent_t fork = nullptr, join = nullptr;
  int arith = SDR_ARITH_EXACT;
  // sdr_stereo_pcm_u8_dev's launch order: -1 auto, 0 serial, 1 forked
  // (sdr_ctx_set_stereo_fork; SDR_STEREO_FORK sets the default at creation)
  int stereo_fork = -1;
  // grow-only device scratch for the host-pointer wrappers and internal use
  void* buf[20] = {};
  size_t cap[20] = {};
  // live graphs recorded on this context: they hold pointers into buf[], so
  // scratch() refuses to reallocate while any exists (or while capturing)
  int graphs = 0;
  // sdr_ctx_pin_scratch: a caller's own capture (e.g. torch.cuda.graph on the
  // stream given to sdr_ctx_set_stream) holds the buffers too
  bool pinned = false;
  bool grow_refused = false;
  std::string err;
};

namespace {

enum Slot {
  kX0 = 0, kX1, kH, kS0, kS1, kY0, kY1, kOut, kPrev, kTmp,
  kPipe0, kPipe1, kPipe2, kPipe3, kPipe4, kPipe5, kPipe6, kPipe7, kPipe8, kGuard
};

int fail(sdr_ctx* c, int code, const char* fmt, ...) {
  if (c) {
    char msg[512];
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(msg, sizeof msg, fmt, ap);
    va_end(ap);
    c->err = msg;
  }
  return code;
}

int hip_fail(sdr_ctx* c, hipError_t e, const char* where) {
  return fail(c, SDR_EHIP, "%s: %s", where, hipGetErrorString(e));
}

#define SDR_HIP(ctx, call)                                  \
  do {                                                      \
    hipError_t e_ = (call);                                 \
    if (e_ != hipSuccess) return hip_fail((ctx), e_, #call); \
  } while (0)

int enter(sdr_ctx* c) {
  if (!c) return SDR_EINVAL;
  hipError_t e = hipSetDevice(c->device);
  if (e != hipSuccess) return hip_fail(c, e, "hipSetDevice");
  return SDR_OK;
}

bool capturing(hipStream_t s) {
  hipStreamCaptureStatus st = hipStreamCaptureStatusNone;
  return s && hipStreamIsCapturing(s, &st) == hipSuccess && st != hipStreamCaptureStatusNone;
}

// Grow-only scratch.  A HIP graph recorded on the context keeps the buffer
// pointers it was captured with, so growing (free + malloc) is refused --
// nullptr, grow_refused set, see scratch_fail -- while any graph of the
// context is alive or a capture is in progress: size the scratch with one
// direct call of the largest shape first (bench.py and sdr_project do).
void* scratch(sdr_ctx* c, int slot, size_t bytes) {
  if (bytes == 0) bytes = 16;
  if (c->cap[slot] >= bytes) return c->buf[slot];
  if (c->graphs > 0 || c->pinned || capturing(c->cur) || capturing(c->side)) {
    c->grow_refused = true;
    return nullptr;
  }
  if (c->buf[slot]) {
    // the old buffer may still be in use on either stream
    (void)hipStreamSynchronize(c->cur);
    if (c->side) (void)hipStreamSynchronize(c->side);
    (void)hipFree(c->buf[slot]);
    c->buf[slot] = nullptr;
    c->cap[slot] = 0;
  }
  size_t want = bytes + bytes / 4;
  if (hipMalloc(&c->buf[slot], want) != hipSuccess) {
    c->buf[slot] = nullptr;
    return nullptr;
  }
  c->cap[slot] = want;
  return c->buf[slot];
}

// The error for a scratch() that returned nullptr: a refused growth (a live
// graph or a capture holds the old buffers) or an allocation failure.
int scratch_fail(sdr_ctx* c, const char* what) {
  if (c->grow_refused) {
    c->grow_refused = false;
    return fail(c, SDR_EINVAL,
                "%s: scratch would have to grow while a graph recorded on this context is alive or being captured, "
                "or while it is pinned (run one direct call of the largest shape before capturing, or destroy the "
                "graphs / unpin first)",
                what);
  }
  return fail(c, SDR_ENOMEM, "%s", what);
}

// Shared validation of the stateful FIR family (src/filter.cpp:66-83, 123-140).
int check_fir(sdr_ctx* c, int D, long long n, int nstreams, int ntaps, int ns, const void* x, const void* h,
              const void* state) {
  if (!x || !h || !state) return fail(c, SDR_EINVAL, "null pointer");
  if (D < 1) return fail(c, SDR_EINVAL, "decimation factor %d < 1", D);
  if (ntaps < 1) return fail(c, SDR_EINVAL, "ntaps %d < 1", ntaps);
  if (nstreams < 1) return fail(c, SDR_EINVAL, "nstreams %d < 1", nstreams);
  if (n <= 0) return fail(c, SDR_EINVAL, "empty block");
  if (n % D != 0)
    return fail(c, SDR_EINVAL, "block length %lld is not a multiple of %d (reference writes past y, filter.cpp:127-132)",
                n, D);
  if (ns < ntaps - 1)
    return fail(c, SDR_EINVAL, "state length %d < ntaps-1 = %d (reference reads before state, filter.cpp:134)", ns,
                ntaps - 1);
  if (n < ns) return fail(c, SDR_EINVAL, "block length %lld < state length %d (filter.cpp:139 state.assign)", n, ns);
  return SDR_OK;
}

sdr::FirLaunch fir_args(long long n, int nstreams, int ntaps, int D, int ns) {
  sdr::FirLaunch a;
  std::memset(&a, 0, sizeof a);
  a.n = n;
  a.nstreams = nstreams;
  a.ntaps = ntaps;
  a.D = D;
  a.ns = ns;
  return a;
}

// Vector paths need 16-B aligned bases and strides that keep every stream
// row aligned; otherwise the generic (scalar) kernel runs -- same results.
bool vec_ok(const void* p, long long stride_elems, int elem_bytes, int nstreams, int align = 16) {
  return ((uintptr_t)p % align) == 0 && (nstreams == 1 || ((stride_elems * elem_bytes) % align) == 0);
}

}  // namespace

// ------------------------------------------------------- launch helpers --
namespace sdr {
int device_cu_count() {
  // one slot per device, written once with the same value by whichever
  // thread gets there first (relaxed atomics: no torn or racy reads)
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || n <= 0) n = 256;
  cache[dev].store(n, std::memory_order_relaxed);
  return n;
}

int device_lds_bytes() {
  // LDS per CU (160 KiB on gfx950), cached per device like the CU count
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMaxSharedMemoryPerMultiprocessor, dev) != hipSuccess || n <= 0)
    n = 65536;  // the smallest LDS a CDNA CU has: never over-subscribe
  cache[dev].store(n, std::memory_order_relaxed);
  return n;
}

int device_grid_y_max() {
  static std::atomic<int> cache[64];
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) dev = 0;
  int n = cache[dev].load(std::memory_order_relaxed);
  if (n > 0) return n;
  if (hipDeviceGetAttribute(&n, hipDeviceAttributeMaxGridDimY, dev) != hipSuccess || n <= 0) n = 65535;
  cache[dev].store(n, std::memory_order_relaxed);
  return n;
}

int env_int(const char* name, int dflt) {
  const char* e = std::getenv(name);
  return e ? std::atoi(e) : dflt;
}

namespace {
struct SwitchDef {
  const char* name;
  int dflt;
};
// the measured defaults (DESIGN.md 5.2 lists the A/Bs behind each)
constexpr SwitchDef kSwitchDefs[kSwCount] = {
    {"SDR_FIR_SC", 1},          {"SDR_FIR_SC_U8", 1},    {"SDR_RESAMPLE_LP", 1}, {"SDR_RESAMPLE_LOADER", 1},
    {"SDR_RESAMPLE_RS", 1},     {"SDR_RESAMPLE_PP", 1},  {"SDR_LONG_VTAP", 1},   {"SDR_F16_MFMA", 1},
    {"SDR_F16_HEAD", 1},        {"SDR_F16_W8", 1},       {"SDR_PLL_FAST", 1},    {"SDR_PLL_GUARD", 1},
    {"SDR_LONG_COMMIT", 1}};
std::atomic<int> g_switch[kSwCount];
std::once_flag g_switch_once;

void switches_init() {
  std::call_once(g_switch_once, [] {
    for (int i = 0; i < kSwCount; ++i) g_switch[i].store(env_int(kSwitchDefs[i].name, kSwitchDefs[i].dflt));
  });
}

int switch_index(const char* name) {
  if (!name) return -1;
  for (int i = 0; i < kSwCount; ++i)
    if (std::strcmp(name, kSwitchDefs[i].name) == 0) return i;
  return -1;
}
}  // namespace

int sw(Switch s) {
  switches_init();
  return g_switch[s].load(std::memory_order_relaxed);
}
}  // namespace sdr

extern "C" {

const char* sdr_version(void) { return "sdrhip 0.3 (gfx950, ABI 3)"; }

int sdr_abi_version(void) { return SDR_ABI_VERSION; }

const char* sdr_strerror(int code) {
  switch (code) {
    case SDR_OK: return "ok";
    case SDR_EINVAL: return "invalid argument / reference precondition violated";
    case SDR_EHIP: return "HIP runtime error";
    case SDR_ENOMEM: return "device allocation failed";
    case SDR_ENODEV: return "no such device";
    default: return "unknown error";
  }
}

int sdr_set_switch(const char* name, int value) {
  const int i = sdr::switch_index(name);
  if (i < 0) return SDR_EINVAL;
  sdr::switches_init();
  sdr::g_switch[i].store(value, std::memory_order_relaxed);
  return SDR_OK;
}

int sdr_get_switch(const char* name, int* value) {
  const int i = sdr::switch_index(name);
  if (i < 0 || !value) return SDR_EINVAL;
  *value = sdr::sw(static_cast<sdr::Switch>(i));
  return SDR_OK;
}

int sdr_device_count(int* count) {
  if (!count) return SDR_EINVAL;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess) n = 0;
  *count = n;
  return SDR_OK;
}

int sdr_ctx_create(int device, sdr_ctx** out) {
  if (!out) return SDR_EINVAL;
  *out = nullptr;
  int n = 0;
  if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return SDR_ENODEV;
  if (hipSetDevice(device) != hipSuccess) return SDR_ENODEV;
  sdr_ctx* c = new sdr_ctx();
  c->device = device;
  if (hipStreamCreateWithFlags(&c->own, hipStreamNonBlocking) != hipSuccess) {
    delete c;
    return SDR_EHIP;
  }
  c->cur = c->own;
  c->stereo_fork = sdr::env_int("SDR_STEREO_FORK", -1);
  if (c->stereo_fork > 1 || c->stereo_fork < -1) c->stereo_fork = -1;
  *out = c;
  return SDR_OK;
}

int sdr_ctx_destroy(sdr_ctx* c) {
  if (!c) return SDR_EINVAL;
  (void)hipSetDevice(c->device);
  (void)hipStreamSynchronize(c->cur);
  if (c->side) (void)hipStreamSynchronize(c->side);
  for (void* b : c->buf)
    if (b) (void)hipFree(b);
  if (c->own) (void)hipStreamDestroy(c->own);
  if (c->side) (void)hipStreamDestroy(c->side);
  if (c->fork) (void)hipEventDestroy(c->fork);
  if (c->join) (void)hipEventDestroy(c->join);
  delete c;
  return SDR_OK;
}

int sdr_ctx_set_stream(sdr_ctx* c, void* s) {
  if (!c) return SDR_EINVAL;
  c->cur = s ? static_cast<hipStream_t>(s) : c->own;
  return SDR_OK;
}

void* sdr_ctx_get_stream(sdr_ctx* c) { return c ? static_cast<void*>(c->cur) : nullptr; }

int sdr_ctx_set_arith(sdr_ctx* c, int mode) {
  if (!c) return SDR_EINVAL;
  if (mode != SDR_ARITH_EXACT && mode != SDR_ARITH_FMA) return fail(c, SDR_EINVAL, "unknown arithmetic mode %d", mode);
  c->arith = mode;
  return SDR_OK;
}

int sdr_ctx_pin_scratch(sdr_ctx* c, int pinned) {
  if (!c) return SDR_EINVAL;
  c->pinned = pinned != 0;
  return SDR_OK;
}

int sdr_ctx_set_stereo_fork(sdr_ctx* c, int mode) {
  if (!c) return SDR_EINVAL;
  if (mode < -1 || mode > 1) return fail(c, SDR_EINVAL, "unknown stereo fork mode %d", mode);
  c->stereo_fork = mode;
  return SDR_OK;
}

int sdr_ctx_synchronize(sdr_ctx* c) {
  int rc = enter(c);
  if (rc) return rc;
  SDR_HIP(c, hipStreamSynchronize(c->cur));
  return SDR_OK;
}

const char* sdr_ctx_last_error(sdr_ctx* c) { return c ? c->err.c_str() : "null context"; }

int sdr_dev_alloc(sdr_ctx* c, size_t bytes, void** p) {
  int rc = enter(c);
  if (rc) return rc;
  if (!p) return fail(c, SDR_EINVAL, "null out pointer");
  if (hipMalloc(p, bytes ? bytes : 16) != hipSuccess) return fail(c, SDR_ENOMEM, "hipMalloc(%zu)", bytes);
  return SDR_OK;
}

int sdr_dev_free(sdr_ctx* c, void* p) {
  int rc = enter(c);
  if (rc) return rc;
  SDR_HIP(c, hipFree(p));
  return SDR_OK;
}

int sdr_copy_h2d(sdr_ctx* c, void* dst, const void* src, size_t bytes) {
  int rc = enter(c);
  if (rc) return rc;
  SDR_HIP(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->cur));
  SDR_HIP(c, hipStreamSynchronize(c->cur));
  return SDR_OK;
}

int sdr_copy_d2h(sdr_ctx* c, void* dst, const void* src, size_t bytes) {
  int rc = enter(c);
  if (rc) return rc;
  SDR_HIP(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->cur));
  SDR_HIP(c, hipStreamSynchronize(c->cur));
  return SDR_OK;
}

int sdr_dev_memset(sdr_ctx* c, void* dst, int value, size_t bytes) {
  int rc = enter(c);
  if (rc) return rc;
  SDR_HIP(c, hipMemsetAsync(dst, value, bytes, c->cur));
  return SDR_OK;
}

// Pinned host memory, stream-ordered copies and events: what a streaming
// host program needs to overlap its I/O with the device work (the block
// pipeline of host/sdr_project.cpp).
int sdr_host_alloc(sdr_ctx* c, size_t bytes, void** ptr) {
  int rc = enter(c);
  if (rc) return rc;
  if (!ptr) return fail(c, SDR_EINVAL, "null ptr");
  *ptr = nullptr;
  hipError_t e = hipHostMalloc(ptr, bytes ? bytes : 1, hipHostMallocDefault);
  if (e != hipSuccess) return e == hipErrorOutOfMemory ? fail(c, SDR_ENOMEM, "hipHostMalloc %zu", bytes)
                                                       : hip_fail(c, e, "hipHostMalloc");
  return SDR_OK;
}

int sdr_host_free(sdr_ctx* c, void* ptr) {
  int rc = enter(c);
  if (rc) return rc;
  if (ptr) SDR_HIP(c, hipHostFree(ptr));
  return SDR_OK;
}

int sdr_copy_h2d_async(sdr_ctx* c, void* dst, const void* src, size_t bytes) {
  int rc = enter(c);
  if (rc) return rc;
  SDR_HIP(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyHostToDevice, c->cur));
  return SDR_OK;
}

int sdr_copy_d2h_async(sdr_ctx* c, void* dst, const void* src, size_t bytes) {
  int rc = enter(c);
  if (rc) return rc;
  SDR_HIP(c, hipMemcpyAsync(dst, src, bytes, hipMemcpyDeviceToHost, c->cur));
  return SDR_OK;
}

struct sdr_event {
  hipEvent_t ev = nullptr;
};

int sdr_event_create(sdr_ctx* c, sdr_event** ev) {
  int rc = enter(c);
  if (rc) return rc;
  if (!ev) return fail(c, SDR_EINVAL, "null event");
  auto* e = new sdr_event;
  hipError_t h = hipEventCreateWithFlags(&e->ev, hipEventDisableTiming);
  if (h != hipSuccess) {
    delete e;
    return hip_fail(c, h, "hipEventCreate");
  }
  *ev = e;
  return SDR_OK;
}

int sdr_event_record(sdr_ctx* c, sdr_event* ev) {
  int rc = enter(c);
  if (rc) return rc;
  if (!ev) return fail(c, SDR_EINVAL, "null event");
  SDR_HIP(c, hipEventRecord(ev->ev, c->cur));
  return SDR_OK;
}

int sdr_event_synchronize(sdr_ctx* c, sdr_event* ev) {
  int rc = enter(c);
  if (rc) return rc;
  if (!ev) return fail(c, SDR_EINVAL, "null event");
  SDR_HIP(c, hipEventSynchronize(ev->ev));
  return SDR_OK;
}

int sdr_ctx_wait_event(sdr_ctx* c, sdr_event* ev) {
  int rc = enter(c);
  if (rc) return rc;
  if (!ev) return fail(c, SDR_EINVAL, "null event");
  SDR_HIP(c, hipStreamWaitEvent(c->cur, ev->ev, 0));
  return SDR_OK;
}

int sdr_event_destroy(sdr_ctx* c, sdr_event* ev) {
  int rc = enter(c);
  if (rc) return rc;
  if (ev) {
    hipError_t h = hipEventDestroy(ev->ev);
    delete ev;
    if (h != hipSuccess) return hip_fail(c, h, "hipEventDestroy");
  }
  return SDR_OK;
}

// Stream capture -> instantiated HIP graph -> stream-ordered replay: a
// caller's per-block launch sequence (the mono/stereo pipelines' ~10
// launches per block, bench.py's steps) becomes one launch.  Thread-local
// capture mode, so other host threads (other devices' contexts) keep
// working while this one records.
struct sdr_graph {
  hipGraph_t g = nullptr;
  hipGraphExec_t exec = nullptr;
  sdr_ctx* owner = nullptr;  // whose scratch the recorded launches point into
};

int sdr_graph_begin(sdr_ctx* c) {
  int rc = enter(c);
  if (rc) return rc;
  if (!c->cur) return fail(c, SDR_EINVAL, "graph capture needs a non-null stream");
  SDR_HIP(c, hipStreamBeginCapture(c->cur, hipStreamCaptureModeThreadLocal));
  return SDR_OK;
}

int sdr_graph_end(sdr_ctx* c, sdr_graph** out) {
  int rc = enter(c);
  if (rc) return rc;
  if (!out) return fail(c, SDR_EINVAL, "null graph");
  *out = nullptr;
  auto* g = new sdr_graph;
  hipError_t h = hipStreamEndCapture(c->cur, &g->g);
  if (h == hipSuccess) h = hipGraphInstantiate(&g->exec, g->g, nullptr, nullptr, 0);
  if (h != hipSuccess) {
    if (g->g) (void)hipGraphDestroy(g->g);
    delete g;
    return hip_fail(c, h, "stream capture");
  }
  g->owner = c;
  ++c->graphs;
  *out = g;
  return SDR_OK;
}

int sdr_graph_launch(sdr_ctx* c, sdr_graph* g) {
  int rc = enter(c);
  if (rc) return rc;
  if (!g) return fail(c, SDR_EINVAL, "null graph");
  SDR_HIP(c, hipGraphLaunch(g->exec, c->cur));
  return SDR_OK;
}

int sdr_graph_destroy(sdr_ctx* c, sdr_graph* g) {
  int rc = enter(c);
  if (rc) return rc;
  if (g) {
    if (g->exec) (void)hipGraphExecDestroy(g->exec);
    if (g->g) (void)hipGraphDestroy(g->g);
    if (g->owner && g->owner->graphs > 0) --g->owner->graphs;
    delete g;
  }
  return SDR_OK;
}

// ------------------------------------------------------------ taps (host) --
// Windowed-sinc design, src/filter.cpp:14-49: the sinc in double, stored to
// float, then widened again for the sin^2 window and the up-factor gain.
// Host code (setup, once per run) -- bit-identical to the reference.
static constexpr double kPi = 3.14159265358979323846;  // include/dy4.h:14

static float window_gain(float tap, int i, int ntaps, int up) {
  const double s = std::sin((double)i * kPi / (double)ntaps);
  return (float)((double)tap * (s * s) * (double)(float)up);
}

int sdr_taps_lpf(float Fs, float Fc, int ntaps, int up, float* h) {
  if (!h || ntaps < 1 || ntaps > 65535) return SDR_EINVAL;  // filter.h takes unsigned short
  const int T = ntaps;
  const double cutoff = (double)(Fc / (Fs / 2));
  const double centre = ((double)(float)T - 1.0) / 2.0;
  for (int i = 0; i < T; i++) {
    float v;
    if (i == (T - 1) / 2) {
      v = (float)cutoff;
    } else {
      const double arg = kPi * cutoff * ((double)i - centre);
      v = (float)(cutoff * std::sin(arg) / arg);
    }
    h[i] = window_gain(v, i, T, up);
  }
  return SDR_OK;
}

int sdr_taps_bpf(float Fs, float Fb, float Fe, int ntaps, int up, float* h) {
  if (!h || ntaps < 1 || ntaps > 65535) return SDR_EINVAL;
  const int T = ntaps;
  const double centre_f = (double)(((Fe + Fb) / 2) / (Fs / 2));
  const double pass = (double)((Fe - Fb) / (Fs / 2));
  const double centre = ((double)(float)T - 1.0) / 2.0;
  for (int i = 0; i < T; i++) {
    float v;
    if (i == (T - 1) / 2) {
      v = (float)pass;
    } else {
      const double arg = kPi * pass / 2 * ((double)i - centre);
      v = (float)(pass * std::sin(arg) / arg);
    }
    v = (float)((double)v * std::cos((double)(i - (T - 1) / 2) * kPi * centre_f));
    h[i] = window_gain(v, i, T, up);
  }
  return SDR_OK;
}

long long sdr_resample_out_len(int up, int down, long long n) {
  if (up <= 0 || down <= 0 || n < 0) return -1;
  const float q = (float)n / (float)down;  // src/filter.cpp:149
  return (long long)(q * (float)up);
}

// ------------------------------------------------------ device, batched --

// side: the fast kernel's side copy (FirLaunch), pcm: s16 outputs instead of
// y -- both only where the tiled fast path runs (the mono pipeline checks
// fir_fast_f32 first)
static int fir_decim_dev(sdr_ctx* c, int D, const float* x, long long n, int nstreams, long long x_stride,
                         const float* h, int ntaps, float* state, int ns, float* y, long long y_stride,
                         const sdr::FirLaunch* side = nullptr, int16_t* pcm = nullptr, long long pcm_stride = 0) {
  int rc = enter(c);
  if (rc) return rc;
  if ((rc = check_fir(c, D, n, nstreams, ntaps, ns, x, h, state))) return rc;
  if (!y && !pcm) return fail(c, SDR_EINVAL, "null output");
  if (nstreams > 1 && (x_stride < n || (pcm ? pcm_stride : y_stride) < n / D))
    return fail(c, SDR_EINVAL, "stream strides overlap");
  sdr::FirLaunch a = fir_args(n, nstreams, ntaps, D, ns);
  a.x0 = x;
  a.x_stride = x_stride;
  a.state0 = state;
  a.y0 = y;
  a.y_stride = y_stride;
  a.pcm = pcm;
  a.pcm_stride = pcm_stride;
  if (side) {
    a.side_src = side->side_src;
    a.side_dst = side->side_dst;
    a.side_src_stride = side->side_src_stride;
    a.side_dst_stride = side->side_dst_stride;
    a.side_n = side->side_n;
  }
  const bool fast = vec_ok(x, x_stride, 4, nstreams);  // output alignment is handled in-kernel
  if ((pcm || a.side_n > 0) && !(fast && sdr::fir_has_fast_path(D, ntaps, ns, 1, false, sdr::Src::F32)))
    return fail(c, SDR_EINVAL, "internal: fused FIR outputs need the tiled fast path");
  hipError_t e = sdr::launch_fir(a, h, false, 1, sdr::Src::F32, c->cur, nullptr, nullptr, fast);
  if (e != hipSuccess) return hip_fail(c, e, "fir_decim launch");
  return SDR_OK;
}

int sdr_fir_decim_f32_dev(sdr_ctx* c, int D, const float* x, long long n, int nstreams, long long x_stride,
                          const float* h, int ntaps, float* state, int ns, float* y, long long y_stride) {
  return fir_decim_dev(c, D, x, n, nstreams, x_stride, h, ntaps, state, ns, y, y_stride);
}

int sdr_fir_block_f32_dev(sdr_ctx* c, const float* x, long long n, int nstreams, long long x_stride, const float* h,
                          int ntaps, float* state, int ns, float* y, long long y_stride) {
  return sdr_fir_decim_f32_dev(c, 1, x, n, nstreams, x_stride, h, ntaps, state, ns, y, y_stride);
}

int sdr_fm_demod_f32_dev(sdr_ctx* c, const float* I, const float* Q, long long n, int nstreams, long long stride,
                         float* prev_i, float* prev_q, float* out, long long out_stride) {
  int rc = enter(c);
  if (rc) return rc;
  if (!I || !Q || !prev_i || !prev_q || !out) return fail(c, SDR_EINVAL, "null pointer");
  if (n <= 0) return fail(c, SDR_EINVAL, "empty block (reference reads I[-1], filter.cpp:100)");
  if (nstreams < 1) return fail(c, SDR_EINVAL, "nstreams < 1");
  hipError_t e = sdr::launch_demod(I, Q, n, nstreams, stride, prev_i, prev_q, out, out_stride, c->cur);
  if (e != hipSuccess) return hip_fail(c, e, "demod launch");
  return SDR_OK;
}

static int frontend_dev(sdr_ctx* c, sdr::Src src, int D, const float* I, const float* Q, const uint8_t* iq,
                        long long n, int nstreams, long long x_stride, const float* h, int ntaps, float* state_i,
                        float* state_q, int ns, float* prev_i, float* prev_q, float* demod, long long out_stride,
                        const sdr::FirLaunch* side = nullptr) {
  int rc = enter(c);
  if (rc) return rc;
  const void* xin = src == sdr::Src::F32 ? (const void*)I : (const void*)iq;
  if ((rc = check_fir(c, D, n, nstreams, ntaps, ns, xin, h, state_i))) return rc;
  if (src == sdr::Src::F32 && !Q) return fail(c, SDR_EINVAL, "null Q");
  if (!state_q || !prev_i || !prev_q || !demod) return fail(c, SDR_EINVAL, "null pointer");
  const long long nout = n / D;
  const long long per = src == sdr::Src::F32 ? n : 2 * n;
  if (nstreams > 1 && (x_stride < per || out_stride < nout)) return fail(c, SDR_EINVAL, "stream strides overlap");
  sdr::FirLaunch a = fir_args(n, nstreams, ntaps, D, ns);
  a.x0 = I;
  a.x1 = Q;
  a.iq = iq;
  a.x_stride = x_stride;
  a.state0 = state_i;
  a.state1 = state_q;
  a.prev0 = prev_i;
  a.prev1 = prev_q;
  a.out = demod;
  a.out_stride = out_stride;
  a.fma = c->arith == SDR_ARITH_FMA;
  bool fast;
  if (src == sdr::Src::F32)
    fast = vec_ok(I, x_stride, 4, nstreams) && vec_ok(Q, x_stride, 4, nstreams);
  else
    fast = vec_ok(iq, x_stride, 1, nstreams, 8);  // 8-B (4-pair) loads
  if (side) {  // (the mono pipeline's delay line: fast path only, checked by the caller)
    if (!(fast && sdr::fir_has_fast_path(D, ntaps, ns, 2, true, src)))
      return fail(c, SDR_EINVAL, "internal: the front end's side copy needs the tiled fast path");
    a.side_src = side->side_src;
    a.side_dst = side->side_dst;
    a.side_src_stride = side->side_src_stride;
    a.side_dst_stride = side->side_dst_stride;
    a.side_n = side->side_n;
  }
  float* y0 = nullptr;
  float* y1 = nullptr;
  if (!fast || !sdr::fir_has_fast_path(D, ntaps, ns, 2, true, src)) {
    const size_t bytes = (size_t)nout * (size_t)nstreams * sizeof(float);
    y0 = static_cast<float*>(scratch(c, kY0, bytes));
    y1 = static_cast<float*>(scratch(c, kY1, bytes));
    if (!y0 || !y1) return scratch_fail(c, "scratch for decimated I/Q");
  }
  hipError_t e = sdr::launch_fir(a, h, true, 2, src, c->cur, y0, y1, fast);
  if (e != hipSuccess) return hip_fail(c, e, "frontend launch");
  return SDR_OK;
}

int sdr_frontend_f32_dev(sdr_ctx* c, int D, const float* I, const float* Q, long long n, int nstreams,
                         long long x_stride, const float* h, int ntaps, float* state_i, float* state_q, int ns,
                         float* prev_i, float* prev_q, float* demod, long long out_stride) {
  return frontend_dev(c, sdr::Src::F32, D, I, Q, nullptr, n, nstreams, x_stride, h, ntaps, state_i, state_q, ns,
                      prev_i, prev_q, demod, out_stride);
}

int sdr_frontend_u8_dev(sdr_ctx* c, int D, const uint8_t* iq, long long npairs, int nstreams, long long iq_stride,
                        const float* h, int ntaps, float* state_i, float* state_q, int ns, float* prev_i,
                        float* prev_q, float* demod, long long out_stride) {
  return frontend_dev(c, sdr::Src::U8, D, nullptr, nullptr, iq, npairs, nstreams, iq_stride, h, ntaps, state_i,
                      state_q, ns, prev_i, prev_q, demod, out_stride);
}

static int resample_dev(sdr_ctx* c, int up, int down, const float* x, long long n, int nstreams, long long x_stride,
                        const float* h, int ntaps, float* state, int ns, float* y, long long y_stride,
                        const float* lp_tables);

int sdr_resample_f32_dev(sdr_ctx* c, int up, int down, const float* x, long long n, int nstreams, long long x_stride,
                         const float* h, int ntaps, float* state, int ns, float* y, long long y_stride) {
  return resample_dev(c, up, down, x, n, nstreams, x_stride, h, ntaps, state, ns, y, y_stride, nullptr);
}

static int resample_dev(sdr_ctx* c, int up, int down, const float* x, long long n, int nstreams, long long x_stride,
                        const float* h, int ntaps, float* state, int ns, float* y, long long y_stride,
                        const float* lp_tables) {
  int rc = enter(c);
  if (rc) return rc;
  if (!x || !h || !state || !y) return fail(c, SDR_EINVAL, "null pointer");
  if (up < 1 || down < 1) return fail(c, SDR_EINVAL, "up/down factors must be >= 1");
  if (ntaps < 1 || nstreams < 1 || n <= 0) return fail(c, SDR_EINVAL, "empty taps/streams/block");
  const long long ny = sdr_resample_out_len(up, down, n);
  if ((n * up + down - 1) / down > ny)
    return fail(c, SDR_EINVAL,
                "n*up/down does not divide: the reference loop writes %lld outputs into %lld (filter.cpp:149-162)",
                (n * up + down - 1) / down, ny);
  if ((ntaps - 1) / up > ns)
    return fail(c, SDR_EINVAL, "state length %d < (ntaps-1)/up = %d (filter.cpp:164)", ns, (ntaps - 1) / up);
  if (n < ns) return fail(c, SDR_EINVAL, "block length %lld < state length %d (filter.cpp:169)", n, ns);
  if (nstreams > 1 && (x_stride < n || y_stride < ny)) return fail(c, SDR_EINVAL, "stream strides overlap");
  if (up == 1) {
    // identical arithmetic to FIR + decimate by `down` (k = 0..T-1, x[n-k])
    return sdr_fir_decim_f32_dev(c, down, x, n, nstreams, x_stride, h, ntaps, state, ns, y, y_stride);
  }
  float* hp = static_cast<float*>(scratch(c, kTmp, sdr::resample_scratch_floats(up, ntaps) * sizeof(float)));
  if (!hp) return scratch_fail(c, "polyphase table");
  hipError_t e = sdr::launch_resample(up, down, x, n, nstreams, x_stride, h, ntaps, state, ns, y, y_stride, ny, hp,
                                      c->cur, lp_tables);
  if (e != hipSuccess) return hip_fail(c, e, "resample launch");
  return SDR_OK;
}

// The streams that used a device object (a resample plan's tables, a stereo
// work's buffers): one event per stream, recorded after each direct launch
// that reads or writes the object (and after the plan's table build), so
// destroy waits for exactly that work -- on whichever contexts' streams it
// was enqueued -- before freeing.  Launches recorded into a graph are not
// seen: the graph's replays must have completed before destroy (sdr_hip.h).
struct StreamUses {
  std::mutex mu;
  std::vector<std::pair<hipStream_t, hipEvent_t>> v;
  hipError_t mark(hipStream_t s) {
    if (capturing(s)) return hipSuccess;
    std::lock_guard<std::mutex> lk(mu);
    hipEvent_t ev = nullptr;
    for (auto& u : v)
      if (u.first == s) ev = u.second;
    if (!ev) {
      const hipError_t e = hipEventCreateWithFlags(&ev, hipEventDisableTiming);
      if (e != hipSuccess) return e;
      v.emplace_back(s, ev);
    }
    return hipEventRecord(ev, s);
  }
  void wait_and_release() {
    std::lock_guard<std::mutex> lk(mu);
    for (auto& u : v) {
      (void)hipEventSynchronize(u.second);
      (void)hipEventDestroy(u.second);
    }
    v.clear();
  }
};

// A tap plan for the fp16 arm: the MFMA kernel's eight shifted copies of
// the reversed fp16 taps built once (src/project.cpp designs its taps once),
// instead of in every workgroup of every call.
struct sdr_fir_f16_plan {
  int ntaps = 0;
  const float* h = nullptr;
  void* copies = nullptr;  // nullptr: the shape takes no plan (calls build per launch / run v_dot2)
  StreamUses uses;
};

struct sdr_resample_plan {
  int up = 0, down = 0, ntaps = 0;
  const float* h = nullptr;
  float* tables = nullptr;  // resample_lp's tables, or nullptr when the shape takes another kernel
  StreamUses uses;          // the table build and every direct launch with the tables
};

int sdr_resample_plan_create(sdr_ctx* c, int up, int down, const float* h, int ntaps, sdr_resample_plan** out) {
  int rc = enter(c);
  if (rc) return rc;
  if (!out || !h) return fail(c, SDR_EINVAL, "null pointer");
  *out = nullptr;
  if (up < 1 || down < 1 || ntaps < 1) return fail(c, SDR_EINVAL, "up/down/ntaps must be >= 1");
  auto* p = new sdr_resample_plan;
  p->up = up;
  p->down = down;
  p->ntaps = ntaps;
  p->h = h;
  if (up > 1) {
    const size_t bytes = sdr::resample_rs_scratch_floats(up, ntaps) * sizeof(float);
    hipError_t e = hipMalloc(&p->tables, bytes);
    if (e != hipSuccess) {
      delete p;
      return fail(c, SDR_ENOMEM, "resample plan tables");
    }
    if (!sdr::resample_lp_tables(up, down, h, ntaps, 0, p->tables, c->cur, &e)) {
      (void)hipFree(p->tables);
      p->tables = nullptr;  // another kernel: built per call as before
    } else if (e != hipSuccess) {
      (void)hipFree(p->tables);
      delete p;
      return hip_fail(c, e, "resample plan tables");
    } else if ((e = hipStreamSynchronize(c->cur)) != hipSuccess || (e = p->uses.mark(c->cur)) != hipSuccess) {
      // built before the plan is handed out: a later call may run on
      // another stream (sdr_ctx_set_stream), which nothing would order;
      // the build is recorded as a use of the plan too
      (void)hipFree(p->tables);
      delete p;
      return hip_fail(c, e, "resample plan tables");
    }
  }
  *out = p;
  return SDR_OK;
}

int sdr_resample_plan_destroy(sdr_ctx* c, sdr_resample_plan* p) {
  int rc = enter(c);
  if (rc) return rc;
  if (p) {
    // every stream that used the plan, not only the current one (graph
    // replays of calls with the plan must have completed, sdr_hip.h)
    p->uses.wait_and_release();
    if (p->tables) (void)hipFree(p->tables);
    delete p;
  }
  return SDR_OK;
}

int sdr_resample_plan_f32_dev(sdr_ctx* c, const sdr_resample_plan* p, const float* x, long long n, int nstreams,
                              long long x_stride, float* state, int ns, float* y, long long y_stride) {
  if (!p) return fail(c, SDR_EINVAL, "null plan");
  const int rc = resample_dev(c, p->up, p->down, x, n, nstreams, x_stride, p->h, p->ntaps, state, ns, y, y_stride,
                              p->tables);
  if (rc || !p->tables) return rc;
  SDR_HIP(c, const_cast<sdr_resample_plan*>(p)->uses.mark(c->cur));
  return SDR_OK;
}

int sdr_fir_block_f16_kernel(int ntaps) { return sdr::fir_f16_uses_mfma(ntaps) ? 1 : 0; }

static int fir_block_f16(sdr_ctx* c, const void* x, long long n, int nstreams, long long x_stride, const float* h,
                         int ntaps, void* state, int ns, float* y, long long y_stride, const void* plan);

int sdr_fir_block_f16_dev(sdr_ctx* c, const void* x, long long n, int nstreams, long long x_stride, const float* h,
                          int ntaps, void* state, int ns, float* y, long long y_stride) {
  return fir_block_f16(c, x, n, nstreams, x_stride, h, ntaps, state, ns, y, y_stride, nullptr);
}

int sdr_fir_block_f16_plan_dev(sdr_ctx* c, const sdr_fir_f16_plan* p, const void* x, long long n, int nstreams,
                               long long x_stride, void* state, int ns, float* y, long long y_stride) {
  if (!p) return fail(c, SDR_EINVAL, "null plan");
  const int rc = fir_block_f16(c, x, n, nstreams, x_stride, p->h, p->ntaps, state, ns, y, y_stride, p->copies);
  if (rc || !p->copies) return rc;
  SDR_HIP(c, const_cast<sdr_fir_f16_plan*>(p)->uses.mark(c->cur));
  return SDR_OK;
}

static int fir_block_f16(sdr_ctx* c, const void* x, long long n, int nstreams, long long x_stride, const float* h,
                         int ntaps, void* state, int ns, float* y, long long y_stride, const void* plan) {
  int rc = enter(c);
  if (rc) return rc;
  if (!x || !h || !state || !y) return fail(c, SDR_EINVAL, "null pointer");
  if (ntaps < 1 || nstreams < 1 || n <= 0) return fail(c, SDR_EINVAL, "empty taps/streams/block");
  if (ns < ntaps - 1) return fail(c, SDR_EINVAL, "state length %d < ntaps-1 = %d (filter.cpp:74)", ns, ntaps - 1);
  if (n < ns) return fail(c, SDR_EINVAL, "block length %lld < state length %d (filter.cpp:82)", n, ns);
  if (nstreams > 1 && (x_stride < n || y_stride < n)) return fail(c, SDR_EINVAL, "stream strides overlap");
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (nstreams > 1 && x_stride % 8))
    return fail(c, SDR_EINVAL, "fp16 input rows must be 16-B aligned (x_stride %% 8 == 0)");
  uint32_t* pairs = static_cast<uint32_t*>(scratch(c, kTmp, sdr::fir_long_h_pairs(ntaps) * sizeof(uint32_t)));
  if (!pairs) return scratch_fail(c, "tap pair table");
  hipError_t e =
      sdr::launch_fir_long_h(x, n, nstreams, x_stride, h, ntaps, state, ns, y, y_stride, pairs, c->cur, plan);
  if (e != hipSuccess) return hip_fail(c, e, "fir_block_f16 launch");
  return SDR_OK;
}

int sdr_fir_f16_plan_create(sdr_ctx* c, const float* h, int ntaps, sdr_fir_f16_plan** out) {
  int rc = enter(c);
  if (rc) return rc;
  if (!out || !h) return fail(c, SDR_EINVAL, "null pointer");
  *out = nullptr;
  if (ntaps < 1) return fail(c, SDR_EINVAL, "ntaps %d < 1", ntaps);
  auto* p = new sdr_fir_f16_plan;
  p->ntaps = ntaps;
  p->h = h;
  const size_t halves = sdr::fir_f16_plan_halves(ntaps);
  if (halves) {
    hipError_t e = hipMalloc(&p->copies, halves * 2);
    if (e != hipSuccess) {
      delete p;
      return fail(c, SDR_ENOMEM, "fp16 tap plan");
    }
    if ((e = sdr::build_fir_f16_plan(h, ntaps, p->copies, c->cur)) != hipSuccess ||
        (e = hipStreamSynchronize(c->cur)) != hipSuccess || (e = p->uses.mark(c->cur)) != hipSuccess) {
      (void)hipFree(p->copies);
      delete p;
      return hip_fail(c, e, "fp16 tap plan");
    }
  }
  *out = p;
  return SDR_OK;
}

int sdr_fir_f16_plan_destroy(sdr_ctx* c, sdr_fir_f16_plan* p) {
  int rc = enter(c);
  if (rc) return rc;
  if (p) {
    p->uses.wait_and_release();
    if (p->copies) (void)hipFree(p->copies);
    delete p;
  }
  return SDR_OK;
}

int sdr_f32_to_f16_dev(sdr_ctx* c, const float* x, long long count, void* y) {
  int rc = enter(c);
  if (rc) return rc;
  if (!x || !y || count < 0) return fail(c, SDR_EINVAL, "bad conversion arguments");
  if (count == 0) return SDR_OK;
  hipError_t e = sdr::launch_f32_to_f16(x, count, y, c->cur);
  if (e != hipSuccess) return hip_fail(c, e, "f32_to_f16 launch");
  return SDR_OK;
}

int sdr_delay_f32_dev(sdr_ctx* c, const float* in, long long n, int nstreams, long long in_stride, float* state,
                      int ns, float* out, long long out_stride) {
  int rc = enter(c);
  if (rc) return rc;
  if (!in || !state || !out) return fail(c, SDR_EINVAL, "null pointer");
  if (n <= 0 || nstreams < 1 || ns < 0) return fail(c, SDR_EINVAL, "empty block / bad sizes");
  if (n < ns) return fail(c, SDR_EINVAL, "block length %lld < delay %d (filter.cpp delayBlock reads past the block)", n,
                          ns);
  if (ns > 256) return fail(c, SDR_EINVAL, "delay %d > 256 not supported on the device path", ns);
  if (nstreams > 1 && (in_stride < n || out_stride < n)) return fail(c, SDR_EINVAL, "stream strides overlap");
  hipError_t e = sdr::launch_delay(in, n, nstreams, in_stride, state, ns, out, out_stride, c->cur);
  if (e != hipSuccess) return hip_fail(c, e, "delay launch");
  return SDR_OK;
}

int sdr_pcm_s16_dev(sdr_ctx* c, const float* x, long long n, int nstreams, long long x_stride, int16_t* pcm,
                    long long pcm_stride) {
  int rc = enter(c);
  if (rc) return rc;
  if (!x || !pcm || n < 0 || nstreams < 1) return fail(c, SDR_EINVAL, "bad pcm arguments");
  if (n == 0) return SDR_OK;
  hipError_t e = sdr::launch_pcm(x, n, nstreams, x_stride, pcm, pcm_stride, c->cur);
  if (e != hipSuccess) return hip_fail(c, e, "pcm launch");
  return SDR_OK;
}

int sdr_mono_pcm_u8_dev(sdr_ctx* c, int D, const uint8_t* iq, long long npairs, int nstreams, long long iq_stride,
                        const float* h_rf, int rf_taps, float* state_i, float* state_q, int ns_rf, float* prev_i,
                        float* prev_q, float* delay_state, int ns_delay, int up, int down, const float* h_audio,
                        int audio_taps, float* state_audio, int ns_audio, int16_t* pcm, long long pcm_stride) {
  int rc = enter(c);
  if (rc) return rc;
  if (D < 1 || npairs <= 0 || npairs % D) return fail(c, SDR_EINVAL, "block of %lld pairs is not a multiple of %d",
                                                   npairs, D);
  const long long nd = npairs / D;  // demodulated samples per stream
  const long long na = sdr_resample_out_len(up, down, nd);
  if (na <= 0) return fail(c, SDR_EINVAL, "empty audio block");
  if (nstreams > 1 && pcm_stride < na) return fail(c, SDR_EINVAL, "pcm stride < audio samples per block");
  // Fused (the tiled kernels on both filters, up == 1 -- mode 0's audio
  // stage is FIR + decimate): one row buffer [delay state | demod] per
  // stream.  The front end writes its output at row offset ns_delay, and its
  // tile-0 workgroups copy the carried delay state into the row's head (their
  // side copy), so the row's first nd floats ARE delayBlock's output
  // (src/filter.cpp:230-238, src/project.cpp:114).  The audio FIR reads them
  // in place, copies the row's last ns_delay floats (the new delay state) out
  // as its side copy and stores s16 PCM itself (src/project.cpp:311-314): no
  // delay or PCM launch, no delayed copy of the block.
  const bool fuse_ok = up == 1 && iq && h_rf && h_audio && delay_state && state_audio && pcm && ns_delay >= 0 &&
                       ns_delay <= 256 /* the side copy's 4 per lane of a wave */ && nd >= ns_delay && nd % down == 0 &&
                       vec_ok(iq, iq_stride, 1, nstreams, 8) &&
                       sdr::fir_has_fast_path(D, rf_taps, ns_rf, 2, true, sdr::Src::U8) &&
                       sdr::fir_has_fast_path(down, audio_taps, ns_audio, 1, false, sdr::Src::F32);
  if (fuse_ok) {
    const long long rstride = (ns_delay + nd + 3) / 4 * 4;  // 16-B rows: the audio FIR's fast path reads them
    float* row = static_cast<float*>(scratch(c, kPipe0, (size_t)nstreams * rstride * sizeof(float)));
    if (!row) return scratch_fail(c, "pipeline buffer");
    sdr::FirLaunch head;
    std::memset(&head, 0, sizeof head);
    head.side_src = delay_state;
    head.side_src_stride = ns_delay;
    head.side_dst = row;
    head.side_dst_stride = rstride;
    head.side_n = ns_delay;
    if ((rc = frontend_dev(c, sdr::Src::U8, D, nullptr, nullptr, iq, npairs, nstreams, iq_stride, h_rf, rf_taps,
                           state_i, state_q, ns_rf, prev_i, prev_q, row + ns_delay, rstride, &head)))
      return rc;
    sdr::FirLaunch tail;
    std::memset(&tail, 0, sizeof tail);
    tail.side_src = row + nd;
    tail.side_src_stride = rstride;
    tail.side_dst = delay_state;
    tail.side_dst_stride = ns_delay;
    tail.side_n = ns_delay;
    return fir_decim_dev(c, down, row, nd, nstreams, rstride, h_audio, audio_taps, state_audio, ns_audio, nullptr, 0,
                         &tail, pcm, nstreams > 1 ? pcm_stride : na);
  }
  // rows of the intermediate buffers: multiples of 4 floats (16-B aligned rows for the tiled kernels)
  const long long dstride = (nd + 3) / 4 * 4, astride = (na + 3) / 4 * 4;
  float* demod = static_cast<float*>(scratch(c, kPipe0, (size_t)nstreams * dstride * sizeof(float)));
  float* delayed = static_cast<float*>(scratch(c, kPipe1, (size_t)nstreams * dstride * sizeof(float)));
  float* audio = static_cast<float*>(scratch(c, kPipe2, (size_t)nstreams * astride * sizeof(float)));
  if (!demod || !delayed || !audio) return scratch_fail(c, "pipeline buffers");
  if ((rc = sdr_frontend_u8_dev(c, D, iq, npairs, nstreams, iq_stride, h_rf, rf_taps, state_i, state_q, ns_rf, prev_i,
                                prev_q, demod, dstride)))
    return rc;
  if ((rc = sdr_delay_f32_dev(c, demod, nd, nstreams, dstride, delay_state, ns_delay, delayed, dstride))) return rc;
  if ((rc = sdr_resample_f32_dev(c, up, down, delayed, nd, nstreams, dstride, h_audio, audio_taps, state_audio,
                                 ns_audio, audio, astride)))
    return rc;
  return sdr_pcm_s16_dev(c, audio, na, nstreams, astride, pcm, pcm_stride);
}

int sdr_fm_pll_dev(sdr_ctx* c, const float* in, long long n, int nstreams, long long in_stride, float freq, float Fs,
                   float nco_scale, float phase_adjust, float norm_bw, float* pll, const float* mix,
                   long long mix_stride, float* out, long long out_stride) {
  int rc = enter(c);
  if (rc) return rc;
  if (!in || !pll || !out) return fail(c, SDR_EINVAL, "null pointer");
  if (n <= 0 || nstreams < 1) return fail(c, SDR_EINVAL, "empty block (fmPLL writes ncoOut[0], filter.cpp:186)");
  if (nstreams > 1 && (in_stride < n || out_stride < n || (mix && mix_stride < n)))
    return fail(c, SDR_EINVAL, "stream strides overlap");
  const long long astride = (n + 1 + 3) / 4 * 4;  // trigArg per sample (+ the incoming nco_state)
  float* args = static_cast<float*>(scratch(c, kPipe6, (size_t)nstreams * astride * sizeof(float)));
  if (!args) return scratch_fail(c, "pll argument buffer");
  auto* guard = static_cast<uint8_t*>(scratch(c, kGuard, sdr::pll_guard_bytes(n, nstreams)));
  if (!guard) return scratch_fail(c, "pll guard buffer");
  hipError_t e = sdr::launch_pll(in, n, nstreams, in_stride, freq, Fs, nco_scale, phase_adjust, norm_bw, pll, mix,
                                 mix_stride, out, out_stride, args, astride, c->cur, guard);
  if (e != hipSuccess) return hip_fail(c, e, "pll launch");
  return SDR_OK;
}

int sdr_stereo_pcm_dev(sdr_ctx* c, const float* mono, const float* stereo, long long n, int nstreams,
                       long long stride, int16_t* pcm, long long pcm_stride) {
  int rc = enter(c);
  if (rc) return rc;
  if (!mono || !stereo || !pcm || n < 0 || nstreams < 1) return fail(c, SDR_EINVAL, "bad stereo pcm arguments");
  if (nstreams > 1 && (stride < n || pcm_stride < 2 * n)) return fail(c, SDR_EINVAL, "stream strides overlap");
  if (n == 0) return SDR_OK;
  hipError_t e = sdr::launch_stereo_pcm(mono, stereo, n, nstreams, stride, pcm, pcm_stride, c->cur);
  if (e != hipSuccess) return hip_fail(c, e, "stereo pcm launch");
  return SDR_OK;
}

int sdr_stereo_pcm_u8_dev(sdr_ctx* c, int D, const uint8_t* iq, long long npairs, int nstreams, long long iq_stride,
                          int up, int down, float audio_fs, const sdr_stereo_taps* taps, sdr_stereo_state* st,
                          int16_t* pcm, long long pcm_stride) {
  int rc = enter(c);
  if (rc) return rc;
  if (!taps || !st) return fail(c, SDR_EINVAL, "null taps / state");
  if (D < 1 || npairs <= 0 || npairs % D) return fail(c, SDR_EINVAL, "block of %lld pairs is not a multiple of %d",
                                                   npairs, D);
  const long long nd = npairs / D;
  const long long na = sdr_resample_out_len(up, down, nd);
  if (na <= 0) return fail(c, SDR_EINVAL, "empty audio block");
  if (nstreams > 1 && pcm_stride < 2 * na) return fail(c, SDR_EINVAL, "pcm stride < 2 x audio samples per block");
  const long long dstride = (nd + 3) / 4 * 4, astride = (na + 3) / 4 * 4;
  const size_t dbytes = (size_t)nstreams * dstride * sizeof(float), abytes = (size_t)nstreams * astride * sizeof(float);
  const long long pstride = (nd + 1 + 3) / 4 * 4;  // PLL oscillator arguments (+ the incoming nco_state)
  float* demod = static_cast<float*>(scratch(c, kPipe0, dbytes));
  float* delayed = static_cast<float*>(scratch(c, kPipe1, dbytes));
  float* mono = static_cast<float*>(scratch(c, kPipe2, abytes));
  float* pilot = static_cast<float*>(scratch(c, kPipe3, dbytes));
  float* sband = static_cast<float*>(scratch(c, kPipe4, dbytes));
  float* slp = static_cast<float*>(scratch(c, kPipe5, abytes));
  float* args = static_cast<float*>(scratch(c, kPipe6, (size_t)nstreams * pstride * sizeof(float)));
  float* mixed = static_cast<float*>(scratch(c, kPipe7, dbytes));
  auto* guard = static_cast<uint8_t*>(scratch(c, kGuard, sdr::pll_guard_bytes(nd, nstreams)));
  if (!demod || !delayed || !mono || !pilot || !sband || !slp || !args || !mixed || !guard)
    return scratch_fail(c, "pipeline buffers");
  if (!c->side) {
    SDR_HIP(c, hipStreamCreateWithFlags(&c->side, hipStreamNonBlocking));
    SDR_HIP(c, hipEventCreateWithFlags(&c->fork, hipEventDisableTiming));
    SDR_HIP(c, hipEventCreateWithFlags(&c->join, hipEventDisableTiming));
  }
  // The PLL recurrence (one lane per stream, latency-bound) is the critical
  // path: front end -> pilot BPF -> recurrence -> NCO x stereo band ->
  // stereo LPF -> PCM.  The branches that do not wait for it -- delay + mono
  // resampler (src/project.cpp:114-116) and the stereo band-pass (:121) --
  // run on a second stream beside it and join before the mixer.  Captured
  // into a HIP graph, the fork/join becomes two parallel branches.
  // src/project.cpp:72-93: front end
  if ((rc = sdr_frontend_u8_dev(c, D, iq, npairs, nstreams, iq_stride, taps->h_rf, taps->rf_taps, st->state_i,
                                st->state_q, st->ns_rf, st->prev_i, st->prev_q, demod, dstride)))
    return rc;
  // Fork only while the recurrence (one lane per stream, 64 streams per
  // wave) leaves most of the chip idle: at 1,024 streams (16 waves) the side
  // branch runs in the gaps (stereo0 -1.6 %), at 16,384 (256 waves, one per
  // CU) it competes with the latency-bound recurrence for the CUs and slows
  // it (stereo0w +14 %, same box).  sdr_ctx_set_stereo_fork (default from
  // SDR_STEREO_FORK at context creation) forces either way.
  const long long pll_waves = (nstreams + 63) / 64;
  const bool fork = c->stereo_fork >= 0 ? c->stereo_fork != 0 : 4 * pll_waves <= sdr::device_cu_count();
  if (fork) {
    SDR_HIP(c, hipEventRecord(c->fork, c->cur));
    SDR_HIP(c, hipStreamWaitEvent(c->side, c->fork, 0));
  }
  {
    hipStream_t main = c->cur;
    if (fork) c->cur = c->side;
    // :114-116: mono = resample(delay(demod)); :121: stereo band-pass
    rc = sdr_delay_f32_dev(c, demod, nd, nstreams, dstride, st->delay_state, st->ns_delay, delayed, dstride);
    if (!rc)
      rc = sdr_resample_f32_dev(c, up, down, delayed, nd, nstreams, dstride, taps->h_audio, taps->audio_taps,
                                st->state_audio, st->ns_audio, mono, astride);
    if (!rc)
      rc = sdr_fir_block_f32_dev(c, demod, nd, nstreams, dstride, taps->h_stereo, taps->bpf_taps, st->stereo_state,
                                 st->ns_bpf, sband, dstride);
    // the join is recorded even when a side-branch call failed, and then
    // waited on here, so nothing left on the side stream overlaps later
    // main-stream work or a scratch free
    hipError_t e = fork ? hipEventRecord(c->join, c->side) : hipSuccess;
    c->cur = main;
    if (rc) {
      if (fork && e == hipSuccess) (void)hipStreamWaitEvent(main, c->join, 0);
      return rc;
    }
    if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
  }
  // :120: pilot band-pass, then the PLL recurrence (:123-126: 19 kHz, ncoScale 2,
  // phaseAdjust 0, bandwidth 0.01)
  if ((rc = sdr_fir_block_f32_dev(c, demod, nd, nstreams, dstride, taps->h_pilot, taps->bpf_taps, st->pilot_state,
                                  st->ns_bpf, pilot, dstride)))
    return rc;
  hipError_t e = sdr::launch_pll_recurrence(pilot, nd, nstreams, dstride, 19e3f, audio_fs, 2.0f, 0.0f, 0.01f, st->pll,
                                            args, pstride, c->cur, guard);
  if (e != hipSuccess) return hip_fail(c, e, "pll launch");
  // join: the NCO mixed with the stereo band (pointwiseMultiply x2, :127)
  if (fork) SDR_HIP(c, hipStreamWaitEvent(c->cur, c->join, 0));
  e = sdr::launch_nco(args, pstride, nd, nstreams, 2.0f, 0.0f, sband, dstride, mixed, dstride, c->cur);
  if (e != hipSuccess) return hip_fail(c, e, "nco launch");
  // :129: the stereo channel through the same audio resampler, its own state
  if ((rc = sdr_resample_f32_dev(c, up, down, mixed, nd, nstreams, dstride, taps->h_audio, taps->audio_taps,
                                 st->stereo_lp_state, st->ns_audio, slp, astride)))
    return rc;
  // :131-132 + 304-314: L/R, interleave, s16
  return sdr_stereo_pcm_dev(c, mono, slp, na, nstreams, astride, pcm, pcm_stride);
}

// ---------------------------------------------- stereo path in two stages --
// The same calls as sdr_stereo_pcm_u8_dev, cut where the PLL recurrence
// starts, with one block's intermediates in a caller-owned work object so a
// block's front stage can run on one context's stream while the previous
// block's back stage (the recurrence) runs on another's (host/sdr_project.cpp).
// The stages touch disjoint state: front = RF front end, delay, mono
// resampler, pilot and stereo band-pass states; back = PLL and the stereo
// resampler state.
struct sdr_stereo_work {
  int D = 0, up = 0, down = 0, nstreams = 0;
  long long npairs = 0, nd = 0, na = 0, dstride = 0, astride = 0, pstride = 0;
  void* mem = nullptr;
  float *demod = nullptr, *delayed = nullptr, *mono = nullptr, *pilot = nullptr, *sband = nullptr, *slp = nullptr,
        *args = nullptr, *mixed = nullptr;
  uint8_t* guard = nullptr;
  bool guard_ready = false;  // the front stage wrote this block's PLL guard (host order: front, then back)
  StreamUses uses;  // every stream a stage ran on (destroy waits for them)
};

int sdr_stereo_work_create(sdr_ctx* c, int D, long long npairs, int up, int down, int nstreams,
                           sdr_stereo_work** out) {
  int rc = enter(c);
  if (rc) return rc;
  if (!out) return fail(c, SDR_EINVAL, "null work");
  *out = nullptr;
  if (D < 1 || npairs <= 0 || npairs % D || nstreams < 1 || up < 1 || down < 1)
    return fail(c, SDR_EINVAL, "bad stereo work shape");
  auto* w = new sdr_stereo_work;
  w->D = D, w->up = up, w->down = down, w->nstreams = nstreams, w->npairs = npairs;
  w->nd = npairs / D;
  w->na = sdr_resample_out_len(up, down, w->nd);
  if (w->na <= 0) {
    delete w;
    return fail(c, SDR_EINVAL, "empty audio block");
  }
  w->dstride = (w->nd + 3) / 4 * 4, w->astride = (w->na + 3) / 4 * 4, w->pstride = (w->nd + 1 + 3) / 4 * 4;
  const size_t d = (size_t)nstreams * w->dstride, a = (size_t)nstreams * w->astride,
               p = (size_t)nstreams * w->pstride;
  const size_t g = (sdr::pll_guard_bytes(w->nd, nstreams) + 15) / 16 * 16;
  const size_t floats = 5 * d + 2 * a + p;
  hipError_t e = hipMalloc(&w->mem, floats * sizeof(float) + g);
  if (e != hipSuccess) {
    delete w;
    return fail(c, SDR_ENOMEM, "stereo work buffers");
  }
  float* f = static_cast<float*>(w->mem);
  w->demod = f, f += d;
  w->delayed = f, f += d;
  w->pilot = f, f += d;
  w->sband = f, f += d;
  w->mixed = f, f += d;
  w->mono = f, f += a;
  w->slp = f, f += a;
  w->args = f, f += p;
  w->guard = reinterpret_cast<uint8_t*>(f);
  *out = w;
  return SDR_OK;
}

int sdr_stereo_work_destroy(sdr_ctx* c, sdr_stereo_work* w) {
  int rc = enter(c);
  if (rc) return rc;
  if (w) {
    // the stages may have run on other contexts' streams (the two-stage
    // pipeline: front on one, back on another): wait for every one of them
    w->uses.wait_and_release();
    (void)hipFree(w->mem);
    delete w;
  }
  return SDR_OK;
}

// front end (src/project.cpp:72-93), delay + mono resampler (:114-116),
// stereo band-pass (:121), pilot band-pass (:120)
int sdr_stereo_front_u8_dev(sdr_ctx* c, const uint8_t* iq, long long iq_stride, const sdr_stereo_taps* taps,
                            sdr_stereo_state* st, sdr_stereo_work* w) {
  int rc = enter(c);
  if (rc) return rc;
  if (!taps || !st || !w) return fail(c, SDR_EINVAL, "null taps / state / work");
  const int n = w->nstreams;
  rc = sdr_frontend_u8_dev(c, w->D, iq, w->npairs, n, iq_stride, taps->h_rf, taps->rf_taps, st->state_i,
                           st->state_q, st->ns_rf, st->prev_i, st->prev_q, w->demod, w->dstride);
  if (!rc)
    rc = sdr_delay_f32_dev(c, w->demod, w->nd, n, w->dstride, st->delay_state, st->ns_delay, w->delayed, w->dstride);
  if (!rc)
    rc = sdr_resample_f32_dev(c, w->up, w->down, w->delayed, w->nd, n, w->dstride, taps->h_audio, taps->audio_taps,
                              st->state_audio, st->ns_audio, w->mono, w->astride);
  if (!rc)
    rc = sdr_fir_block_f32_dev(c, w->demod, w->nd, n, w->dstride, taps->h_stereo, taps->bpf_taps, st->stereo_state,
                               st->ns_bpf, w->sband, w->dstride);
  if (!rc)
    rc = sdr_fir_block_f32_dev(c, w->demod, w->nd, n, w->dstride, taps->h_pilot, taps->bpf_taps, st->pilot_state,
                               st->ns_bpf, w->pilot, w->dstride);
  // the recurrence's input guard from the pilot, here: off the back stage's
  // critical path (the back stage waits for this stage anyway)
  w->guard_ready = false;
  hipError_t ge = hipSuccess;
  if (!rc) ge = sdr::launch_pll_guard(w->pilot, w->nd, n, w->dstride, w->guard, c->cur, &w->guard_ready);
  // marked even after a failed launch: whatever was enqueued uses the work
  const hipError_t e = w->uses.mark(c->cur);
  if (rc) return rc;
  if (ge != hipSuccess) return hip_fail(c, ge, "pll guard launch");
  if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
  return SDR_OK;
}

// PLL recurrence (:123-126): the block's oscillator arguments into the work.
// (A three-context split -- recurrence | post stage on a third context's
// stream -- measured slower than two stages in round 5; the
// halves are exported again for the two-stream schedule below.)
static int stereo_pll(sdr_ctx* c, float audio_fs, sdr_stereo_state* st, sdr_stereo_work* w) {
  if (!st || !w) return fail(c, SDR_EINVAL, "null state / work");
  hipError_t e = sdr::launch_pll_recurrence(w->pilot, w->nd, w->nstreams, w->dstride, 19e3f, audio_fs, 2.0f, 0.0f,
                                            0.01f, st->pll, w->args, w->pstride, c->cur, w->guard, w->guard_ready);
  w->guard_ready = false;  // one block's guard serves one recurrence
  if (e != hipSuccess) return hip_fail(c, e, "pll launch");
  return SDR_OK;
}

// NCO x stereo band (:127), stereo resampler (:129), L/R + interleave + s16
// (:131-132, 304-314)
static int stereo_post(sdr_ctx* c, const sdr_stereo_taps* taps, sdr_stereo_state* st, sdr_stereo_work* w,
                       int16_t* pcm, long long pcm_stride) {
  int rc = SDR_OK;
  if (!taps || !st || !w || !pcm) return fail(c, SDR_EINVAL, "null taps / state / work / pcm");
  const int n = w->nstreams;
  if (n > 1 && pcm_stride < 2 * w->na) return fail(c, SDR_EINVAL, "pcm stride < 2 x audio samples per block");
  hipError_t e =
      sdr::launch_nco(w->args, w->pstride, w->nd, n, 2.0f, 0.0f, w->sband, w->dstride, w->mixed, w->dstride, c->cur);
  if (e != hipSuccess) return hip_fail(c, e, "nco launch");
  if ((rc = sdr_resample_f32_dev(c, w->up, w->down, w->mixed, w->nd, n, w->dstride, taps->h_audio, taps->audio_taps,
                                 st->stereo_lp_state, st->ns_audio, w->slp, w->astride)))
    return rc;
  return sdr_stereo_pcm_dev(c, w->mono, w->slp, w->na, n, w->astride, pcm, pcm_stride);
}

// the PLL stage and the post stage in one call on this context's stream
int sdr_stereo_back_dev(sdr_ctx* c, float audio_fs, const sdr_stereo_taps* taps, sdr_stereo_state* st,
                        sdr_stereo_work* w, int16_t* pcm, long long pcm_stride) {
  int rc = enter(c);
  if (rc) return rc;
  if (!taps || !st || !w || !pcm) return fail(c, SDR_EINVAL, "null taps / state / work / pcm");
  if (w->nstreams > 1 && pcm_stride < 2 * w->na) return fail(c, SDR_EINVAL, "pcm stride < 2 x audio samples per block");
  rc = stereo_pll(c, audio_fs, st, w);
  if (!rc) rc = stereo_post(c, taps, st, w, pcm, pcm_stride);
  const hipError_t e = w->uses.mark(c->cur);  // marked even after a failed launch
  if (rc) return rc;
  if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
  return SDR_OK;
}

// The back stage in its two halves, for a schedule that keeps the second
// context's stream on the recurrences alone: block b's post stage (NCO,
// stereo resampler, PCM) runs on the front stream after block b+1's front
// stage, beside block b+1's recurrence (bench.py --stereo-pipeline 2).  The
// post stage waits for its block's recurrence (the caller's event); the
// stereo resampler state is the post stage's, the PLL state the recurrence's.
int sdr_stereo_pll_dev(sdr_ctx* c, float audio_fs, sdr_stereo_state* st, sdr_stereo_work* w) {
  int rc = enter(c);
  if (rc) return rc;
  if (!st || !w) return fail(c, SDR_EINVAL, "null state / work");
  rc = stereo_pll(c, audio_fs, st, w);
  const hipError_t e = w->uses.mark(c->cur);  // marked even after a failed launch
  if (rc) return rc;
  if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
  return SDR_OK;
}

int sdr_stereo_post_dev(sdr_ctx* c, const sdr_stereo_taps* taps, sdr_stereo_state* st, sdr_stereo_work* w,
                        int16_t* pcm, long long pcm_stride) {
  int rc = enter(c);
  if (rc) return rc;
  if (!taps || !st || !w || !pcm) return fail(c, SDR_EINVAL, "null taps / state / work / pcm");
  rc = stereo_post(c, taps, st, w, pcm, pcm_stride);
  const hipError_t e = w->uses.mark(c->cur);
  if (rc) return rc;
  if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
  return SDR_OK;
}

// ------------------------------------------------ mono path in two stages --
// sdr_mono_pcm_u8_dev's work cut between the front end and the audio stage,
// one block's demodulated row in a caller-owned work object, so block b+1's
// front end can run on one context's stream while block b's audio stage runs
// on another's (bench.py mono0, like the stereo pair above).  Disjoint state:
// front = RF FIR states and prev_I/Q (src/project.cpp:86-90); back = the delay
// line (:114) and the audio filter state (:116).  Unlike the one-call fused
// layout (where the front end's tile-0 workgroups copy the delay line into the
// row head), the back stage copies the delay line in itself -- the front end
// of the next block may be running, and the delay line belongs to the back.
struct sdr_mono_work {
  int D = 0, up = 0, down = 0, nstreams = 0, ns_delay = 0;
  long long npairs = 0, nd = 0, na = 0, rstride = 0, astride = 0;
  bool fused = false;  // [delay head | demod] rows (up == 1, fast paths): the audio FIR reads them in place
  void* mem = nullptr;
  float *row = nullptr, *delayed = nullptr, *audio = nullptr;  // delayed / audio: the general layout only
  StreamUses uses;
};

int sdr_mono_work_create(sdr_ctx* c, int D, long long npairs, int up, int down, int nstreams, int ns_delay,
                         const float* h_rf, int rf_taps, int ns_rf, const float* h_audio, int audio_taps, int ns_audio,
                         sdr_mono_work** out) {
  int rc = enter(c);
  if (rc) return rc;
  if (!out) return fail(c, SDR_EINVAL, "null work");
  *out = nullptr;
  if (D < 1 || npairs <= 0 || npairs % D || nstreams < 1 || up < 1 || down < 1 || ns_delay < 0)
    return fail(c, SDR_EINVAL, "bad mono work shape");
  auto* w = new sdr_mono_work;
  w->D = D, w->up = up, w->down = down, w->nstreams = nstreams, w->npairs = npairs, w->ns_delay = ns_delay;
  w->nd = npairs / D;
  w->na = sdr_resample_out_len(up, down, w->nd);
  if (w->na <= 0 || w->nd < ns_delay) {
    delete w;
    return fail(c, SDR_EINVAL, "empty audio block, or block shorter than the delay line");
  }
  // the fused layout's conditions (sdr_mono_pcm_u8_dev), row alignment aside
  w->fused = up == 1 && h_rf && h_audio && ns_delay <= 256 && w->nd % down == 0 &&
             sdr::fir_has_fast_path(D, rf_taps, ns_rf, 2, true, sdr::Src::U8) &&
             sdr::fir_has_fast_path(down, audio_taps, ns_audio, 1, false, sdr::Src::F32);
  w->rstride = ((w->fused ? ns_delay : 0) + w->nd + 3) / 4 * 4;
  w->astride = (w->na + 3) / 4 * 4;
  const size_t floats = (size_t)nstreams * (w->rstride + (w->fused ? 0 : w->rstride + w->astride));
  if (hipMalloc(&w->mem, floats * sizeof(float)) != hipSuccess) {
    delete w;
    return fail(c, SDR_ENOMEM, "mono work buffers");
  }
  float* f = static_cast<float*>(w->mem);
  w->row = f, f += (size_t)nstreams * w->rstride;
  if (!w->fused) {
    w->delayed = f, f += (size_t)nstreams * w->rstride;
    w->audio = f;
  }
  *out = w;
  return SDR_OK;
}

int sdr_mono_work_destroy(sdr_ctx* c, sdr_mono_work* w) {
  int rc = enter(c);
  if (rc) return rc;
  if (w) {
    w->uses.wait_and_release();  // the stages may have run on other contexts' streams
    (void)hipFree(w->mem);
    delete w;
  }
  return SDR_OK;
}

// src/project.cpp:72-93: the front end into the work's row
int sdr_mono_front_u8_dev(sdr_ctx* c, const uint8_t* iq, long long iq_stride, const float* h_rf, int rf_taps,
                          float* state_i, float* state_q, int ns_rf, float* prev_i, float* prev_q, sdr_mono_work* w) {
  int rc = enter(c);
  if (rc) return rc;
  if (!w) return fail(c, SDR_EINVAL, "null work");
  rc = sdr_frontend_u8_dev(c, w->D, iq, w->npairs, w->nstreams, iq_stride, h_rf, rf_taps, state_i, state_q, ns_rf,
                           prev_i, prev_q, w->row + (w->fused ? w->ns_delay : 0), w->rstride);
  const hipError_t e = w->uses.mark(c->cur);  // marked even after a failed launch
  if (rc) return rc;
  if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
  return SDR_OK;
}

// src/project.cpp:114-118 + 304-314: delay line, audio filter, s16 PCM
int sdr_mono_back_dev(sdr_ctx* c, const float* h_audio, int audio_taps, float* state_audio, int ns_audio,
                      float* delay_state, sdr_mono_work* w, int16_t* pcm, long long pcm_stride) {
  int rc = enter(c);
  if (rc) return rc;
  if (!w || !pcm || !delay_state) return fail(c, SDR_EINVAL, "null work / pcm / delay state");
  const int n = w->nstreams;
  if (n > 1 && pcm_stride < w->na) return fail(c, SDR_EINVAL, "pcm stride < audio samples per block");
  if (w->fused) {
    // the delay line into the row head (delayBlock's first ns_delay outputs,
    // src/filter.cpp:230-238); the audio FIR then reads [head | demod] in
    // place and copies the row's last ns_delay floats out as the new line
    if (w->ns_delay > 0)
      SDR_HIP(c, hipMemcpy2DAsync(w->row, (size_t)w->rstride * sizeof(float), delay_state,
                                  (size_t)w->ns_delay * sizeof(float), (size_t)w->ns_delay * sizeof(float), (size_t)n,
                                  hipMemcpyDeviceToDevice, c->cur));
    sdr::FirLaunch tail;
    std::memset(&tail, 0, sizeof tail);
    tail.side_src = w->row + w->nd;
    tail.side_src_stride = w->rstride;
    tail.side_dst = delay_state;
    tail.side_dst_stride = w->ns_delay;
    tail.side_n = w->ns_delay;
    rc = fir_decim_dev(c, w->down, w->row, w->nd, n, w->rstride, h_audio, audio_taps, state_audio, ns_audio, nullptr,
                       0, &tail, pcm, n > 1 ? pcm_stride : w->na);
  } else {
    rc = sdr_delay_f32_dev(c, w->row, w->nd, n, w->rstride, delay_state, w->ns_delay, w->delayed, w->rstride);
    if (!rc)
      rc = sdr_resample_f32_dev(c, w->up, w->down, w->delayed, w->nd, n, w->rstride, h_audio, audio_taps, state_audio,
                                ns_audio, w->audio, w->astride);
    if (!rc) rc = sdr_pcm_s16_dev(c, w->audio, w->na, n, w->astride, pcm, pcm_stride);
  }
  const hipError_t e = w->uses.mark(c->cur);
  if (rc) return rc;
  if (e != hipSuccess) return hip_fail(c, e, "hipEventRecord");
  return SDR_OK;
}

int sdr_synth_fm_u8_dev(sdr_ctx* c, uint8_t* iq, long long npairs, int nstreams, long long iq_stride,
                        unsigned long long seed) {
  int rc = enter(c);
  if (rc) return rc;
  if (!iq || npairs <= 0 || nstreams < 1) return fail(c, SDR_EINVAL, "bad synth arguments");
  hipError_t e = sdr::launch_synth_fm_u8(iq, npairs, nstreams, iq_stride, seed, c->cur);
  if (e != hipSuccess) return hip_fail(c, e, "synth launch");
  return SDR_OK;
}

int sdr_u8_to_planar_dev(sdr_ctx* c, const uint8_t* iq, long long npairs, int nstreams, long long iq_stride, float* I,
                         float* Q, long long x_stride) {
  int rc = enter(c);
  if (rc) return rc;
  if (!iq || !I || !Q || npairs <= 0 || nstreams < 1) return fail(c, SDR_EINVAL, "bad u8_to_planar arguments");
  if (!vec_ok(iq, iq_stride, 1, nstreams, 8) || !vec_ok(I, x_stride, 4, nstreams) || !vec_ok(Q, x_stride, 4, nstreams))
    return fail(c, SDR_EINVAL, "u8_to_planar needs 8-B aligned u8 rows and 16-B aligned float rows");
  hipError_t e = sdr::launch_u8_to_planar(iq, npairs, nstreams, iq_stride, I, Q, x_stride, c->cur);
  if (e != hipSuccess) return hip_fail(c, e, "u8_to_planar launch");
  return SDR_OK;
}

// -------------------------------------------------- host, synchronous --
// Each wrapper: copy inputs + state into context scratch, run the device
// path on one stream, copy outputs + state back, synchronise.

int sdr_fir_decim_f32(sdr_ctx* c, int D, const float* x, long long n, const float* h, int ntaps, float* state, int ns,
                      float* y) {
  int rc = enter(c);
  if (rc) return rc;
  if ((rc = check_fir(c, D, n, 1, ntaps, ns, x, h, state))) return rc;
  if (!y) return fail(c, SDR_EINVAL, "null output");
  const long long nout = n / D;
  float* dx = static_cast<float*>(scratch(c, kX0, n * sizeof(float)));
  float* dh = static_cast<float*>(scratch(c, kH, ntaps * sizeof(float)));
  float* ds = static_cast<float*>(scratch(c, kS0, (ns ? ns : 1) * sizeof(float)));
  float* dy = static_cast<float*>(scratch(c, kY0, nout * sizeof(float)));
  if (!dx || !dh || !ds || !dy) return scratch_fail(c, "scratch");
  SDR_HIP(c, hipMemcpyAsync(dx, x, n * sizeof(float), hipMemcpyHostToDevice, c->cur));
  SDR_HIP(c, hipMemcpyAsync(dh, h, ntaps * sizeof(float), hipMemcpyHostToDevice, c->cur));
  if (ns) SDR_HIP(c, hipMemcpyAsync(ds, state, ns * sizeof(float), hipMemcpyHostToDevice, c->cur));
  if ((rc = sdr_fir_decim_f32_dev(c, D, dx, n, 1, n, dh, ntaps, ds, ns, dy, nout))) return rc;
  SDR_HIP(c, hipMemcpyAsync(y, dy, nout * sizeof(float), hipMemcpyDeviceToHost, c->cur));
  if (ns) SDR_HIP(c, hipMemcpyAsync(state, ds, ns * sizeof(float), hipMemcpyDeviceToHost, c->cur));
  SDR_HIP(c, hipStreamSynchronize(c->cur));
  return SDR_OK;
}

int sdr_fir_block_f32(sdr_ctx* c, const float* x, long long n, const float* h, int ntaps, float* state, int ns,
                      float* y) {
  return sdr_fir_decim_f32(c, 1, x, n, h, ntaps, state, ns, y);
}

int sdr_resample_f32(sdr_ctx* c, int up, int down, const float* x, long long n, const float* h, int ntaps,
                     float* state, int ns, float* y, long long y_cap) {
  int rc = enter(c);
  if (rc) return rc;
  if (!x || !h || !state || !y) return fail(c, SDR_EINVAL, "null pointer");
  const long long ny = sdr_resample_out_len(up, down, n);
  if (ny < 0) return fail(c, SDR_EINVAL, "bad up/down");
  if (y_cap < ny) return fail(c, SDR_EINVAL, "output capacity %lld < %lld", y_cap, ny);
  float* dx = static_cast<float*>(scratch(c, kX0, (n > 0 ? n : 1) * sizeof(float)));
  float* dh = static_cast<float*>(scratch(c, kH, ntaps * sizeof(float)));
  float* ds = static_cast<float*>(scratch(c, kS0, (ns ? ns : 1) * sizeof(float)));
  float* dy = static_cast<float*>(scratch(c, kY0, (ny ? ny : 1) * sizeof(float)));
  if (!dx || !dh || !ds || !dy) return scratch_fail(c, "scratch");
  if (n > 0) SDR_HIP(c, hipMemcpyAsync(dx, x, n * sizeof(float), hipMemcpyHostToDevice, c->cur));
  if (ntaps > 0) SDR_HIP(c, hipMemcpyAsync(dh, h, ntaps * sizeof(float), hipMemcpyHostToDevice, c->cur));
  if (ns) SDR_HIP(c, hipMemcpyAsync(ds, state, ns * sizeof(float), hipMemcpyHostToDevice, c->cur));
  if ((rc = sdr_resample_f32_dev(c, up, down, dx, n, 1, n, dh, ntaps, ds, ns, dy, ny))) return rc;
  SDR_HIP(c, hipMemcpyAsync(y, dy, ny * sizeof(float), hipMemcpyDeviceToHost, c->cur));
  if (ns) SDR_HIP(c, hipMemcpyAsync(state, ds, ns * sizeof(float), hipMemcpyDeviceToHost, c->cur));
  SDR_HIP(c, hipStreamSynchronize(c->cur));
  return SDR_OK;
}

int sdr_fm_demod_f32(sdr_ctx* c, const float* I, const float* Q, long long n, float* prev_i, float* prev_q,
                     float* out) {
  int rc = enter(c);
  if (rc) return rc;
  if (!I || !Q || !prev_i || !prev_q || !out) return fail(c, SDR_EINVAL, "null pointer");
  if (n <= 0) return fail(c, SDR_EINVAL, "empty block (reference reads I[-1], filter.cpp:100)");
  float* di = static_cast<float*>(scratch(c, kX0, n * sizeof(float)));
  float* dq = static_cast<float*>(scratch(c, kX1, n * sizeof(float)));
  float* dp = static_cast<float*>(scratch(c, kPrev, 4 * sizeof(float)));
  float* dout = static_cast<float*>(scratch(c, kOut, n * sizeof(float)));
  if (!di || !dq || !dp || !dout) return scratch_fail(c, "scratch");
  SDR_HIP(c, hipMemcpyAsync(di, I, n * sizeof(float), hipMemcpyHostToDevice, c->cur));
  SDR_HIP(c, hipMemcpyAsync(dq, Q, n * sizeof(float), hipMemcpyHostToDevice, c->cur));
  SDR_HIP(c, hipMemcpyAsync(dp, prev_i, sizeof(float), hipMemcpyHostToDevice, c->cur));
  SDR_HIP(c, hipMemcpyAsync(dp + 1, prev_q, sizeof(float), hipMemcpyHostToDevice, c->cur));
  if ((rc = sdr_fm_demod_f32_dev(c, di, dq, n, 1, n, dp, dp + 1, dout, n))) return rc;
  SDR_HIP(c, hipMemcpyAsync(out, dout, n * sizeof(float), hipMemcpyDeviceToHost, c->cur));
  SDR_HIP(c, hipMemcpyAsync(prev_i, dp, sizeof(float), hipMemcpyDeviceToHost, c->cur));
  SDR_HIP(c, hipMemcpyAsync(prev_q, dp + 1, sizeof(float), hipMemcpyDeviceToHost, c->cur));
  SDR_HIP(c, hipStreamSynchronize(c->cur));
  return SDR_OK;
}

static int frontend_host(sdr_ctx* c, sdr::Src src, int D, const float* I, const float* Q, const uint8_t* iq,
                         long long n, const float* h, int ntaps, float* state_i, float* state_q, int ns,
                         float* prev_i, float* prev_q, float* demod) {
  int rc = enter(c);
  if (rc) return rc;
  const void* xin = src == sdr::Src::F32 ? (const void*)I : (const void*)iq;
  if ((rc = check_fir(c, D, n, 1, ntaps, ns, xin, h, state_i))) return rc;
  if ((src == sdr::Src::F32 && !Q) || !state_q || !prev_i || !prev_q || !demod)
    return fail(c, SDR_EINVAL, "null pointer");
  const long long nout = n / D;
  float* dx0 = nullptr;
  float* dx1 = nullptr;
  uint8_t* du = nullptr;
  if (src == sdr::Src::F32) {
    dx0 = static_cast<float*>(scratch(c, kX0, n * sizeof(float)));
    dx1 = static_cast<float*>(scratch(c, kX1, n * sizeof(float)));
    if (!dx0 || !dx1) return scratch_fail(c, "scratch");
  } else {
    du = static_cast<uint8_t*>(scratch(c, kX0, 2 * n));
    if (!du) return scratch_fail(c, "scratch");
  }
  float* dh = static_cast<float*>(scratch(c, kH, ntaps * sizeof(float)));
  float* ds0 = static_cast<float*>(scratch(c, kS0, (ns ? ns : 1) * sizeof(float)));
  float* ds1 = static_cast<float*>(scratch(c, kS1, (ns ? ns : 1) * sizeof(float)));
  float* dp = static_cast<float*>(scratch(c, kPrev, 4 * sizeof(float)));
  float* dout = static_cast<float*>(scratch(c, kOut, nout * sizeof(float)));
  if (!dh || !ds0 || !ds1 || !dp || !dout) return scratch_fail(c, "scratch");
  if (src == sdr::Src::F32) {
    SDR_HIP(c, hipMemcpyAsync(dx0, I, n * sizeof(float), hipMemcpyHostToDevice, c->cur));
    SDR_HIP(c, hipMemcpyAsync(dx1, Q, n * sizeof(float), hipMemcpyHostToDevice, c->cur));
  } else {
    SDR_HIP(c, hipMemcpyAsync(du, iq, 2 * n, hipMemcpyHostToDevice, c->cur));
  }
  SDR_HIP(c, hipMemcpyAsync(dh, h, ntaps * sizeof(float), hipMemcpyHostToDevice, c->cur));
  if (ns) {
    SDR_HIP(c, hipMemcpyAsync(ds0, state_i, ns * sizeof(float), hipMemcpyHostToDevice, c->cur));
    SDR_HIP(c, hipMemcpyAsync(ds1, state_q, ns * sizeof(float), hipMemcpyHostToDevice, c->cur));
  }
  SDR_HIP(c, hipMemcpyAsync(dp, prev_i, sizeof(float), hipMemcpyHostToDevice, c->cur));
  SDR_HIP(c, hipMemcpyAsync(dp + 1, prev_q, sizeof(float), hipMemcpyHostToDevice, c->cur));
  if ((rc = frontend_dev(c, src, D, dx0, dx1, du, n, 1, src == sdr::Src::F32 ? n : 2 * n, dh, ntaps, ds0, ds1, ns,
                         dp, dp + 1, dout, nout)))
    return rc;
  SDR_HIP(c, hipMemcpyAsync(demod, dout, nout * sizeof(float), hipMemcpyDeviceToHost, c->cur));
  if (ns) {
    SDR_HIP(c, hipMemcpyAsync(state_i, ds0, ns * sizeof(float), hipMemcpyDeviceToHost, c->cur));
    SDR_HIP(c, hipMemcpyAsync(state_q, ds1, ns * sizeof(float), hipMemcpyDeviceToHost, c->cur));
  }
  SDR_HIP(c, hipMemcpyAsync(prev_i, dp, sizeof(float), hipMemcpyDeviceToHost, c->cur));
  SDR_HIP(c, hipMemcpyAsync(prev_q, dp + 1, sizeof(float), hipMemcpyDeviceToHost, c->cur));
  SDR_HIP(c, hipStreamSynchronize(c->cur));
  return SDR_OK;
}

int sdr_frontend_f32(sdr_ctx* c, int D, const float* I, const float* Q, long long n, const float* h, int ntaps,
                     float* state_i, float* state_q, int ns, float* prev_i, float* prev_q, float* demod) {
  return frontend_host(c, sdr::Src::F32, D, I, Q, nullptr, n, h, ntaps, state_i, state_q, ns, prev_i, prev_q, demod);
}

int sdr_frontend_u8(sdr_ctx* c, int D, const uint8_t* iq, long long npairs, const float* h, int ntaps,
                    float* state_i, float* state_q, int ns, float* prev_i, float* prev_q, float* demod) {
  return frontend_host(c, sdr::Src::U8, D, nullptr, nullptr, iq, npairs, h, ntaps, state_i, state_q, ns, prev_i,
                       prev_q, demod);
}

// ------------------------------------------ device transcendental routines --
int sdr_libm_sincos_hash_dev(sdr_ctx* c, int mode, unsigned chunk_lo, unsigned chunk_hi, unsigned long long* hash) {
  int rc = enter(c);
  if (rc) return rc;
  if (!hash || (mode != 0 && mode != 1) || chunk_hi > 4096u || chunk_lo >= chunk_hi)
    return fail(c, SDR_EINVAL, "libm sincos hash: mode %d, chunks [%u, %u) of 4096", mode, chunk_lo, chunk_hi);
  SDR_HIP(c, sdr::launch_libm_sincos_hash(mode, chunk_lo, chunk_hi - chunk_lo, hash, c->cur));
  return SDR_OK;
}

int sdr_libm_sincos_diff_dev(sdr_ctx* c, unsigned chunk_lo, unsigned chunk_hi, unsigned long long* count,
                             unsigned* args, long long cap) {
  int rc = enter(c);
  if (rc) return rc;
  if (!count || !args || cap < 0 || chunk_hi > 4096u || chunk_lo >= chunk_hi)
    return fail(c, SDR_EINVAL, "libm sincos diff: chunks [%u, %u) of 4096, cap %lld", chunk_lo, chunk_hi, cap);
  SDR_HIP(c, sdr::launch_libm_sincos_diff(chunk_lo, chunk_hi - chunk_lo, count, args, cap, c->cur));
  return SDR_OK;
}

int sdr_libm_eval_dev(sdr_ctx* c, int fn, const float* a, const float* b, long long n, float* out) {
  int rc = enter(c);
  if (rc) return rc;
  if (!a || !out || fn < 0 || fn > 5 || ((fn == 2 || fn == 5) && !b) || n < 0)
    return fail(c, SDR_EINVAL, "libm eval: fn %d, n %lld", fn, n);
  if (n == 0) return SDR_OK;
  SDR_HIP(c, sdr::launch_libm_eval(fn, a, b, n, out, c->cur));
  return SDR_OK;
}

int sdr_libm_atan2_screen_dev(sdr_ctx* c, unsigned long long seed, unsigned long long first, unsigned long long count,
                              unsigned* cand, long long cand_cap, unsigned* out, long long out_cap,
                              unsigned long long* counters) {
  int rc = enter(c);
  if (rc) return rc;
  if (!cand || !out || !counters || cand_cap < 1 || out_cap < 0 || count == 0 || count > (1ull << 32))
    return fail(c, SDR_EINVAL, "libm atan2 screen: count %llu (1 .. 2^32), cand_cap %lld", count, cand_cap);
  SDR_HIP(c, sdr::launch_libm_atan2_screen(seed, first, count, cand, cand_cap, out, out_cap, counters, c->cur));
  return SDR_OK;
}

}  // extern "C"
