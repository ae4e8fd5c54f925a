// resample.hip -- polyphase rational resampler, the reference's
// resampleBlockConvolveFIR (src/filter.cpp:142-173), for up > 1.
// (up == 1 is FIR+decimate by `down` and takes the tiled FIR path.)
//
// Reference loop, restated per output j (n = j*down):
//   p = n mod up,  q = n div up
//   y[j] = sum_{i: k = p + i*up < T} h[k] * x~[q - i]     (ascending k)
// with x~[i] = x[i] for i >= 0 and state[ns + i] before the block (the
// reference's state[state.size() - (k-n)/up]).  Same fp32 op order as the
// reference: separately rounded products and sums from 0.0f.
//
// Layout: a 256-thread workgroup takes 256 consecutive outputs of one
// stream.  Their input windows [q_j - (cnt-1), q_j] overlap heavily
// (consecutive q differ by down/up ~ 5.4 samples at 147/800), so the
// workgroup stages the union of them once in LDS with coalesced loads; each
// lane then walks its own window from LDS.  The taps are re-laid out as a
// polyphase table hp[p][i] = h[p + i*up] (built once per call into device
// scratch) so each lane streams its branch contiguously (16-B loads, L1/L2
// resident: the whole table is T floats).
#include "sdr_common.hpp"

#pragma clang fp contract(off)

namespace sdr {
namespace {

constexpr int kMaxSpan = 8192;  // LDS floats per workgroup for the staged window

// hp[p*cmax + i] = h[p + i*up] for p + i*up < T, else 0 (never read).
__global__ __launch_bounds__(kWG) void build_polyphase(const float* __restrict__ h, int ntaps, int up, int cmax,
                                                       float* hp) {
  const int idx = blockIdx.x * kWG + threadIdx.x;
  if (idx >= up * cmax) return;
  const int p = idx / cmax, i = idx - p * cmax;
  const int k = p + i * up;
  hp[idx] = k < ntaps ? h[k] : 0.0f;
}

__global__ __launch_bounds__(kWG) void resample_tile(const float* __restrict__ x, long long n, long long x_stride,
                                                     const float* __restrict__ hp, int ntaps, int up, int down,
                                                     int cmax, const float* __restrict__ state, int ns,
                                                     float* __restrict__ y, long long y_stride, long long ny) {
  extern __shared__ __attribute__((aligned(16))) float win[];
  const int s = blockIdx.y;
  const long long j0 = (long long)blockIdx.x * kWG;
  const long long jl = j0 + kWG - 1 < ny - 1 ? j0 + kWG - 1 : ny - 1;  // last output of this workgroup
  const long long lo = (j0 * down) / up - (cmax - 1);                  // lowest input index touched
  const long long hi = (jl * down) / up;                               // highest
  const int span = (int)(hi - lo + 1);
  const float* xs = x + (long long)s * x_stride;
  const float* st = state + (long long)s * ns;
  for (int i = threadIdx.x; i < span; i += kWG) {
    const long long g = lo + i;
    win[i] = g >= 0 ? (g < n ? xs[g] : 0.0f) : (g >= -ns ? st[ns + g] : 0.0f);
  }
  __syncthreads();
  const long long j = j0 + threadIdx.x;
  if (j >= ny) return;
  const long long nn = j * down;
  const int p = (int)(nn % up);
  const long long q = nn / up;
  const int cnt = (ntaps - p + up - 1) / up;
  const float* hr = hp + (long long)p * cmax;
  const float* wq = win + (q - lo);
  float acc = 0.0f;
  int i = 0;
  for (; i + 4 <= cnt; i += 4) {
    const float4 hv = *reinterpret_cast<const float4*>(hr + i);
    acc = acc + hv.x * wq[-i];
    acc = acc + hv.y * wq[-i - 1];
    acc = acc + hv.z * wq[-i - 2];
    acc = acc + hv.w * wq[-i - 3];
  }
  for (; i < cnt; ++i) acc = acc + hr[i] * wq[-i];
  y[(long long)s * y_stride + j] = acc;
}

// Fallback when the staged window would not fit LDS (huge down/up ratios):
// the same sum straight from global memory.
__global__ __launch_bounds__(kWG) void resample_direct(const float* __restrict__ x, long long n, long long x_stride,
                                                       const float* __restrict__ hp, int ntaps, int up, int down,
                                                       int cmax, const float* __restrict__ state, int ns,
                                                       float* __restrict__ y, long long y_stride, long long ny) {
  const int s = blockIdx.y;
  const long long j = (long long)blockIdx.x * kWG + threadIdx.x;
  if (j >= ny) return;
  const float* xs = x + (long long)s * x_stride;
  const float* st = state + (long long)s * ns;
  const long long nn = j * down;
  const int p = (int)(nn % up);
  const long long q = nn / up;
  const int cnt = (ntaps - p + up - 1) / up;
  const float* hr = hp + (long long)p * cmax;
  float acc = 0.0f;
  for (int i = 0; i < cnt; ++i) {
    const long long g = q - i;
    const float v = g >= 0 ? xs[g] : st[ns + g];
    acc = acc + hr[i] * v;
  }
  y[(long long)s * y_stride + j] = acc;
}

// state <- last ns inputs (src/filter.cpp:169), after every reader is done.
__global__ __launch_bounds__(kWG) void resample_commit(const float* __restrict__ x, long long n, long long x_stride,
                                                       float* state, int ns) {
  const int s = blockIdx.y;
  const int i = blockIdx.x * kWG + threadIdx.x;
  if (i >= ns) return;
  state[(long long)s * ns + i] = x[(long long)s * x_stride + n - ns + i];
}

}  // namespace

size_t resample_scratch_floats(int up, int ntaps) {
  const int cmax = (ntaps + up - 1) / up;
  return (size_t)up * (size_t)((cmax + 3) / 4 * 4);
}

hipError_t launch_resample(int up, int down, const float* x, long long n, int nstreams, long long x_stride,
                           const float* h, int ntaps, float* state, int ns, float* y, long long y_stride,
                           long long ny, float* scratch_taps, hipStream_t st) {
  const int cmax = ((ntaps + up - 1) / up + 3) / 4 * 4;  // padded row length (16-B rows)
  const int tab = up * cmax;
  hipLaunchKernelGGL(build_polyphase, dim3((tab + kWG - 1) / kWG), dim3(kWG), 0, st, h, ntaps, up, cmax,
                     scratch_taps);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const dim3 grid((unsigned)((ny + kWG - 1) / kWG), (unsigned)nstreams);
  const int cnt_max = (ntaps + up - 1) / up;
  // widest staged window: 256 outputs span (255*down)/up + 1 inputs + taps
  const long long span = (255LL * down) / up + 2 + cmax;
  if (span <= kMaxSpan && cnt_max <= cmax) {
    hipLaunchKernelGGL(resample_tile, grid, dim3(kWG), (size_t)span * sizeof(float), st, x, n, x_stride,
                       scratch_taps, ntaps, up, down, cmax, state, ns, y, y_stride, ny);
  } else {
    hipLaunchKernelGGL(resample_direct, grid, dim3(kWG), 0, st, x, n, x_stride, scratch_taps, ntaps, up, down, cmax,
                       state, ns, y, y_stride, ny);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ns > 0) {
    hipLaunchKernelGGL(resample_commit, dim3((ns + kWG - 1) / kWG, (unsigned)nstreams), dim3(kWG), 0, st, x, n,
                       x_stride, state, ns);
    e = hipGetLastError();
  }
  return e;
}

}  // namespace sdr
