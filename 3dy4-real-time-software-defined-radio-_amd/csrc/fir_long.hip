// fir_long.hip -- long FIRs without decimation: the reference's
// blockConvolveFIR (src/filter.cpp:66-83) for T a multiple of 32 (cfg5:
// T = 1024 on 1 M-sample I and Q blocks).
//
// Same arithmetic contract as fir_tile.hip: y[m] = sum over k = 0..T-1, in
// order, of separately rounded h[k]*x~[m-k] added to an accumulator that
// starts at 0.0f; x~ reads the carried state before the block.
//
// Structure.  A workgroup of NW waves takes 64*R*NW consecutive outputs of
// one stream; its input image (the outputs' span plus a T-1 halo) is
// staged in LDS once with 16-B loads.  Lane l of wave w owns R consecutive
// outputs and walks its window in passes of KP = 32 taps: the pass's taps
// are SGPR operands (one batch of scalar loads, one wait per pass) and its
// inputs are (32 + R)/4 + 1 16-B LDS reads (lane stride R floats:
// conflict-free).  Every pass has the same shape, shifted by 8 chunks, so
// the pass body is unrolled once and looped at run time.  At R = 4 a pass
// is 256 multiplies/adds per lane against 10 LDS reads: VALU-bound, the
// bound of this config (4,096 FLOP per IQ pair).
#include "sdr_common.hpp"

#pragma clang fp contract(off)

namespace sdr {
namespace {

constexpr int kLongKP = 32;  // taps per pass
constexpr int kLongR = 4;    // outputs per lane
constexpr int kLongNW = 4;   // waves per workgroup

struct LongArgs {
  const float* x;
  long long n, x_stride;
  const float* h;
  int ntaps;  // multiple of kLongKP
  const float* state;
  int ns;
  float* y;
  long long y_stride;
  int tiles_per_stream;
  int halo;   // roundup4(ntaps - 1)
  int img;    // LDS floats per workgroup image
};

__global__ __launch_bounds__(64 * kLongNW) void fir_long(LongArgs a) {
  extern __shared__ __attribute__((aligned(16))) float img[];
  constexpr int R = kLongR, KP = kLongKP, NTH = 64 * kLongNW;
  constexpr int OUT_WG = 64 * R * kLongNW;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int s = blockIdx.x / a.tiles_per_stream;
  const int tile = blockIdx.x - s * a.tiles_per_stream;
  const long long m0 = (long long)tile * OUT_WG;      // first output of the workgroup
  const long long pb = m0 - a.halo;                   // stream position of image element 0
  const float* xs = a.x + (long long)s * a.x_stride;
  const float* st = a.state + (long long)s * a.ns;

  // ---- stage [pb, pb + img): 16-B loads, element-wise at the block edges
  const int n4 = a.img >> 2;
  for (int c = tid; c < n4; c += NTH) {
    const long long p = pb + 4LL * c;
    float4 v;
    if (p >= 0 && p + 4 <= a.n) {
      v = *reinterpret_cast<const float4*>(xs + p);
    } else {
      float w[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long long q = p + r;
        w[r] = q >= 0 ? (q < a.n ? xs[q] : 0.0f) : (q >= -a.ns ? st[a.ns + q] : 0.0f);
      }
      v = make_float4(w[0], w[1], w[2], w[3]);
    }
    *reinterpret_cast<float4*>(img + 4 * c) = v;
  }
  __syncthreads();

  // ---- passes.  Lane window: output r of this lane sits at image index
  // lb + halo + r; tap k reads image index lb + halo + r - k.  Pass P covers
  // k in [32P, 32P+32): indices lb + halo - 32P - 32 + (32 + r - kk), kk = k - 32P.
  const int lb = (wave * 64 + lane) * R;
  using hconst = const __attribute__((address_space(4))) float*;
  const hconst hc = (hconst)a.h;
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0f;
  const int npass = a.ntaps / KP;
  constexpr int NC = (KP + R - 1) / 4 + 1;  // chunks per pass (relative indices 1 .. KP+R-1)
  for (int P = 0; P < npass; ++P) {
    float hs[KP];
#pragma unroll
    for (int i = 0; i < KP; ++i) hs[i] = hc[P * KP + i];
#pragma unroll
    for (int i = 0; i < KP; ++i) asm volatile("" : "+s"(hs[i]));
    const float* base = img + lb + a.halo - KP * (P + 1);  // relative index 0, 16-B aligned
    float4 q = *reinterpret_cast<const float4*>(base + 4 * (NC - 1));
#pragma unroll
    for (int c = NC - 1; c >= 0; --c) {
      float4 nx = q;
      if (c > 0) nx = *reinterpret_cast<const float4*>(base + 4 * (c - 1));
      const float e[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 3; j >= 0; --j) {
        const int rel = 4 * c + j;  // = KP + r - kk
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int kk = KP + r - rel;
          if (kk >= 0 && kk < KP) acc[r] = acc[r] + hs[kk] * e[j];
        }
      }
      q = nx;
#pragma unroll
      for (int r = 0; r < R; ++r) asm volatile("" : "+v"(acc[r]));
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  const long long m = m0 + lb;
  float* ys = a.y + (long long)s * a.y_stride;
  if (m + R <= a.n && ((reinterpret_cast<uintptr_t>(ys + m) & 15) == 0)) {
    *reinterpret_cast<float4*>(ys + m) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (m + r < a.n) ys[m + r] = acc[r];
  }
}

// state <- last ns inputs, after every reader of the old state is done.
__global__ __launch_bounds__(kWG) void long_commit(const float* __restrict__ x, long long n, long long x_stride,
                                                   float* state, int ns) {
  const int s = blockIdx.y;
  const int i = blockIdx.x * kWG + threadIdx.x;
  if (i >= ns) return;
  state[(long long)s * ns + i] = x[(long long)s * x_stride + n - ns + i];
}

}  // namespace

bool fir_long_ok(int D, int ntaps, int ns, long long n) {
  return D == 1 && ntaps >= 2 * kLongKP && ntaps % kLongKP == 0 && ns >= ntaps - 1 && n >= ns &&
         ntaps <= 8192;
}

hipError_t launch_fir_long(const FirLaunch& f, const float* h, hipStream_t st) {
  LongArgs a;
  a.x = f.x0;
  a.n = f.n;
  a.x_stride = f.x_stride;
  a.h = h;
  a.ntaps = f.ntaps;
  a.state = f.state0;
  a.ns = f.ns;
  a.y = f.y0;
  a.y_stride = f.y_stride;
  constexpr int OUT_WG = 64 * kLongR * kLongNW;
  a.tiles_per_stream = (int)((f.n + OUT_WG - 1) / OUT_WG);
  a.halo = (f.ntaps - 1 + 3) / 4 * 4;
  a.img = a.halo + OUT_WG + 4;
  const long long blocks = (long long)a.tiles_per_stream * f.nstreams;
  if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fir_long, dim3((unsigned)blocks), dim3(64 * kLongNW), (size_t)a.img * sizeof(float), st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || f.ns <= 0) return e;
  hipLaunchKernelGGL(long_commit, dim3((f.ns + kWG - 1) / kWG, (unsigned)f.nstreams), dim3(kWG), 0, st, f.x0, f.n,
                     f.x_stride, f.state0, f.ns);
  return hipGetLastError();
}

}  // namespace sdr
