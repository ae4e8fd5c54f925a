// libm_check.hip -- the device's transcendental routines (libm_exact.hpp,
// the ones the PLL and NCO kernels of stereo.hip call) evaluated in bulk, so
// the parity tests can prove on the GPU that they reproduce glibc's floats:
//   - every finite fp32 argument of sin / cos, folded into per-chunk hashes
//     that must equal glibc's (tests/golden/libm_sincos.npz);
//   - the same sweep through ROCm's own double sin / cos (what the PLL used
//     before), listing the arguments where its float differs;
//   - explicit argument lists (the committed near-midpoint fixtures);
//   - a seeded atan2 screen: ~2^36 pairs, every one whose exact value lies
//     within 4 double ulps of a float rounding midpoint written out for the
//     host to check against glibc (the others are decided by the error bounds).
#include <hip/hip_runtime.h>

#include "libm_exact.hpp"
#include "sdr_common.hpp"

#pragma clang fp contract(off)

namespace sdr {
namespace {

__device__ inline unsigned long long sm64(unsigned long long z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
// tests/libm_sweep.cpp rec_hash: one argument's (sin, cos) floats
__device__ inline unsigned long long rec_hash(unsigned u, unsigned s, unsigned c) {
  return sm64(((unsigned long long)u << 32) | s) + sm64((((unsigned long long)u << 32) | c) ^ 0x5bd1e9955bd1e995ull);
}
__device__ inline unsigned fbits(float f) { return __builtin_bit_cast(unsigned, f); }

// mode 0: libmx::sincos_f (the product routine); 1: the platform library in
// double, rounded to float (ROCm's OCML: what the PLL's fallback ran before)
__device__ inline void eval_sincos(int mode, float x, float& s, float& c) {
  if (mode == 0) {
    const libmx::SinCos v = libmx::sincos_f(x);
    s = v.s;
    c = v.c;
  } else {
    s = (float)::sin((double)x);
    c = (float)::cos((double)x);
  }
}

constexpr int kArgsPerThread = 16;
constexpr int kBlocksPerChunk = (1 << 20) / (kWG * kArgsPerThread);  // 256

// grid (kBlocksPerChunk, nchunks): chunk = chunk_lo + blockIdx.y holds the 2^20
// bit patterns u with u >> 20 == chunk; non-finite patterns contribute 0
__global__ __launch_bounds__(kWG) void sincos_hash_kernel(unsigned chunk_lo, int mode,
                                                          unsigned long long* __restrict__ hash) {
  const unsigned chunk = chunk_lo + blockIdx.y;
  unsigned long long h = 0;
  for (int i = 0; i < kArgsPerThread; ++i) {
    const unsigned u = (chunk << 20) | (blockIdx.x * (kWG * kArgsPerThread) + i * kWG + threadIdx.x);
    if ((u & 0x7f800000u) == 0x7f800000u) continue;
    float s, c;
    eval_sincos(mode, __builtin_bit_cast(float, u), s, c);
    h += rec_hash(u, fbits(s), fbits(c));
  }
  __shared__ unsigned long long red[kWG];
  red[threadIdx.x] = h;
  __syncthreads();
  for (int w = kWG / 2; w > 0; w >>= 1) {
    if ((int)threadIdx.x < w) red[threadIdx.x] += red[threadIdx.x + w];
    __syncthreads();
  }
  if (threadIdx.x == 0) atomicAdd(&hash[chunk], red[0]);
}

// arguments where the platform library's float differs from sincos_f's:
// args[2k] = u, args[2k+1] = 1 (sin) | 2 (cos); count[0] = how many
__global__ __launch_bounds__(kWG) void sincos_diff_kernel(unsigned chunk_lo, unsigned long long* __restrict__ count,
                                                          unsigned* __restrict__ args, long long cap) {
  const unsigned chunk = chunk_lo + blockIdx.y;
  for (int i = 0; i < kArgsPerThread; ++i) {
    const unsigned u = (chunk << 20) | (blockIdx.x * (kWG * kArgsPerThread) + i * kWG + threadIdx.x);
    if ((u & 0x7f800000u) == 0x7f800000u) continue;
    const float x = __builtin_bit_cast(float, u);
    float s0, c0, s1, c1;
    eval_sincos(0, x, s0, c0);
    eval_sincos(1, x, s1, c1);
    const unsigned flags = (fbits(s0) != fbits(s1) ? 1u : 0u) | (fbits(c0) != fbits(c1) ? 2u : 0u);
    if (flags) {
      const unsigned long long k = atomicAdd(count, 1ull);
      if ((long long)k < cap) {
        args[2 * k] = u;
        args[2 * k + 1] = flags;
      }
    }
  }
}

// fn: 0 sin_f(a), 1 cos_f(a), 2 atan2_f(a, b); 3..5 the platform library's
__global__ __launch_bounds__(kWG) void eval_kernel(int fn, const float* __restrict__ a, const float* __restrict__ b,
                                                   long long n, float* __restrict__ out) {
  const long long i = (long long)blockIdx.x * kWG + threadIdx.x;
  if (i >= n) return;
  const float x = a[i];
  float r;
  switch (fn) {
    case 0: r = libmx::sin_f(x); break;
    case 1: r = libmx::cos_f(x); break;
    case 2: r = libmx::atan2_f(x, b[i]); break;
    case 3: r = (float)::sin((double)x); break;
    case 4: r = (float)::cos((double)x); break;
    default: r = (float)::atan2((double)x, (double)b[i]); break;
  }
  out[i] = r;
}

// ---- atan2 screen ------------------------------------------------------------
__device__ inline float rnd_float(unsigned long long r, int elo, int ehi) {
  const int e = elo + (int)((r >> 32) % (unsigned long long)(ehi - elo + 1));
  const unsigned be = e < -126 ? 0u : (unsigned)(e + 127);
  return __builtin_bit_cast(float, ((unsigned)(r >> 63) << 31) | (be << 23) | ((unsigned)r & 0x7fffffu));
}
// pair idx of the seeded screen (the families of tests/libm_sweep.cpp)
__device__ inline void screen_pair(unsigned long long seed, unsigned long long idx, float& y, float& x) {
  const unsigned long long r1 = sm64(seed ^ (idx * 0xd1342543de82ef95ull)), r2 = sm64(r1 + 1);
  switch (idx & 3) {
    case 0: {  // the phase detector: v * -fbQ, v * fbI with a pilot-sized v and unit feedback
      const float v = rnd_float(r1, -12, -1);
      const float th = (float)((double)(r2 >> 40) * 0x1p-24 * 6.283185307179586);
      const libmx::SinCos sc = libmx::sincos_f(th);
      y = v * -sc.s;
      x = v * sc.c;
      break;
    }
    case 1:
      y = rnd_float(r1, -60, 60);
      x = rnd_float(r2, -60, 60);
      break;
    case 2:  // near the diagonal (the swap branch) and sign flips
      y = rnd_float(r1, -4, 4);
      x = __builtin_bit_cast(float, fbits(y) ^ (unsigned)(r2 & 0x800000ffull));
      break;
    default:  // the whole float range, subnormals included
      y = rnd_float(r1, -149, 127);
      x = rnd_float(r2, -149, 127);
      break;
  }
}
__device__ inline bool screen_special(float y, float x) {
  return !(__builtin_fabsf(x) <= 0x1.fffffep127f && __builtin_fabsf(y) <= 0x1.fffffep127f) || x == 0.0f ||
         y == 0.0f;
}

// pass 1: every pair the fast path does not certify -> cand (offsets from first)
__global__ __launch_bounds__(kWG) void atan2_fast_kernel(unsigned long long seed, unsigned long long first,
                                                         unsigned long long count, unsigned* __restrict__ cand,
                                                         long long cap, unsigned long long* __restrict__ counters) {
  const unsigned long long stride = (unsigned long long)gridDim.x * kWG;
  for (unsigned long long i = (unsigned long long)blockIdx.x * kWG + threadIdx.x; i < count; i += stride) {
    float y, x;
    screen_pair(seed, first + i, y, x);
    if (screen_special(y, x)) continue;
    unsigned score = ~0u;
    const double a = pllfast::atan2_abs<libmx::ExactOps>(y, x, score);
    if (score < pllfast::kCertified || !libmx::normal_or_float(a)) {
      const unsigned long long k = atomicAdd(&counters[0], 1ull);
      if ((long long)k < cap) cand[k] = (unsigned)i;
    }
  }
}

// pass 2: the candidates through the double-double path; those within 4 ulps
// of a float midpoint -> out[4k..4k+3] = {y, x, atan2_f(y, x), 0}
__global__ __launch_bounds__(kWG) void atan2_slow_kernel(unsigned long long seed, unsigned long long first,
                                                         const unsigned* __restrict__ cand, long long cap,
                                                         unsigned* __restrict__ out, long long out_cap,
                                                         unsigned long long* __restrict__ counters) {
  const unsigned long long ncand = counters[0] < (unsigned long long)cap ? counters[0] : (unsigned long long)cap;
  const unsigned long long stride = (unsigned long long)gridDim.x * kWG;
  for (unsigned long long i = (unsigned long long)blockIdx.x * kWG + threadIdx.x; i < ncand; i += stride) {
    float y, x;
    screen_pair(seed, first + cand[i], y, x);
    unsigned score = ~0u;
    const double a = pllfast::atan2_abs<libmx::ExactOps>(y, x, score);
    const double d = libmx::atan2_slow_d(y, x, __builtin_copysign(a, (double)y));
    if (libmx::near_float_mid(d, 4.0)) {
      const unsigned long long k = atomicAdd(&counters[1], 1ull);
      if ((long long)k < out_cap) {
        out[4 * k] = fbits(y);
        out[4 * k + 1] = fbits(x);
        out[4 * k + 2] = fbits(libmx::atan2_f(y, x));
        out[4 * k + 3] = 0u;
      }
    }
  }
}

}  // namespace

hipError_t launch_libm_sincos_hash(int mode, unsigned chunk_lo, unsigned nchunks, unsigned long long* hash,
                                   hipStream_t st) {
  hipLaunchKernelGGL(sincos_hash_kernel, dim3(kBlocksPerChunk, nchunks), dim3(kWG), 0, st, chunk_lo, mode, hash);
  return hipGetLastError();
}

hipError_t launch_libm_sincos_diff(unsigned chunk_lo, unsigned nchunks, unsigned long long* count, unsigned* args,
                                   long long cap, hipStream_t st) {
  hipLaunchKernelGGL(sincos_diff_kernel, dim3(kBlocksPerChunk, nchunks), dim3(kWG), 0, st, chunk_lo, count, args, cap);
  return hipGetLastError();
}

hipError_t launch_libm_eval(int fn, const float* a, const float* b, long long n, float* out, hipStream_t st) {
  hipLaunchKernelGGL(eval_kernel, dim3((unsigned)((n + kWG - 1) / kWG)), dim3(kWG), 0, st, fn, a, b, n, out);
  return hipGetLastError();
}

hipError_t launch_libm_atan2_screen(unsigned long long seed, unsigned long long first, unsigned long long count,
                                    unsigned* cand, long long cand_cap, unsigned* out, long long out_cap,
                                    unsigned long long* counters, hipStream_t st) {
  const unsigned grid = (unsigned)(device_cu_count() * 16);
  hipLaunchKernelGGL(atan2_fast_kernel, dim3(grid), dim3(kWG), 0, st, seed, first, count, cand, cand_cap, counters);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  hipLaunchKernelGGL(atan2_slow_kernel, dim3(grid), dim3(kWG), 0, st, seed, first, cand, cand_cap, out, out_cap,
                     counters);
  return hipGetLastError();
}

}  // namespace sdr
