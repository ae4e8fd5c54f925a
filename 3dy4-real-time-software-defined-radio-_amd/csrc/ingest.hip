// ingest.hip -- wire-format kernels around the front end:
//   * u8 interleaved I/Q -> planar f32, exactly src/iofunc.cpp:117-119's
//     float(((unsigned char)u - 128) / 128.0) followed by the de-interleave
//     of src/project.cpp:78-81;
//   * an on-device synthetic FM source (for the benchmark: no host traffic).
#include "sdr_common.hpp"

namespace sdr {
namespace {

// 4 pairs (8 bytes) per thread: one 8-B load, two 16-B stores.
__global__ __launch_bounds__(kWG) void u8_to_planar(const uint8_t* __restrict__ iq, long long npairs,
                                                    long long iq_stride, float* __restrict__ I,
                                                    float* __restrict__ Q, long long x_stride) {
  const int s = blockIdx.y;
  const long long g = ((long long)blockIdx.x * kWG + threadIdx.x) * 4;
  if (g >= npairs) return;
  const uint8_t* src = iq + (long long)s * iq_stride + 2 * g;
  float* di = I + (long long)s * x_stride + g;
  float* dq = Q + (long long)s * x_stride + g;
  if (g + 4 <= npairs) {
    const uint2 b = *reinterpret_cast<const uint2*>(src);
    *reinterpret_cast<float4*>(di) = make_float4(u8_byte_to_f32<0>(b.x), u8_byte_to_f32<2>(b.x),
                                                 u8_byte_to_f32<0>(b.y), u8_byte_to_f32<2>(b.y));
    *reinterpret_cast<float4*>(dq) = make_float4(u8_byte_to_f32<1>(b.x), u8_byte_to_f32<3>(b.x),
                                                 u8_byte_to_f32<1>(b.y), u8_byte_to_f32<3>(b.y));
  } else {
    for (long long k = 0; g + k < npairs; ++k) {
      di[k] = u8_to_f32(src[2 * k]);
      dq[k] = u8_to_f32(src[2 * k + 1]);
    }
  }
}

__device__ __forceinline__ uint64_t mix64(uint64_t z) {
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ULL;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebULL;
  return z ^ (z >> 31);
}

__device__ __forceinline__ float u01(uint64_t r) { return ((float)(r >> 40) + 0.5f) * (1.0f / 16777216.0f); }

// Noisy FM carrier, per stream its own time offset and noise stream:
// message 0.8 sin(2 pi 1k t) + 0.1 sin(2 pi 19k t), 75 kHz deviation,
// amplitude 0.7, AWGN sigma 0.02, Fs = 2.4 MS/s; u8 = clip(rint(128 x + 128)).
__global__ __launch_bounds__(kWG) void synth_fm_u8(uint8_t* __restrict__ iq, long long npairs, long long iq_stride,
                                                   unsigned long long seed) {
  const int s = blockIdx.y;
  const long long g = (long long)blockIdx.x * kWG + threadIdx.x;
  if (g >= npairs) return;
  const double fs = 2.4e6, dev = 75e3, amp = 0.7;
  const double w1 = 2.0 * M_PI * 1e3, w2 = 2.0 * M_PI * 19e3;
  const double t = (double)(g + (long long)s * 7919LL * 1000LL) / fs;
  const double ph = 2.0 * M_PI * dev * (0.8 * (1.0 - cos(w1 * t)) / w1 + 0.1 * (1.0 - cos(w2 * t)) / w2);
  const uint64_t r1 = mix64(seed ^ mix64((uint64_t)s * 0x9e3779b97f4a7c15ULL + (uint64_t)g));
  const uint64_t r2 = mix64(r1 + 0x632be59bd9b4e019ULL);
  const float rad = sqrtf(-2.0f * logf(u01(r1)));
  const float ang = 6.28318530718f * u01(r2);
  const float ni = 0.02f * rad * cosf(ang), nq = 0.02f * rad * sinf(ang);
  const float vi = (float)(amp * cos(ph)) + ni, vq = (float)(amp * sin(ph)) + nq;
  const float ui = fminf(fmaxf(rintf(128.0f * vi + 128.0f), 0.0f), 255.0f);
  const float uq = fminf(fmaxf(rintf(128.0f * vq + 128.0f), 0.0f), 255.0f);
  uint8_t* d = iq + (long long)s * iq_stride + 2 * g;
  d[0] = (uint8_t)ui;
  d[1] = (uint8_t)uq;
}

}  // namespace

hipError_t launch_u8_to_planar(const uint8_t* iq, long long npairs, int nstreams, long long iq_stride, float* I,
                               float* Q, long long x_stride, hipStream_t st) {
  const long long threads = (npairs + 3) / 4;
  hipLaunchKernelGGL(u8_to_planar, dim3((unsigned)((threads + kWG - 1) / kWG), (unsigned)nstreams), dim3(kWG), 0,
                     st, iq, npairs, iq_stride, I, Q, x_stride);
  return hipGetLastError();
}

hipError_t launch_synth_fm_u8(uint8_t* iq, long long npairs, int nstreams, long long iq_stride,
                              unsigned long long seed, hipStream_t st) {
  hipLaunchKernelGGL(synth_fm_u8, dim3((unsigned)((npairs + kWG - 1) / kWG), (unsigned)nstreams), dim3(kWG), 0, st,
                     iq, npairs, iq_stride, seed);
  return hipGetLastError();
}

}  // namespace sdr
