// pipeline.hip -- the device-resident mono back end around the front end
// (SURVEY.md section 8(f) rows 2 and 4): delayBlock (src/filter.cpp:230-238
// as src/project.cpp:114 uses it) and the s16 output stage of
// src/project.cpp:311-314, batched over streams.  The audio resampler
// between them is resample.hip / fir_tile.hip.
#include "sdr_common.hpp"

namespace sdr {
namespace {

// out = state ++ in[0 .. n-ns), state <- in[n-ns .. n).  Only workgroup
// (0, s) reads state[s]; it rewrites it after a barrier, so one launch.
__global__ __launch_bounds__(kWG) void delay_kernel(const float* __restrict__ in, long long n, long long in_stride,
                                                    float* state, int ns, float* __restrict__ out,
                                                    long long out_stride) {
  const int s = blockIdx.y;
  const float* x = in + (long long)s * in_stride;
  float* y = out + (long long)s * out_stride;
  float* st = state + (long long)s * ns;
  for (long long i = (long long)blockIdx.x * kWG + threadIdx.x; i < n; i += (long long)gridDim.x * kWG)
    y[i] = i < ns ? st[i] : x[i - ns];
  if (blockIdx.x == 0) {
    __syncthreads();  // every read of the old state in this workgroup is done
    for (int j = threadIdx.x; j < ns; j += kWG) st[j] = x[n - ns + j];
  }
}

// The same with V-float vector accesses (V = 4 or 2), when ns, n and both
// row strides are multiples of V and the rows V*4-byte aligned: every vector
// of out then comes whole from state or from in (the reference's mono delay
// is (101 taps)/2 = 50 samples: V = 2).  A pure copy, the scalar kernel's bits.
template <class VT>
__global__ __launch_bounds__(kWG) void delay_kernel_v(const VT* __restrict__ in, long long nv, long long in_stride_v,
                                                      VT* state, int nsv, VT* __restrict__ out, long long out_stride_v) {
  const int s = blockIdx.y;
  const VT* x = in + (long long)s * in_stride_v;
  VT* y = out + (long long)s * out_stride_v;
  VT* st = state + (long long)s * nsv;
  for (long long i = (long long)blockIdx.x * kWG + threadIdx.x; i < nv; i += (long long)gridDim.x * kWG)
    y[i] = i < nsv ? st[i] : x[i - nsv];
  if (blockIdx.x == 0) {
    __syncthreads();  // every read of the old state in this workgroup is done
    for (int j = threadIdx.x; j < nsv; j += kWG) st[j] = x[nv - nsv + j];
  }
}

// src/project.cpp:311-314 (pcm_quantise, sdr_common.hpp)
__global__ __launch_bounds__(kWG) void pcm_kernel(const float* __restrict__ x, long long n, long long x_stride,
                                                  int16_t* __restrict__ pcm, long long pcm_stride) {
  const int s = blockIdx.y;
  const long long i = (long long)blockIdx.x * kWG + threadIdx.x;
  if (i >= n) return;
  pcm[(long long)s * pcm_stride + i] = pcm_quantise(x[(long long)s * x_stride + i]);
}

}  // namespace

hipError_t launch_delay(const float* in, long long n, int nstreams, long long in_stride, float* state, int ns,
                        float* out, long long out_stride, hipStream_t st) {
  const uintptr_t align = reinterpret_cast<uintptr_t>(in) | reinterpret_cast<uintptr_t>(out) |
                          reinterpret_cast<uintptr_t>(state);
  auto vec_ok = [&](int V) {
    return n % V == 0 && ns % V == 0 && in_stride % V == 0 && out_stride % V == 0 && (align & (4 * V - 1)) == 0;
  };
  if (n >= ns && (vec_ok(4) || vec_ok(2))) {
    const int V = vec_ok(4) ? 4 : 2;
    long long gx = (n / V + kWG - 1) / kWG;
    if (gx > 1024) gx = 1024;
    if (V == 4)
      hipLaunchKernelGGL(delay_kernel_v<float4>, dim3((unsigned)gx, (unsigned)nstreams), dim3(kWG), 0, st,
                         reinterpret_cast<const float4*>(in), n / 4, in_stride / 4, reinterpret_cast<float4*>(state),
                         ns / 4, reinterpret_cast<float4*>(out), out_stride / 4);
    else
      hipLaunchKernelGGL(delay_kernel_v<float2>, dim3((unsigned)gx, (unsigned)nstreams), dim3(kWG), 0, st,
                         reinterpret_cast<const float2*>(in), n / 2, in_stride / 2, reinterpret_cast<float2*>(state),
                         ns / 2, reinterpret_cast<float2*>(out), out_stride / 2);
    return hipGetLastError();
  }
  long long gx = (n + kWG - 1) / kWG;
  if (gx > 1024) gx = 1024;
  hipLaunchKernelGGL(delay_kernel, dim3((unsigned)gx, (unsigned)nstreams), dim3(kWG), 0, st, in, n, in_stride, state,
                     ns, out, out_stride);
  return hipGetLastError();
}

hipError_t launch_pcm(const float* x, long long n, int nstreams, long long x_stride, int16_t* pcm,
                      long long pcm_stride, hipStream_t st) {
  hipLaunchKernelGGL(pcm_kernel, dim3((unsigned)((n + kWG - 1) / kWG), (unsigned)nstreams), dim3(kWG), 0, st, x, n,
                     x_stride, pcm, pcm_stride);
  return hipGetLastError();
}

}  // namespace sdr
