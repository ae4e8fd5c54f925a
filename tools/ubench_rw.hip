// What do the front end's output writes cost beside its input reads?
// A clean streaming read of the cfg2 input volume (537 MB: 2 x 1024 x 65,540
// f32), with and without a 1/20-volume write stream (the demod output is
// 0.4 B per 8 B read), in several write shapes:
//   ro        read only (float4 per lane, grid-stride, sums kept live)
//   w4        + one float4 store per lane per 20 float4 read, coalesced
//   w2        + one float2 store per lane per 10 float4 read, coalesced
//   w1        + one float store per lane per 5 float4 read, coalesced
//   w4win     as w4 into a 1 MiB window (L2-resident: no HBM writes)
//   w4late    the same bytes written after all reads (per wave, at the end)
//   wo        write only, 27 MB
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_rw.hip -o tools/ubench_rw
#include <hip/hip_runtime.h>

#include <cstdio>

typedef float f4 __attribute__((ext_vector_type(4)));

#define CK(x)                                                                        \
  do {                                                                               \
    hipError_t e_ = (x);                                                             \
    if (e_ != hipSuccess) {                                                          \
      std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
      std::exit(1);                                                                  \
    }                                                                                \
  } while (0)

template <int MODE, bool NT>
__global__ __launch_bounds__(256) void rw(const f4* __restrict__ x, long long n4, f4* __restrict__ out,
                                         long long win4) {
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long nth = (long long)gridDim.x * blockDim.x;
  f4 acc = {0.f, 0.f, 0.f, 0.f};
  constexpr int PER = MODE == 2 ? 10 : MODE == 3 ? 5 : 20;  // float4 read per store
  long long j = 0;                                          // stores so far
  for (long long base = tid; base < n4; base += nth * PER) {
#pragma unroll
    for (int u = 0; u < PER; ++u) {
      const long long i = base + (long long)u * nth;
      if (i < n4) {
        const f4 v = NT ? __builtin_nontemporal_load(x + i) : x[i];
        acc += v;
      }
    }
    if (MODE == 1 || MODE == 4) {
      long long o = j * nth + tid;
      if (MODE == 4) o %= win4;
      out[o] = acc;
    } else if (MODE == 2) {
      reinterpret_cast<float2*>(out)[j * nth + tid] = make_float2(acc.x, acc.y);
    } else if (MODE == 3) {
      reinterpret_cast<float*>(out)[j * nth + tid] = acc.x;
    }
    ++j;
  }
  if (MODE == 5) {  // the same bytes, written at the end
    for (long long k = 0; k < j; ++k) out[k * nth + tid] = acc + (float)k;
  }
  if (MODE == 0 && acc.x == 1234.5f) out[tid] = acc;
}

__global__ __launch_bounds__(256) void wo(f4* __restrict__ out, long long m4) {
  const long long tid = (long long)blockIdx.x * blockDim.x + threadIdx.x;
  const long long nth = (long long)gridDim.x * blockDim.x;
  for (long long i = tid; i < m4; i += nth) out[i] = f4{(float)i, 0.f, 1.f, 2.f};
}

int main() {
  const long long n = 2LL * 1024 * 65540;  // floats read
  const long long n4 = n / 4;
  const long long m4 = n4 / 5 + 65536;  // output float4 (+ slack; w1 writes n4/5 floats)
  f4 *x, *out;
  CK(hipMalloc(&x, n4 * 16));
  CK(hipMalloc(&out, m4 * 16));
  CK(hipMemset(x, 0, n4 * 16));
  CK(hipMemset(out, 0, m4 * 16));
  int ncu = 256;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  hipEvent_t e0, e1;
  CK(hipEventCreate(&e0));
  CK(hipEventCreate(&e1));
  auto timeit = [&](const char* name, auto launch, double bytes) {
    for (int i = 0; i < 3; ++i) launch();
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) launch();
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    ms /= reps;
    std::printf("%-28s %8.1f us  %6.2f TB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
  };
  const double rb = (double)n * 4;
  for (int wpc : {8, 16}) {
    const int grid = ncu * wpc / 4;
    std::printf("-- %d waves per CU (TB/s = read bytes / time)\n", wpc);
    timeit("ro", [&] { rw<0, false><<<grid, 256>>>(x, n4, out, 0); }, rb);
    timeit("ro nt", [&] { rw<0, true><<<grid, 256>>>(x, n4, out, 0); }, rb);
    timeit("w4", [&] { rw<1, false><<<grid, 256>>>(x, n4, out, 0); }, rb);
    timeit("w4 nt", [&] { rw<1, true><<<grid, 256>>>(x, n4, out, 0); }, rb);
    timeit("w2 nt", [&] { rw<2, true><<<grid, 256>>>(x, n4, out, 0); }, rb);
    timeit("w1 nt", [&] { rw<3, true><<<grid, 256>>>(x, n4, out, 0); }, rb);
    timeit("w4win nt", [&] { rw<4, true><<<grid, 256>>>(x, n4, out, 65536); }, rb);
    timeit("w4late nt", [&] { rw<5, true><<<grid, 256>>>(x, n4, out, 0); }, rb);
  }
  timeit("wo 27MB (write bytes)", [&] { wo<<<ncu * 4, 256>>>(out, n4 / 20); }, (double)(n4 / 20) * 16);
  return 0;
}
