// LDS-read + VALU mix micro-benchmark (gfx950): resample_lp's scan shape --
// K chains per lane, each chunk step one ds_read_b128 per chain (4 inputs)
// then 4 separately rounded multiply-adds per chain against VGPR taps --
// with the reads every chunk (RD = 1, 4 B of LDS per multiply-add, as
// resample_lp), every other chunk (RD = 2: the inputs of one read feed two
// chunks' taps, 2 B per multiply-add, what pairing two phases per lane
// would give) or never (RD = 0).  W waves per SIMD.  Prints cycles per VALU
// instruction per SIMD at the measured clock and LDS bytes per CU cycle.
//   hipcc --offload-arch=gfx950 -O3 -ffp-contract=off -o tools/ubench_ldsmix tools/ubench_ldsmix.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#pragma clang fp contract(off)

typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const f4v lds4;

constexpr int kNC = 39;  // chunks per item scan (151 taps + pad)

template <int K, int NT, int RD>
__global__ __launch_bounds__(256) void mix(const float* __restrict__ taps, float* out, int iters) {
  __shared__ __attribute__((aligned(16))) float buf[64 * 4 * 8 * 4 + 64 * 4];
  const int lane = threadIdx.x & 63;
  for (int i = threadIdx.x; i < (int)(sizeof buf / 4); i += 256) buf[i] = 1.0f + 1e-3f * (i & 255);
  __syncthreads();
  float tp[NT];
#pragma unroll
  for (int u = 0; u < NT; ++u) tp[u] = taps[(lane + u) & 255];
  lds4* ptr[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    // consecutive lanes read consecutive chunks: conflict-free ds_read_b128
    ptr[k] = (lds4*)(buf + 4 * (lane + 64 * k));
    asm volatile("" : "+v"(ptr[k]));
  }
  float acc[K];
  f4v cur[K], nxt[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    acc[k] = 0.0f;
    cur[k] = ptr[k][0];
  }
  for (int it = 0; it < iters; ++it) {
#pragma unroll
    for (int cc = 0; cc < kNC; ++cc) {
      if (RD && (cc % RD) == 0) {
#pragma unroll
        for (int k = 0; k < K; ++k) nxt[k] = ptr[k][(cc & 7) * 64];
      } else {
#pragma unroll
        for (int k = 0; k < K; ++k) {
          nxt[k] = cur[k];
          asm volatile("" : "+v"(nxt[k]));
        }
      }
      __builtin_amdgcn_sched_barrier(0);
#pragma unroll
      for (int jj = 3; jj >= 0; --jj) {
        const int u = (4 * cc + 3 - jj) % NT;
#pragma unroll
        for (int k = 0; k < K; ++k) acc[k] = acc[k] + tp[u] * cur[k][jj];
      }
#pragma unroll
      for (int k = 0; k < K; ++k) {
        cur[k] = nxt[k];
        asm volatile("" : "+v"(acc[k]));
      }
      __builtin_amdgcn_sched_barrier(0);
    }
  }
  float s = 0.0f;
#pragma unroll
  for (int k = 0; k < K; ++k) s += acc[k];
  out[blockIdx.x * 256 + threadIdx.x] = s;
}

template <int K, int NT, int RD>
void run(const char* name, int W, const float* d_taps, float* d_out, int ncu, int clk_khz) {
  const int iters = 64;
  const int blocks = ncu * W;  // 4 waves per block, one per SIMD
  hipLaunchKernelGGL((mix<K, NT, RD>), dim3(blocks), dim3(256), 0, 0, d_taps, d_out, iters);  // warm
  (void)hipDeviceSynchronize();
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  (void)hipEventRecord(e0);
  const int reps = 5;
  for (int r = 0; r < reps; ++r)
    hipLaunchKernelGGL((mix<K, NT, RD>), dim3(blocks), dim3(256), 0, 0, d_taps, d_out, iters);
  (void)hipEventRecord(e1);
  (void)hipEventSynchronize(e1);
  float ms = 0.0f;
  (void)hipEventElapsedTime(&ms, e0, e1);
  ms /= reps;
  const double waves = (double)blocks * 4;
  const double valu = waves * iters * kNC * K * 8.0;
  const double reads = RD ? waves * iters * ((kNC + RD - 1) / RD) * K : 0.0;
  const double cyc = ms * 1e-3 * clk_khz * 1e3;  // per SIMD / per CU over the run
  std::printf("%-34s W=%d  %8.3f ms  %5.2f cyc/VALU/SIMD  LDS %6.1f B/clk/CU  (%4.2f B/MAC)\n", name, W, ms,
              cyc * 4 * ncu / valu, reads * 1024.0 / ncu / cyc, RD ? 4.0 / RD : 0.0);
}

int main() {
  int dev = 0, ncu = 0, clk = 0;
  (void)hipGetDevice(&dev);
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
  (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, dev);
  std::printf("CUs %d, clock %d kHz\n", ncu, clk);
  float* d_taps;
  float* d_out;
  (void)hipMalloc(&d_taps, 256 * 4);
  (void)hipMemset(d_taps, 0, 256 * 4);
  (void)hipMalloc(&d_out, (size_t)ncu * 8 * 256 * 4);
  for (int W = 1; W <= 2; ++W) {
    run<7, 156, 1>("K7 taps156 read every chunk", W, d_taps, d_out, ncu, clk);
    run<7, 156, 2>("K7 taps156 read every 2nd chunk", W, d_taps, d_out, ncu, clk);
    run<7, 156, 0>("K7 taps156 no reads", W, d_taps, d_out, ncu, clk);
  }
  for (int W = 1; W <= 4; ++W) {
    run<4, 64, 1>("K4 taps64 read every chunk", W, d_taps, d_out, ncu, clk);
    run<4, 64, 2>("K4 taps64 read every 2nd chunk", W, d_taps, d_out, ncu, clk);
    run<4, 64, 0>("K4 taps64 no reads", W, d_taps, d_out, ncu, clk);
  }
  return 0;
}
