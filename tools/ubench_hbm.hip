// Read-bandwidth ceiling on MI355X for the front end's access pattern:
// two planar f32 arrays (I, Q) streamed once, ~1/20 of the bytes written.
#include <hip/hip_runtime.h>
#include <cstdio>
#include <vector>

// grid-stride: each thread reads U float4 from I and from Q per step
template <int U>
__global__ __launch_bounds__(256) void rd(const float4* __restrict__ I, const float4* __restrict__ Q, long long n4,
                                          float* __restrict__ out) {
  float acc = 0.f;
  const long long stride = (long long)gridDim.x * 256 * U;
  for (long long base = (long long)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
    float4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = base + u * 256;
      a[u] = i < n4 ? I[i] : make_float4(0, 0, 0, 0);
      b[u] = i < n4 ? Q[i] : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += a[u].x + a[u].y + a[u].z + a[u].w + b[u].x + b[u].y + b[u].z + b[u].w;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// tile pattern like fir_tile: each block reads a contiguous 5 KB span per channel per tile, tiles per block contiguous
__global__ __launch_bounds__(64) void tiles(const float4* __restrict__ I, const float4* __restrict__ Q, int tiles_per_blk,
                                            int span4, int adv4, long long n4, float* __restrict__ out) {
  float acc = 0.f;
  for (int t = 0; t < tiles_per_blk; ++t) {
    const long long base = ((long long)blockIdx.x * tiles_per_blk + t) * adv4;
    float4 a[6], b[6];
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const long long i = base + threadIdx.x + u * 64;
      const bool ok = (threadIdx.x + u * 64) < span4 && i < n4;
      a[u] = ok ? I[i] : make_float4(0, 0, 0, 0);
      b[u] = ok ? Q[i] : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < 6; ++u) acc += a[u].x + a[u].y + a[u].z + a[u].w + b[u].x + b[u].y + b[u].z + b[u].w;
  }
  out[blockIdx.x * 64 + threadIdx.x] = acc;
}

int main() {
  const long long n = 1024LL * 65540;  // floats per channel
  const long long n4 = n / 4;
  float4 *I, *Q;
  float* out;
  (void)hipMalloc(&I, n * 4);
  (void)hipMalloc(&Q, n * 4);
  (void)hipMalloc(&out, 64LL << 20);
  (void)hipMemset(I, 0, n * 4);
  (void)hipMemset(Q, 0, n * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  auto time = [&](auto launch, const char* name) {
    for (int w = 0; w < 3; ++w) launch();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 20; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 20;
    printf("%-40s %8.1f us  %6.2f TB/s\n", name, ms * 1e3, 2.0 * n * 4 / (ms * 1e-3) / 1e12);
  };
  for (int g : {1024, 2048, 4096, 8192}) {
    char nm[64];
    snprintf(nm, sizeof nm, "grid-stride U=4 grid=%d", g);
    time([&] { hipLaunchKernelGGL(rd<4>, dim3(g), dim3(256), 0, 0, I, Q, n4, out); }, nm);
  }
  for (int g : {2048, 4096}) {
    char nm[64];
    snprintf(nm, sizeof nm, "grid-stride U=8 grid=%d", g);
    time([&] { hipLaunchKernelGGL(rd<8>, dim3(g), dim3(256), 0, 0, I, Q, n4, out); }, nm);
  }
  // fir-like tiles: 1260 floats advance (315 float4), span 343 float4
  const long long ntiles = n4 / 315;
  for (int tpb : {1, 4, 18}) {
    const int blocks = (int)((ntiles + tpb - 1) / tpb);
    char nm[64];
    snprintf(nm, sizeof nm, "tiles 64-thr, %d tiles/blk (%d blks)", tpb, blocks);
    time([&] { hipLaunchKernelGGL(tiles, dim3(blocks), dim3(64), 0, 0, I, Q, tpb, 343, 315, n4, out); }, nm);
  }
  return 0;
}
