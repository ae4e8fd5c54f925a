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

// fir_tile-like per-wave step: 6 float4 per lane per channel (one 5.5 KB
// span each of I and Q), optionally stored to LDS (+ barrier) and/or an
// output of 1/20 of the bytes written -- which part of the front end's
// memory path costs what.
template <bool LDS, bool OUT, int WMODE = 0>
__global__ __launch_bounds__(64) void tiles2(const float4* __restrict__ I, const float4* __restrict__ Q,
                                             int tiles_per_blk, int span4, int adv4, long long n4,
                                             float* __restrict__ out) {
  __shared__ float4 l0[6 * 64], l1[6 * 64];
  float acc = 0.f;
  for (int t = 0; t < tiles_per_blk; ++t) {
    const long long tile = (long long)blockIdx.x * tiles_per_blk + t;
    const long long base = tile * adv4;
    float4 a[6], b[6];
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const long long i = base + threadIdx.x + u * 64;
      const bool ok = (threadIdx.x + u * 64) < span4 && i < n4;
      a[u] = ok ? I[i] : make_float4(0, 0, 0, 0);
      b[u] = ok ? Q[i] : make_float4(0, 0, 0, 0);
    }
    if (LDS) {
      __syncthreads();
#pragma unroll
      for (int u = 0; u < 6; ++u) {
        l0[threadIdx.x + 64 * u] = a[u];
        l1[threadIdx.x + 64 * u] = b[u];
      }
      __syncthreads();
      const float4 v = l0[(threadIdx.x * 5) % 384], w = l1[(threadIdx.x * 7) % 384];
      acc += v.x + w.y;
    } else {
#pragma unroll
      for (int u = 0; u < 6; ++u) acc += a[u].x + a[u].y + a[u].z + a[u].w + b[u].x + b[u].y + b[u].z + b[u].w;
    }
    if (OUT) {
      // 128 outputs per tile-wave (2 per lane): 1/20 of the 5 KB read
      float2* o = reinterpret_cast<float2*>(out) + tile * 64 + threadIdx.x;
      if (WMODE == 0) {
        *o = make_float2(acc, acc * 0.5f);
      } else if (WMODE == 1) {
        __builtin_nontemporal_store(acc, &o->x);
        __builtin_nontemporal_store(acc * 0.5f, &o->y);
      } else {
        // stage in LDS, one 2 KB burst per 4 tiles (float4 per lane x 2)
        __shared__ float2 ob[4 * 64];
        ob[(t & 3) * 64 + threadIdx.x] = make_float2(acc, acc * 0.5f);
        if ((t & 3) == 3) {
          __syncthreads();
          float4* o4 = reinterpret_cast<float4*>(out) + (tile - 3) * 32;
          const float4* s4 = reinterpret_cast<const float4*>(ob);
          o4[threadIdx.x] = s4[threadIdx.x];
          o4[threadIdx.x + 64] = s4[threadIdx.x + 64];
          __syncthreads();
        }
      }
    }
  }
  if (!OUT) out[blockIdx.x * 64 + threadIdx.x] = acc;
}

int main() {
  const long long n = 1024LL * 65540;  // floats per channel
  const long long n4 = n / 4;
  float4 *I, *Q;
  float* out;
  (void)hipMalloc(&I, n * 4);
  (void)hipMalloc(&Q, n * 4);
  (void)hipMalloc(&out, 256LL << 20);
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
  for (int tpb : {4, 8}) {
    const int blocks = (int)((ntiles + tpb - 1) / tpb);
    char nm[80];
    snprintf(nm, sizeof nm, "tiles2 lds   %d tiles/blk", tpb);
    time([&] { hipLaunchKernelGGL((tiles2<true, false>), dim3(blocks), dim3(64), 0, 0, I, Q, tpb, 343, 315, n4, out); }, nm);
    snprintf(nm, sizeof nm, "tiles2 out   %d tiles/blk", tpb);
    time([&] { hipLaunchKernelGGL((tiles2<false, true>), dim3(blocks), dim3(64), 0, 0, I, Q, tpb, 343, 315, n4, out); }, nm);
    snprintf(nm, sizeof nm, "tiles2 lds+out %d tiles/blk", tpb);
    time([&] { hipLaunchKernelGGL((tiles2<true, true>), dim3(blocks), dim3(64), 0, 0, I, Q, tpb, 343, 315, n4, out); }, nm);
    snprintf(nm, sizeof nm, "tiles2 out nt %d tiles/blk", tpb);
    time([&] { hipLaunchKernelGGL((tiles2<false, true, 1>), dim3(blocks), dim3(64), 0, 0, I, Q, tpb, 343, 315, n4, out); }, nm);
    snprintf(nm, sizeof nm, "tiles2 out burst4 %d tiles/blk", tpb);
    time([&] { hipLaunchKernelGGL((tiles2<false, true, 2>), dim3(blocks), dim3(64), 0, 0, I, Q, tpb, 343, 315, n4, out); }, nm);
  }
  return 0;
}
