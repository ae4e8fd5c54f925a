// Staging structures for the front end's tile walk on MI355X, with the
// scan emulated (28 ds_read_b128 per channel per lane + NV VALU ops per
// tile): register staging (global_load_dwordx4 -> VGPRs -> ds_write_b128,
// prefetch depth 1, as fir_tile) against LDS-DMA staging
// (global_load_lds_dwordx4, NBUF tile buffers in LDS, no VGPR round trip).
// Input: two planar f32 channels of 1024 x 65,540 samples (537 MB); tiles of
// 1,260 new samples + 112 halo per channel, 52 per row; 1/20 of the bytes
// written back.  Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_dma.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdint>

constexpr int kRow = 65540, kRows = 1024, kAdv = 1260, kSpan = 1372, kSpan4 = kSpan / 4;  // 343 chunks
constexpr int kTilesPerRow = 52;

template <bool NT>
__device__ __forceinline__ void glds16(const float* g, uint32_t lds) {
  unsigned keep;
  if constexpr (NT)
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
  else
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds) : "memory");
}

__device__ __forceinline__ void walk_range(int& first, int& step, int& last) {
  const int total = kRows * kTilesPerRow;
  const int per_xcd = (total + 7) / 8;
  const int x = blockIdx.x & 7;
  step = gridDim.x >> 3;
  first = x * per_xcd + (blockIdx.x >> 3);
  last = min((x + 1) * per_xcd, total);
}

// the scan stand-in: this lane's 28-chunk window of both channels, NV
// dependent-free VALU ops (mul + add pairs, as the FIR)
template <int NV>
__device__ __forceinline__ float scan(const float* w0, const float* w1, float s) {
  float a0 = 0.f, a1 = 0.f, a2 = 0.f, a3 = 0.f;
  constexpr int PER = NV / 28 / 4 > 0 ? NV / 28 / 4 : 0;  // mul+add pairs per chunk per channel / 2
#pragma unroll
  for (int c = 27; c >= 0; --c) {
    const float4 q0 = *reinterpret_cast<const float4*>(w0 + 4 * c);
    const float4 q1 = *reinterpret_cast<const float4*>(w1 + 4 * c);
#pragma unroll
    for (int v = 0; v < PER; ++v) {
      a0 = a0 + s * q0.x;
      a1 = a1 + s * q0.y;
      a2 = a2 + s * q1.x;
      a3 = a3 + s * q1.y;
    }
    if (PER == 0) a0 += q0.x + q1.w;
    asm volatile("" : "+v"(a0), "+v"(a1), "+v"(a2), "+v"(a3));
    __builtin_amdgcn_sched_barrier(0);
  }
  return a0 + a1 + a2 + a3;
}

// register staging, prefetch depth 1 (fir_tile's structure)
template <int NV, bool NT>
__global__ __launch_bounds__(64) void regwalk(const float* __restrict__ I, const float* __restrict__ Q,
                                             float* __restrict__ out, float s) {
  __shared__ __attribute__((aligned(16))) float l0[kSpan], l1[kSpan];
  int first, step, last;
  walk_range(first, step, last);
  if (first >= last) return;
  const int lane = threadIdx.x;
  float4 v0[6], v1[6];
  auto load = [&](int lin) {
    const int r = lin / kTilesPerRow, t = lin - r * kTilesPerRow;
    const long long base = (long long)r * kRow + (long long)t * kAdv;
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      int e = lane + 64 * u;
      e = e < kSpan4 ? e : kSpan4 - 1;
      const float4* p0 = reinterpret_cast<const float4*>(I + base) + e;
      const float4* p1 = reinterpret_cast<const float4*>(Q + base) + e;
      if constexpr (NT) {
        typedef float f4 __attribute__((ext_vector_type(4)));
        const f4 a = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p0));
        const f4 b = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p1));
        v0[u] = make_float4(a.x, a.y, a.z, a.w);
        v1[u] = make_float4(b.x, b.y, b.z, b.w);
      } else {
        v0[u] = *p0;
        v1[u] = *p1;
      }
    }
  };
  load(first);
  for (int lin = first; lin < last; lin += step) {
    __syncthreads();
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      const int e = lane + 64 * u;
      if (e < kSpan4) {
        reinterpret_cast<float4*>(l0)[e] = v0[u];
        reinterpret_cast<float4*>(l1)[e] = v1[u];
      }
    }
    __syncthreads();
    if (lin + step < last) load(lin + step);
    const float d = scan<NV>(l0 + 20 * lane, l1 + 20 * lane, s);
    const int r = lin / kTilesPerRow, t = lin - r * kTilesPerRow;
    reinterpret_cast<float2*>(out + (long long)r * (kRow / 10) + t * 126)[lane] = make_float2(d, d);
  }
}

// LDS-DMA staging into NBUF tile buffers; tile i+NBUF-1 is issued before
// tile i is scanned
template <int NV, bool NT, int NBUF>
__global__ __launch_bounds__(64) void dmawalk(const float* __restrict__ I, const float* __restrict__ Q,
                                             float* __restrict__ out, float s) {
  extern __shared__ __attribute__((aligned(16))) float lds[];  // [NBUF][2][kSpan + 12]
  constexpr int BUF = 2 * (kSpan + 12);
  int first, step, last;
  walk_range(first, step, last);
  if (first >= last) return;
  const int lane = threadIdx.x;
  const uint32_t lbase = __builtin_amdgcn_readfirstlane((uint32_t)(uintptr_t)lds);
  // 6 DMA instructions per channel: chunks lane + 64u; the sixth runs its 23
  // live lanes only (an LDS-DMA writes base + 16*lane for the active lanes)
  auto issue = [&](int lin, int b) {
    const int r = lin / kTilesPerRow, t = lin - r * kTilesPerRow;
    const long long base = (long long)r * kRow + (long long)t * kAdv;
    const uint32_t d0 = lbase + 4u * (uint32_t)(b * BUF);
    const uint32_t d1 = d0 + 4u * (kSpan + 12);
#pragma unroll
    for (int u = 0; u < 5; ++u) {
      const int e = lane + 64 * u;
      glds16<NT>(I + base + 4 * e, d0 + 1024u * u);
      glds16<NT>(Q + base + 4 * e, d1 + 1024u * u);
    }
    if (lane + 320 < kSpan4) {
      glds16<NT>(I + base + 4 * (lane + 320), d0 + 5120u);
      glds16<NT>(Q + base + 4 * (lane + 320), d1 + 5120u);
    }
  };
  int nb = 0;
#pragma unroll
  for (int p = 0; p < NBUF - 1; ++p)
    if (first + p * step < last) issue(first + p * step, p);
  int b = 0;
  for (int lin = first; lin < last; lin += step) {
    const int ahead = lin + (NBUF - 1) * step;
    // every tile issues exactly 12 DMAs (dummy re-issue of the current tile
    // past the end keeps the count uniform); the store of each tile is one op
    issue(ahead < last ? ahead : lin, (b + NBUF - 1) % NBUF);
    if constexpr (NBUF == 2)
      asm volatile("s_waitcnt vmcnt(13)" ::: "memory");
    else if constexpr (NBUF == 3)
      asm volatile("s_waitcnt vmcnt(26)" ::: "memory");
    else
      asm volatile("s_waitcnt vmcnt(39)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    const float* l0 = lds + b * BUF;
    const float d = scan<NV>(l0 + 20 * lane, l0 + kSpan + 12 + 20 * lane, s);
    const int r = lin / kTilesPerRow, t = lin - r * kTilesPerRow;
    reinterpret_cast<float2*>(out + (long long)r * (kRow / 10) + t * 126)[lane] = make_float2(d, d);
    b = (b + 1) % NBUF;
    ++nb;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

int main() {
  const long long n = (long long)kRows * kRow;
  float *I, *Q, *out;
  (void)hipMalloc(&I, n * 4 + 4096);
  (void)hipMalloc(&Q, n * 4 + 4096);
  (void)hipMalloc(&out, n / 10 * 4 + 4096);
  (void)hipMemset(I, 0, n * 4);
  (void)hipMemset(Q, 0, n * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double bytes = 2.0 * n * 4 + n / 10 * 4;
  auto time = [&](auto launch, const char* name) {
    for (int w = 0; w < 20; ++w) launch();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 50; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 50;
    printf("%-44s %8.1f us  %6.2f TB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    fflush(stdout);
  };
  char nm[96];
#define RUN(NV)                                                                                                      \
  for (int wpc : {14, 28}) {                                                                                         \
    snprintf(nm, sizeof nm, "reg PF1 nt   wpc=%d nv=%d", wpc, NV);                                                   \
    time([&] { hipLaunchKernelGGL((regwalk<NV, true>), dim3(256 * wpc), dim3(64), 0, 0, I, Q, out, 1.0001f); }, nm); \
  }                                                                                                                  \
  for (int nt = 0; nt < 2; ++nt) {                                                                                   \
    const size_t l2 = 2 * 2 * (kSpan + 12) * 4, l3 = 3 * 2 * (kSpan + 12) * 4;                                       \
    snprintf(nm, sizeof nm, "dma NBUF=2 %s wpc=7 nv=%d", nt ? "nt" : "  ", NV);                                      \
    time([&] {                                                                                                       \
      if (nt) hipLaunchKernelGGL((dmawalk<NV, true, 2>), dim3(256 * 7), dim3(64), l2, 0, I, Q, out, 1.0001f);        \
      else hipLaunchKernelGGL((dmawalk<NV, false, 2>), dim3(256 * 7), dim3(64), l2, 0, I, Q, out, 1.0001f);          \
    }, nm);                                                                                                          \
    snprintf(nm, sizeof nm, "dma NBUF=3 %s wpc=4 nv=%d", nt ? "nt" : "  ", NV);                                      \
    time([&] {                                                                                                       \
      if (nt) hipLaunchKernelGGL((dmawalk<NV, true, 3>), dim3(256 * 4), dim3(64), l3, 0, I, Q, out, 1.0001f);        \
      else hipLaunchKernelGGL((dmawalk<NV, false, 3>), dim3(256 * 4), dim3(64), l3, 0, I, Q, out, 1.0001f);          \
    }, nm);                                                                                                          \
    snprintf(nm, sizeof nm, "dma NBUF=4 %s wpc=3 nv=%d", nt ? "nt" : "  ", NV);                                      \
    time([&] {                                                                                                       \
      if (nt) hipLaunchKernelGGL((dmawalk<NV, true, 4>), dim3(256 * 3), dim3(64), l3 / 3 * 4, 0, I, Q, out, 1.0001f); \
      else hipLaunchKernelGGL((dmawalk<NV, false, 4>), dim3(256 * 3), dim3(64), l3 / 3 * 4, 0, I, Q, out, 1.0001f);   \
    }, nm);                                                                                                          \
  }
  RUN(0)
  RUN(448)
  RUN(896)
  return 0;
}
