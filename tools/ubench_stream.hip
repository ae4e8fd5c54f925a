// Streaming-read ceilings on MI355X for the front end's input (two planar
// f32 channels of 1024 x 65,540 samples, 537 MB), by load cache policy and
// access shape.  Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_stream.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));

// POL 0: plain global_load_dwordx4; 1: nontemporal (nt); 2: buffer load aux=2 (nt); 3: aux=1 (sc0)
template <int POL>
__device__ __forceinline__ float4 ld(const float4* p, __amdgpu_buffer_rsrc_t rs, unsigned off) {
  if constexpr (POL == 0) return *p;
  if constexpr (POL == 1) {
    const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
    return make_float4(v.x, v.y, v.z, v.w);
  }
  if constexpr (POL == 2) {
    auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 2);
    return make_float4(__builtin_bit_cast(float, v[0]), __builtin_bit_cast(float, v[1]),
                       __builtin_bit_cast(float, v[2]), __builtin_bit_cast(float, v[3]));
  }
  auto v = __builtin_amdgcn_raw_buffer_load_b128(rs, off, 0, 1);
  return make_float4(__builtin_bit_cast(float, v[0]), __builtin_bit_cast(float, v[1]),
                     __builtin_bit_cast(float, v[2]), __builtin_bit_cast(float, v[3]));
}

template <int U, int POL>
__global__ __launch_bounds__(256) void gs(const float4* __restrict__ I, const float4* __restrict__ Q, long long n4,
                                          float* __restrict__ out) {
  static_assert(POL < 2, "grid-stride: global loads only");
  const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc((void*)I, 0, 0, 0x00020000);
  float acc = 0.f;
  const long long stride = (long long)gridDim.x * 256 * U;
  for (long long base = (long long)blockIdx.x * 256 * U + threadIdx.x; base < n4; base += stride) {
    float4 a[U], b[U];
#pragma unroll
    for (int u = 0; u < U; ++u) {
      const long long i = base + u * 256;
      a[u] = i < n4 ? ld<POL>(I + i, rs, 0) : make_float4(0, 0, 0, 0);
      b[u] = i < n4 ? ld<POL>(Q + i, rs, 0) : make_float4(0, 0, 0, 0);
    }
#pragma unroll
    for (int u = 0; u < U; ++u) acc += a[u].x + a[u].y + a[u].z + a[u].w + b[u].x + b[u].y + b[u].z + b[u].w;
  }
  out[blockIdx.x * 256 + threadIdx.x] = acc;
}

// fir_tile's shape: a tile is 343 float4 of I and of Q starting at tile*315
// (1,260 new samples + the 112-sample halo) within one stream row of
// ROW4 float4; tiles_per_row tiles per row.  One wave per workgroup,
// persistent: workgroup b walks tiles b, b+G, ... (XCD interleaved) or a
// contiguous run (CONTIG), PF tiles of register prefetch.  VALU: NV
// dependent-free adds per tile to emulate the scan.
template <int PF, int POL, bool CONTIG>
__global__ __launch_bounds__(64) void walk(const float* __restrict__ I, const float* __restrict__ Q, int rows,
                                           int row4, int tiles_per_row, int nv, float* __restrict__ out,
                                           unsigned long long* clk) {
  const unsigned long long c0_ = clock64(), w0_ = wall_clock64();
  const bool noload = nv < 0;  // nv < 0: VALU only, no loads
  nv = noload ? -nv : nv;
  const int total = rows * tiles_per_row;
  int first, step, last;
  if (CONTIG) {
    const int per = (total + gridDim.x - 1) / gridDim.x;
    first = blockIdx.x * per;
    step = 1;
    last = min(first + per, total);
  } else {
    const int per_xcd = (total + 7) / 8;
    const int x = blockIdx.x & 7;
    step = gridDim.x >> 3;
    first = x * per_xcd + (blockIdx.x >> 3);
    last = min((x + 1) * per_xcd, total);
  }
  __amdgpu_buffer_rsrc_t ri = __builtin_amdgcn_make_buffer_rsrc((void*)I, 0, 0x7fffffff, 0x00020000);
  __amdgpu_buffer_rsrc_t rq = __builtin_amdgcn_make_buffer_rsrc((void*)Q, 0, 0x7fffffff, 0x00020000);
  float acc = 0.f, c0 = 1.f, c1 = 1.f, c2 = 1.f, c3 = 1.f;
  float4 a[PF][6], b[PF][6];
  const float lin0f = (float)first;
  auto issue = [&](int lin, float4(&x)[6], float4(&y)[6]) {
    const int r = lin / tiles_per_row, t = lin - r * tiles_per_row;
    const long long base = (long long)r * row4 + (long long)t * 315;
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      int e = threadIdx.x + u * 64;
      e = e < 343 ? e : 342;
      long long i = base + e;
      i = i < (long long)(r + 1) * row4 ? i : (long long)(r + 1) * row4 - 1;
      // buffer offsets are 32-bit: rebase per row
      x[u] = ld<POL>(reinterpret_cast<const float4*>(I) + i, ri, (unsigned)(i * 16));
      y[u] = ld<POL>(reinterpret_cast<const float4*>(Q) + i, rq, (unsigned)(i * 16));
    }
  };
#pragma unroll
  for (int p = 0; p < PF; ++p)
    if (first + p * step < last) {
      if (noload) {
#pragma unroll
        for (int u = 0; u < 6; ++u) a[p][u] = b[p][u] = make_float4(lin0f, 0, 0, 0);
      } else {
        issue(first + p * step, a[p], b[p]);
      }
    }
  for (int lin = first; lin < last; lin += PF * step) {
#pragma unroll
    for (int p = 0; p < PF; ++p) {
      const int cur = lin + p * step;
      if (cur < last) {
        float s = 0.f;
#pragma unroll
        for (int u = 0; u < 6; ++u) s += a[p][u].x + a[p][u].y + a[p][u].z + a[p][u].w + b[p][u].x + b[p][u].w;
        if (cur + PF * step < last && !noload) issue(cur + PF * step, a[p], b[p]);
        for (int v = 0; v < nv; v += 4) {  // nv independent-chain VALU ops
          c0 = c0 * 1.0001f + s;
          c1 = c1 * 0.9999f + s;
          c2 = c2 * 1.0002f + s;
          c3 = c3 * 0.9998f + s;
          asm volatile("" : "+v"(c0), "+v"(c1), "+v"(c2), "+v"(c3));
        }
        acc += s;
      }
    }
  }
  out[blockIdx.x * 64 + threadIdx.x] = acc + c0 + c1 + c2 + c3;
  if (threadIdx.x == 0) {
    clk[2 * blockIdx.x] = clock64() - c0_;
    clk[2 * blockIdx.x + 1] = wall_clock64() - w0_;
  }
}

int main(int argc, char** argv) {
  const int rows = 1024, row = 65540, row4 = row / 4;
  const long long n = (long long)rows * row, n4 = n / 4;
  float *I, *Q, *out;
  (void)hipMalloc(&I, n * 4);
  (void)hipMalloc(&Q, n * 4);
  (void)hipMalloc(&out, 64 << 20);
  (void)hipMemset(I, 0, n * 4);
  (void)hipMemset(Q, 0, n * 4);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double bytes = 2.0 * n * 4;
  unsigned long long* clk;
  (void)hipMalloc(&clk, 2 * 256 * 64 * sizeof(unsigned long long));
  int wall_khz = 0;
  (void)hipDeviceGetAttribute(&wall_khz, hipDeviceAttributeWallClockRate, 0);
  int nclk = 0;  // blocks of the last launch that recorded clocks
  auto time = [&](auto launch, const char* name) {
    for (int w = 0; w < 3; ++w) launch();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 20; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 20;
    double sclk = 0;
    if (nclk) {
      std::vector<unsigned long long> h(2 * nclk);
      (void)hipMemcpy(h.data(), clk, h.size() * 8, hipMemcpyDeviceToHost);
      double c = 0, w = 0;
      for (int i = 0; i < nclk; ++i) c += h[2 * i], w += h[2 * i + 1];
      sclk = w > 0 ? c / w * wall_khz / 1e6 : 0;  // GHz
    }
    printf("%-52s %8.1f us  %6.2f TB/s  sclk %.2f GHz\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12, sclk);
    nclk = 0;
    fflush(stdout);
  };
  char nm[96];
  for (int g : {2048, 4096, 8192}) {
    snprintf(nm, sizeof nm, "gs U=4 grid=%d plain", g);
    time([&] { hipLaunchKernelGGL((gs<4, 0>), dim3(g), dim3(256), 0, 0, (const float4*)I, (const float4*)Q, n4, out); }, nm);
    snprintf(nm, sizeof nm, "gs U=4 grid=%d nt", g);
    time([&] { hipLaunchKernelGGL((gs<4, 1>), dim3(g), dim3(256), 0, 0, (const float4*)I, (const float4*)Q, n4, out); }, nm);
  }
  const int tpr = (row / 10 + 125) / 126;  // fir_tile's tiles per stream at D=10, R=2
  for (int nv : {0, 200, 400, 800, -400, -800}) {
    for (int wpc : {12, 24}) {
      const int grid = 256 * wpc;
      snprintf(nm, sizeof nm, "walk PF2 xcd plain wpc=%d nv=%d", wpc, nv);
      time([&] { nclk = grid; hipLaunchKernelGGL((walk<2, 0, false>), dim3(grid), dim3(64), 0, 0, I, Q, rows, row4, tpr, nv, out, clk); }, nm);
      snprintf(nm, sizeof nm, "walk PF2 xcd nt wpc=%d nv=%d", wpc, nv);
      time([&] { nclk = grid; hipLaunchKernelGGL((walk<2, 1, false>), dim3(grid), dim3(64), 0, 0, I, Q, rows, row4, tpr, nv, out, clk); }, nm);
      snprintf(nm, sizeof nm, "walk PF2 contig nt wpc=%d nv=%d", wpc, nv);
      time([&] { nclk = grid; hipLaunchKernelGGL((walk<2, 1, true>), dim3(grid), dim3(64), 0, 0, I, Q, rows, row4, tpr, nv, out, clk); }, nm);
      snprintf(nm, sizeof nm, "walk PF3 xcd nt wpc=%d nv=%d", wpc, nv);
      time([&] { nclk = grid; hipLaunchKernelGGL((walk<3, 1, false>), dim3(grid), dim3(64), 0, 0, I, Q, rows, row4, tpr, nv, out, clk); }, nm);
    }
  }
  return 0;
}
