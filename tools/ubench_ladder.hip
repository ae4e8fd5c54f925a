// Where the headline kernel's time goes, built up one feature at a time on
// the front end's exact access pattern (1024 streams x 65,540 samples, two
// planar f32 channels, fir_tile's 1-wave tiles: 343 float4 per channel per
// tile, advancing 315 float4):
//   base   register-prefetched tile loads (PF 2), nt
//   +lds   staged into a per-wave LDS span (ds_write_b128), barrier
//   +out   126 floats stored per tile (float2 per lane, 512 B contiguous)
//   +rd    the scan's LDS reads: 56 ds_read_b128 per lane per tile
//   +valu  NV VALU per tile (v_mul with an SGPR operand + v_add, the exact
//          FIR's instruction pair)
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_ladder.hip
#include <hip/hip_runtime.h>

#include <cstdio>
#include <vector>

typedef float f4 __attribute__((ext_vector_type(4)));
typedef unsigned u2 __attribute__((ext_vector_type(2)));

__device__ __forceinline__ float4 ldnt(const float* p) {
  const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
}

template <bool LDS, bool OUT, bool RD, int NV, bool NT, int OM = 0, bool CW = false>
__global__ __launch_bounds__(64) void ladder(const float* __restrict__ I, const float* __restrict__ Q, int rows,
                                             int row4, int tiles_per_row, float* __restrict__ out,
                                             const float* __restrict__ h, int noload) {
  __shared__ __attribute__((aligned(16))) float l0[1376], l1[1376];
  const int total = rows * tiles_per_row;
  int first, step, last;
  if (CW) {  // contiguous run per workgroup
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
  const int lane = threadIdx.x;
  float4 a[2][6], b[2][6];
  auto issue = [&](int lin, float4(&xa)[6], float4(&xb)[6]) {
    const int r = lin / tiles_per_row, t = lin - r * tiles_per_row;
    const long long base = (long long)r * row4 + (long long)t * 315;
#pragma unroll
    for (int u = 0; u < 6; ++u) {
      int e = lane + u * 64;
      e = e < 343 ? e : 342;
      long long i = base + e;
      i = i < (long long)(r + 1) * row4 ? i : (long long)(r + 1) * row4 - 1;
      if (NT) {
        xa[u] = ldnt(I + 4 * i);
        xb[u] = ldnt(Q + 4 * i);
      } else {
        xa[u] = *reinterpret_cast<const float4*>(I + 4 * i);
        xb[u] = *reinterpret_cast<const float4*>(Q + 4 * i);
      }
    }
  };
  const float s0 = h[0], s1 = h[1], s2 = h[2], s3 = h[3];
  float2 obuf[8];
  int k8 = 0;
  float acc0 = 0.f, acc1 = 0.f, acc2 = 0.f, acc3 = 0.f;
#pragma unroll
  for (int u = 0; u < 6; ++u) a[0][u] = a[1][u] = b[0][u] = b[1][u] = make_float4(h[5], 0, 0, 0);
  if (first < last && !noload) issue(first, a[0], b[0]);
  if (first + step < last && !noload) issue(first + step, a[1], b[1]);
  for (int lin = first; lin < last; lin += 2 * step) {
#pragma unroll
    for (int p = 0; p < 2; ++p) {
      const int cur = lin + p * step;
      if (cur >= last) break;
      float4 w0 = a[p][0], w1 = b[p][0];
      if (LDS) {
        __syncthreads();
#pragma unroll
        for (int u = 0; u < 6; ++u) {
          const int e = lane + 64 * u;
          if (e < 344) {
            *reinterpret_cast<float4*>(l0 + 4 * e) = a[p][u];
            *reinterpret_cast<float4*>(l1 + 4 * e) = b[p][u];
          }
        }
        __syncthreads();
      } else {
#pragma unroll
        for (int u = 1; u < 6; ++u) {
          w0.x += a[p][u].x + a[p][u].w;
          w1.y += b[p][u].y + b[p][u].z;
        }
      }
      if (cur + 2 * step < last && !noload) issue(cur + 2 * step, a[p], b[p]);
      if (RD) {
        // 28 chunks x 2 channels of this lane's window (stride 20 floats)
#pragma unroll
        for (int c = 27; c >= 0; --c) {
          const float4 q0 = *reinterpret_cast<const float4*>(l0 + 20 * lane + 4 * c);
          const float4 q1 = *reinterpret_cast<const float4*>(l1 + 20 * lane + 4 * c);
          if (NV == 0) {
            acc0 += q0.x;
            acc1 += q1.y;
          } else {
            // NV/28 VALU per chunk: mul(s) + add pairs on 4 chains
#pragma unroll
            for (int v = 0; v < NV / 28 / 8; ++v) {
              acc0 = acc0 + s0 * q0.x;
              acc1 = acc1 + s1 * q1.x;
              acc2 = acc2 + s2 * q0.y;
              acc3 = acc3 + s3 * q1.y;
            }
          }
          asm volatile("" : "+v"(acc0), "+v"(acc1), "+v"(acc2), "+v"(acc3));
          __builtin_amdgcn_sched_barrier(0);
        }
      } else if (NV > 0) {
        for (int v = 0; v < NV / 8; ++v) {
          acc0 = acc0 + s0 * w0.x;
          acc1 = acc1 + s1 * w1.x;
          acc2 = acc2 + s2 * w0.y;
          acc3 = acc3 + s3 * w1.y;
          asm volatile("" : "+v"(acc0), "+v"(acc1), "+v"(acc2), "+v"(acc3));
        }
      } else {
        acc0 += w0.x + w1.z;
      }
      if (OUT) {
        // OM 0: plain float2 per lane; 1: nt; 2: a 1 MB window (L2-resident);
        // 3: buffered in LDS, 2 KB per 4 tiles; 4: buffer store sc1 (aux 16); 5: aux 3 (sc0 sc1)
        const long long oi = OM == 2 ? ((long long)cur * 64 & ((1 << 17) - 1)) : (long long)cur * 64;
        float2* o = reinterpret_cast<float2*>(out) + oi + lane;
        const float2 v = make_float2(acc0 + acc2, acc1 + acc3);
        if constexpr (OM == 1) {
          __builtin_nontemporal_store(v.x, &o->x);
          __builtin_nontemporal_store(v.y, &o->y);
        } else if constexpr (OM == 3) {
          __shared__ float2 ob[4 * 64];
          __shared__ long long obase[4];
          const int k = ((cur - first) / step) & 3;
          ob[k * 64 + lane] = v;
          if (lane == 0) obase[k] = (long long)cur * 64;
          if (k == 3 || cur + step >= last) {
            __syncthreads();
            for (int kk = 0; kk <= k; ++kk) reinterpret_cast<float2*>(out)[obase[kk] + lane] = ob[kk * 64 + lane];
          }
        } else if constexpr (OM == 6) {  // half the lanes, 16 B each
          if (lane < 32) reinterpret_cast<float4*>(out)[(long long)cur * 32 + lane] = make_float4(v.x, v.y, v.x, v.y);
        } else if constexpr (OM == 7) {  // buffer 8 consecutive tiles in registers, 4 KB burst (contiguous walk)
          static_assert(CW, "OM 7 needs the contiguous walk");
          obuf[k8 & 7] = v;
          if ((k8 & 7) == 7 || cur + 1 >= last) {
            const long long t0 = (long long)cur - (k8 & 7);
#pragma unroll
            for (int kk = 0; kk < 8; ++kk)
              if (kk <= (k8 & 7)) reinterpret_cast<float2*>(out)[(t0 + kk) * 64 + lane] = obuf[kk];
          }
          ++k8;
        } else if constexpr (OM == 4 || OM == 5) {
          const __amdgpu_buffer_rsrc_t rs = __builtin_amdgcn_make_buffer_rsrc(out, 0, 0x7fffffff, 0x00020000);
          __builtin_amdgcn_raw_buffer_store_b64(__builtin_bit_cast(u2, v), rs, (unsigned)((oi + lane) * 8), 0, OM == 4 ? 16 : 3);
        } else {
          *o = v;
        }
      }
    }
  }
  if (!OUT) out[blockIdx.x * 64 + lane] = acc0 + acc1 + acc2 + acc3;
}

int main() {
  const int rows = 1024, row = 65540, row4 = row / 4;
  const long long n = (long long)rows * row;
  float *I, *Q, *out, *h;
  (void)hipMalloc(&I, n * 4);
  (void)hipMalloc(&Q, n * 4);
  (void)hipMalloc(&out, 64 << 20);
  (void)hipMalloc(&h, 4096);
  (void)hipMemset(I, 0, n * 4);
  (void)hipMemset(Q, 0, n * 4);
  (void)hipMemset(h, 0, 4096);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const double bytes = 2.0 * n * 4;
  const int tpr = (row / 10 + 125) / 126;
  auto time = [&](auto launch, const char* name) {
    for (int w = 0; w < 3; ++w) launch();
    (void)hipEventRecord(e0);
    for (int r = 0; r < 20; ++r) launch();
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 20;
    printf("%-40s %8.1f us  %6.2f TB/s\n", name, ms * 1e3, bytes / (ms * 1e-3) / 1e12);
    fflush(stdout);
  };
#define RUN(LDS, OUT, RD, NV, NT, nm) RUNX(LDS, OUT, RD, NV, NT, nm, 0, 0)
#define RUNO(OM, nm) RUNX(true, true, false, 0, true, nm, 0, OM)
#define RUNC(OM, nm) RUNY(true, true, false, 0, true, nm, 0, OM, true)
#define RUNX(LDS, OUT, RD, NV, NT, nm, NOLD, OM) RUNY(LDS, OUT, RD, NV, NT, nm, NOLD, OM, false)
#define RUNY(LDS, OUT, RD, NV, NT, nm, NOLD, OM, CW)                                                                                 \
  for (int wpc : {12, 24}) {                                                                                          \
    char s[96];                                                                                                       \
    snprintf(s, sizeof s, "%s wpc=%d", nm, wpc);                                                                      \
    const int grid = 256 * wpc;                                                                                       \
    time([&] { hipLaunchKernelGGL((ladder<LDS, OUT, RD, NV, NT, OM, CW>), dim3(grid), dim3(64), 0, 0, I, Q, rows, row4, tpr, out, h, NOLD); }, s); \
  }
  RUN(true, false, false, 0, true, "+lds")
  RUN(true, false, false, 0, false, "+lds plain loads")
  RUNY(true, false, false, 0, true, "+lds contiguous walk", 0, 0, true)
  RUNC(0, "+lds+out contiguous walk")
  RUNC(7, "+lds+out contiguous, 8-tile bursts")
  RUNO(6, "+lds+out 16B x 32 lanes")
  RUNO(0, "+lds+out plain")

  return 0;
}
