// fir_stream.hip -- the fused RF front end (FIR + decimate + discriminator,
// src/filter.cpp:85-102 and 123-140, sequenced as in src/project.cpp:86-90)
// as a loader / consumer engine: one persistent workgroup per CU, one
// LOADER wave that only streams tile spans from HBM into a ring of LDS slots
// by LDS-DMA, and NC CONSUMER waves that only compute.
//
// Why: the register-staged tile kernel issues a tile's
// loads, then computes for longer than their latency, so its HBM queue runs
// dry while it computes -- loads alone reach ~6.6 TB/s and the scan alone is
// well under the load time, yet the two together overlap poorly.  Here the
// loader's queue never waits on arithmetic: it keeps DEPTH tiles (~55 KB)
// in flight per CU whenever a slot is free, and the consumers, which need
// no staging registers, read their spans straight out of the ring.
//
// Arithmetic, tile geometry, edge handling and the state carry are exactly
// fir_tile's single-wave tile (fir_parts.hpp): a consumer wave computes one
// tile of 64 lanes x R outputs, taps as SGPR operands, every product and sum
// rounded separately in the reference's order -- bit-exact.
//
// Ring protocol (all flags in LDS, one workgroup):
//   * the workgroup owns tiles [first, first + cnt) (local index j); tile j
//     uses slot j % NSLOT and is computed by consumer j % NC;
//   * loader: may fill slot s for tile j once freed[s] == j - NSLOT; it
//     issues NI LDS-DMA instructions per tile, and publishes ready[s] = j
//     after its own s_waitcnt vmcnt shows that tile's DMAs have landed
//     (vmcnt counts in order; the loader issues no other vector memory op);
//   * consumer: waits for ready[s] == j, fixes up edge tiles, scans, drains
//     its LDS reads (lgkmcnt(0)) and sets freed[s] = j, then runs the
//     discriminator, the stores and (tile 0) the state carry.
#include <cstdio>
#include <cstdlib>

#include "fir_parts.hpp"
#include "sdr_common.hpp"

#pragma clang fp contract(off)

#ifndef SDR_STREAM_NL
#define SDR_STREAM_NL 4
#endif

namespace sdr {
namespace {

template <int D, int T, int R>
struct Ring {
  using G = Geom<D, T, R, true, 1>;                        // one consumer wave = one fir_tile tile
  static constexpr int NL = SDR_STREAM_NL;                 // loader waves (one LDS-DMA issues in ~60-180 cycles)
  static constexpr int NC = 8;                             // consumer waves (2 per SIMD)
  static constexpr int CH4 = G::LDS4;                      // float4 per channel per slot
  static constexpr int NI_CH = (CH4 + 63) / 64;            // DMA wave-instructions per channel
  static constexpr int NI = 2 * NI_CH;                     // ... per tile
  static constexpr int SLOT = 2 * G::LDS_LEN;              // floats per slot (I then Q)
  static constexpr int STRIPS = NC * 2 * G::STRIP;         // per-consumer tail strips (tile 0)
  static constexpr int LDS_BYTES = 160 * 1024 - 512;       // leave room for the flags
  static constexpr int NSLOT = (LDS_BYTES / 4 - STRIPS) / SLOT;
  static constexpr int DEPTH0 = 63 / NI;                   // vmcnt is 6 bits
  static constexpr int DEPTH1 = (NSLOT - NC + NL - 1) / NL;
  static constexpr int DEPTH = DEPTH0 < DEPTH1 ? DEPTH0 : DEPTH1;  // tiles in flight per loader
  static_assert(G::LDS_LEN % 4 == 0, "16-B aligned channel images");
  static_assert(DEPTH >= 1, "ring too small for the consumers");
};

// LDS byte address of a pointer into __shared__ memory.
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
  return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}

// One 16-B-per-lane LDS-DMA: lane i's float4 at g lands at lds_byte + 16 i.
// Hidden from hipcc's waitcnt bookkeeping on purpose (the loader counts its
// own vmcnt); M0 is saved and restored inside the statement.
template <bool NT>
__device__ __forceinline__ void dma16(const float* g, uint32_t lds_byte) {
  uint32_t keep;
  if constexpr (NT) {
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off nt\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds_byte) : "memory");
  } else {
    asm volatile("s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\ts_mov_b32 m0, %0"
                 : "=&s"(keep) : "v"(g), "s"(lds_byte) : "memory");
  }
}

// s_waitcnt vmcnt(k * NI) for a run-time k in [0, DEPTH).
template <int NI, int DEPTH>
__device__ __forceinline__ void wait_tiles(int k) {
  static_for<0, DEPTH>([&](auto i) {
    constexpr int K = decltype(i)::value;
    if (k == K) asm volatile("s_waitcnt vmcnt(%0)" ::"i"(K * NI) : "memory");
  });
}

// Ring flags: plain ds_read / ds_write (an access through a generic pointer
// would be a flat op, which also counts in vmcnt -- the loader's DMA count).
typedef __attribute__((address_space(3))) int lds_int;
__device__ __forceinline__ int lds_ld(const int* p) {
  return __builtin_amdgcn_readfirstlane(*(volatile const lds_int*)p);
}
__device__ __forceinline__ void lds_st(int* p, int v) { *(volatile lds_int*)p = v; }

template <int D, int T, int R, bool NT>
__global__ __launch_bounds__(64 * (Ring<D, T, R>::NC + Ring<D, T, R>::NL)) void fir_stream(FirLaunch a, const float* __restrict__ h) {
  using RG = Ring<D, T, R>;
  using G = typename RG::G;
  constexpr int NL = RG::NL, NC = RG::NC, NSLOT = RG::NSLOT, SLOT = RG::SLOT;
  __shared__ __attribute__((aligned(16))) float slots[NSLOT * SLOT];
  __shared__ __attribute__((aligned(16))) float strips[RG::STRIPS];
  __shared__ int ready[NSLOT], freed[NSLOT];

  const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), lane = threadIdx.x & 63;
  const long long n = a.n;
  const long long nout = n / D;
  const int ns = a.ns;
  // this workgroup's tiles: a contiguous run (stream-major order), so
  // consecutive tiles' halos are the previous span's tail (L2 hits)
  const int total = a.nstreams * a.tiles_per_stream;
  const int per = total / (int)gridDim.x, extra = total % (int)gridDim.x;
  const int first = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int cnt = per + ((int)blockIdx.x < extra ? 1 : 0);
  if (threadIdx.x < NSLOT) {
    ready[threadIdx.x] = -1;
    freed[threadIdx.x] = (int)threadIdx.x - NSLOT;
  }
  __syncthreads();
  if (cnt <= 0) return;

  if (wave < NL) {
    // ------------------------------------------------------------ loader --
    const long long n4 = n & ~3LL;
    auto issue = [&](int j) {
      const TileRef tr = tile_ref<D, T, R, true, 1, 2, Src::F32>(a, first + j);
      const bool clamp = !(tr.pb >= 0 && tr.pb + G::LDS_LEN <= n);
      float* slot = slots + (j % NSLOT) * SLOT;
#pragma unroll
      for (int c = 0; c < 2; ++c) {
        const float* x = c ? tr.x1 : tr.x0;
#pragma unroll
        for (int u = 0; u < RG::NI_CH; ++u) {
          const int e = 64 * u + lane;
          long long p = tr.pb + 4LL * e;
          if (clamp) p = p < 0 ? 0 : (p > n4 - 4 ? n4 - 4 : p);
          const uint32_t dst = __builtin_amdgcn_readfirstlane(lds_addr(slot + c * G::LDS_LEN + 256 * u));
          if (u + 1 < RG::NI_CH || e < RG::CH4) dma16<NT>(x + p, dst);
        }
      }
    };
    // loader `wave` moves tiles wave, wave + NL, ...: ji / jp count them
    const int mine = cnt > wave ? (cnt - wave + NL - 1) / NL : 0;
    int ji = 0, jp = 0;  // next of mine to issue / to publish
    while (jp < mine) {
      const int j = wave + NL * ji;
      if (ji < mine && ji - jp < RG::DEPTH && lds_ld(&freed[j % NSLOT]) == j - NSLOT) {
        if (a.ablate != 1) issue(j);  // ablate 1 (timing only): no HBM loads
        ++ji;
      } else if (ji > jp) {
        wait_tiles<RG::NI, RG::DEPTH>(ji - jp - 1);  // that tile's DMAs have landed
        const int jq = wave + NL * jp;
        if (lane == 0) lds_st(&ready[jq % NSLOT], jq);
        ++jp;
      } else {
        __builtin_amdgcn_s_sleep(1);
      }
    }
    return;
  }

  // ------------------------------------------------------------- consumer --
  const int cw = wave - NL;
  float* strip0 = strips + cw * 2 * G::STRIP;
  float* strip1 = strip0 + G::STRIP;
  const int lbase = D * R * lane;  // this lane's window in the slot
  for (int j = cw; j < cnt; j += NC) {
    const int s = j % NSLOT;
    float* lds0 = slots + s * SLOT;
    float* lds1 = lds0 + G::LDS_LEN;
    const TileRef tr = tile_ref<D, T, R, true, 1, 2, Src::F32>(a, first + j);
    float old_pi = 0.0f, old_pq = 0.0f;
    load_prev(a, tr, old_pi, old_pq);
    while (lds_ld(&ready[s]) != j) __builtin_amdgcn_s_sleep(1);
    asm volatile("" ::: "memory");
    if (tr.t == 0 || !interior<D, T, R, true, 1>(tr, n)) {
      edge_fill<D, T, R, true, 1, 2, Src::F32>(tr, lane, n, ns, lds0, lds1, tr.t == 0, strip0, strip1);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    }
    float acc0[R], acc1[R];
#pragma unroll
    for (int r = 0; r < R; ++r) acc0[r] = acc1[r] = 0.0f;
    if (a.ablate == 2) {  // timing only: no FIR arithmetic
      acc0[0] = lds0[lbase];
      acc1[0] = lds1[lbase];
    } else {
      scan_sgpr<D, T, R, 2, G>(lds0 + lbase, lds1 + lbase, h, acc0, acc1, a.ablate);
    }
    // every LDS read of the slot has returned: hand it back to the loader
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    if (lane == 0) lds_st(&freed[s], j);
    tile_epilogue<D, T, R, 1, 2, true, Src::F32>(a, tr, h, lane, lane, 0, n, nout, ns, acc0, acc1, old_pi, old_pq,
                                                 strip0, strip1);
  }
}

template <int D, int T, int R, bool NT>
hipError_t run_stream(const FirLaunch& a0, const float* h, hipStream_t st) {
  using G = typename Ring<D, T, R>::G;
  FirLaunch a = a0;
  const long long nout = a.n / D;
  a.tiles_per_stream = (int)((nout + G::ADV - 1) / G::ADV);
  const long long total = (long long)a.tiles_per_stream * a.nstreams;
  if (total <= 0 || total > 0x7fffffffLL) return hipErrorInvalidValue;
  static int ncu = 0;
  if (!ncu) {
    int dev = 0;
    (void)hipGetDevice(&dev);
    if (hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev) != hipSuccess || ncu <= 0) ncu = 256;
  }
  static const int ablate = [] {
    const char* e = std::getenv("SDR_ABLATE");
    return e ? std::atoi(e) : 0;
  }();
  a.ablate = ablate;
  const long long blocks = total < ncu ? total : ncu;
  hipLaunchKernelGGL((fir_stream<D, T, R, NT>), dim3((unsigned)blocks), dim3(64 * (Ring<D, T, R>::NC + Ring<D, T, R>::NL)), 0, st, a,
                     h);
  return hipGetLastError();
}

}  // namespace

// The loader/consumer engine covers the fused f32 front end at D = 10,
// T = 101 (the headline configuration).  Opt-in (SDR_FIR_STREAM=1): on
// MI355X it measured 5-7 % slower than fir_tile, whose
// register prefetch keeps more bytes in flight per CU than this LDS ring can.
// SDR_FIR_STREAM_NT=0 drops the non-temporal hint on the stream loads.
bool fir_stream_ok(int D, int ntaps, int ns, bool demod, int nch, Src src) {
  static const int env = [] {
    const char* e = std::getenv("SDR_FIR_STREAM");
    return e ? std::atoi(e) : 0;
  }();
  return env != 0 && D == 10 && ntaps == 101 && demod && nch == 2 && src == Src::F32 && ns >= ntaps - 1;
}

hipError_t launch_fir_stream(const FirLaunch& a, const float* h, hipStream_t st) {
  static const int nt = [] {
    const char* e = std::getenv("SDR_FIR_STREAM_NT");
    return e ? std::atoi(e) : 1;
  }();
  return nt ? run_stream<10, 101, 2, true>(a, h, st) : run_stream<10, 101, 2, false>(a, h, st);
}

}  // namespace sdr
