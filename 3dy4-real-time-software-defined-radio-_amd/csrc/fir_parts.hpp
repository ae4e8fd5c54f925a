// fir_parts.hpp -- device building blocks of the opt-in loader/consumer
// front end (fir_stream.hip: loader / consumer waves over an LDS-DMA ring).
// Internal to libsdrhip.so.  The default register-staged tile kernel
// (fir_tile.hip) keeps its own copy of the geometry: a shared-header
// refactor of it measured 2-8 % slower on cfg2 (same-box A/B)
// and was rolled back.
//
// Arithmetic contract (bit-exact with the compiled reference): see
// fir_tile.hip.  Header-only device code; a kernel TU includes it inside
// its own anonymous namespace.
#pragma once

#include <type_traits>

#include "sdr_common.hpp"

#pragma clang fp contract(off)

// Build switches for same-box A/B (scripts/build_ab_tree.sh):
// SDR_STAGE_PIN: pin the issue order of a tile's staging loads;
// SDR_EDGE_DRAIN: retire the edge loads at the end of edge_fill().
#ifndef SDR_STAGE_PIN
#define SDR_STAGE_PIN 1
#endif
#ifndef SDR_EDGE_DRAIN
#define SDR_EDGE_DRAIN 1
#endif

namespace sdr {
namespace {

template <int D, int T, int R, bool DEMOD, int NW>
struct Geom {
  static constexpr int NTH = 64 * NW;                               // threads per workgroup
  static_assert((D * R) % 4 == 0, "lane windows must start on 16-B boundaries");
  static constexpr int E = DEMOD ? R : 0;                          // overlap outputs per wave
  static constexpr int WADV = 64 * R - E;                          // new outputs per wave
  static constexpr int ADV = NW * WADV;                            // new outputs per tile
  static constexpr int HALO = (T - 1 + 3) / 4 * 4;                 // (T-1) rounded up to a float4
  static constexpr int SPAN = HALO + D * (R - 1) + 1;              // positions one lane reads
  static constexpr int NCHUNK = (SPAN + 3) / 4;                    // float4 chunks per lane window
  static constexpr int SPAN4 = 4 * NCHUNK;                         // tap row length
  // tap-row reuse: rows GR apart are offset by D*GR taps = SH whole chunks
  static constexpr int GQ = (D % 4 == 0) ? 1 : (D % 2 == 0) ? 2 : 4;
  static constexpr int GR = GQ < R ? GQ : R;                       // tap rows read from LDS per chunk
  static constexpr int SH = D * GR / 4;                            // chunk shift between reused rows
  static constexpr int LDS_LEN = D * ((NW - 1) * WADV + 63 * R) + SPAN4;  // floats per channel
  static constexpr int LDS4 = LDS_LEN / 4;
  static constexpr int FULL = LDS4 / NTH, REM = LDS4 % NTH;        // staging rows per thread
  // the block's last STRIP inputs per channel, staged by tile 0: the
  // prev_* recompute (D+T-1 inputs) and the new state (ns <= STRIP)
  static constexpr int STRIP = ((D + T - 1 > 128 ? D + T - 1 : 128) + 3) / 4 * 4;
  // vector loads one f32 stage_load issues per channel (ldg4_async)
  static constexpr int STAGE_LOADS = FULL + (REM ? 1 : 0);
  // LDS floats: channels, tap rows, two tail strips
  static constexpr int SMEM = 2 * LDS_LEN + R * SPAN4 + 2 * STRIP;
};

__device__ __forceinline__ float demod_one(float I, float Q, float ip, float qp) {
  // src/filter.cpp:88-98
  const float env = (float)((double)I * (double)I + (double)Q * (double)Q);
  if (env == 0.0f) return 0.0f;
  const float a = I * (Q - qp);
  const float b = Q * (I - ip);
  return (a - b) / env;
}

// Input sample p (>= 0) of channel c of one stream.
template <Src SRC>
__device__ __forceinline__ float in_at(const float* x, const uint8_t* iq, int c, long long p) {
  if constexpr (SRC == Src::F32) {
    return x[p];
  } else {
    return u8_to_f32(iq[2 * p + c]);
  }
}

// Element of the tile span at position p: x~[p], zero outside [-ns, n).
// A guarded load (exec-masked), no branches around it.
template <Src SRC>
__device__ __forceinline__ float edge_at(const float* x, const uint8_t* iq, int c, const float* st, int ns,
                                         long long n, long long p) {
  const bool in_state = p < 0;
  const bool valid = p >= -ns && p < n;
  float v = 0.0f;
  if constexpr (SRC == Src::F32) {
    const float* src = in_state ? st + (ns + p) : x + p;
    if (valid) v = *src;
  } else {
    if (valid) v = in_state ? st[ns + p] : u8_to_f32(iq[2 * p + c]);
  }
  return v;
}

// One 16-B streamed input load.  SDR_FIR_NT (build flag, A/B): non-temporal.
__device__ __forceinline__ float4 ldg4(const float* p) {
#if defined(SDR_FIR_NT) && SDR_FIR_NT
  typedef float f4 __attribute__((ext_vector_type(4)));
  const f4 v = __builtin_nontemporal_load(reinterpret_cast<const f4*>(p));
  return make_float4(v.x, v.y, v.z, v.w);
#else
  return *reinterpret_cast<const float4*>(p);
#endif
}

// Tile-prefetch loads with an explicit wait.  hipcc's waitcnt pass merges the
// vmcnt histories of the kernel's many paths (edge tiles, tile 0's state
// carry, conditional output stores) conservatively, and on the fused kernel
// that merge put a vmcnt(0) in front of every stage_store -- draining the
// prefetch of the next tile, i.e. no software pipelining.  These loads are
// inline asm, invisible to the pass; the kernel waits for them itself with
// vm_wait<N>(), N = the loads issued after the set being consumed (loads
// return in order, so stores and untracked ops in between only make the wait
// stricter).  SDR_FIR_NT=1 (build flag, A/B): non-temporal.
typedef float f4v __attribute__((ext_vector_type(4)));
// Off by default (SDR_FIR_ASYNC=1 build flag to A/B): with untracked loads
// the register allocator may hand a destination VGPR to another value
// before the load returns, and the late write then clobbers it (seen as an
// aperture violation on the GPU).  The default is the tracked ldg4().
__device__ __forceinline__ float4 ldg4_async(const float* p) {
#if !(defined(SDR_FIR_ASYNC) && SDR_FIR_ASYNC)
  return ldg4(p);
#else
  f4v v;
#if defined(SDR_FIR_NT) && SDR_FIR_NT
  asm volatile("global_load_dwordx4 %0, %1, off nt" : "=v"(v) : "v"(p) : "memory");
#else
  asm volatile("global_load_dwordx4 %0, %1, off" : "=v"(v) : "v"(p) : "memory");
#endif
  return make_float4(v.x, v.y, v.z, v.w);
#endif
}

// s_waitcnt vmcnt(N), then a register dependency on every staged value so
// nothing reads them before the wait.
template <int N, int K>
__device__ __forceinline__ void vm_wait(float4 (&v0)[K], float4 (&v1)[K]) {
#if !(defined(SDR_FIR_ASYNC) && SDR_FIR_ASYNC)
  return;  // tracked loads: hipcc places the waits
#endif
  asm volatile("s_waitcnt vmcnt(%0)" ::"n"(N) : "memory");
#pragma unroll
  for (int i = 0; i < K; ++i) {
    f4v a = {v0[i].x, v0[i].y, v0[i].z, v0[i].w};
    f4v b = {v1[i].x, v1[i].y, v1[i].z, v1[i].w};
    asm volatile("" : "+v"(a), "+v"(b));
    v0[i] = make_float4(a.x, a.y, a.z, a.w);
    v1[i] = make_float4(b.x, b.y, b.z, b.w);
  }
}

// Where one tile lives.
struct TileRef {
  int s;              // stream
  int t;              // tile within the stream
  long long m_start;  // first output the tile computes (includes the wave overlap)
  long long pb;       // stream position of LDS index 0
  const float* x0;
  const float* x1;
  const uint8_t* iq;
  float* st0;
  float* st1;
};

template <int D, int T, int R, bool DEMOD, int NW, int NCH, Src SRC>
__device__ __forceinline__ TileRef tile_ref(const FirLaunch& a, int lin) {
  using G = Geom<D, T, R, DEMOD, NW>;
  TileRef r;
  r.s = lin / a.tiles_per_stream;
  r.t = lin - r.s * a.tiles_per_stream;
  r.m_start = (long long)r.t * G::ADV - G::E;
  r.pb = (long long)D * r.m_start - G::HALO;
  r.st0 = a.state0 + (long long)r.s * a.ns;
  r.st1 = NCH == 2 ? a.state1 + (long long)r.s * a.ns : nullptr;
  r.x0 = r.x1 = nullptr;
  r.iq = nullptr;
  if constexpr (SRC == Src::F32) {
    r.x0 = a.x0 + (long long)r.s * a.x_stride;
    if (NCH == 2) r.x1 = a.x1 + (long long)r.s * a.x_stride;
  } else {
    r.iq = a.iq + (long long)r.s * a.x_stride;
  }
  return r;
}

// A tile no clamped chunk of which holds a sample a stored output reads:
// its span starts at p >= 0 and, when n is not a multiple of 4, ends before
// the chunk straddling n.  (Chunks past n only feed outputs >= n/D, which
// are never stored.)
template <int D, int T, int R, bool DEMOD, int NW>
__device__ __forceinline__ bool interior(const TileRef& tr, long long n) {
  const long long n4 = n & ~3LL;
  return tr.pb >= 0 && (n4 == n || tr.pb + Geom<D, T, R, DEMOD, NW>::LDS_LEN <= n4);
}

// Issue every global load of one tile span into registers (16-B f32 / 8-B
// u8 coalesced vectors).  Chunk addresses are clamped into the block, so an
// edge tile loads in-bounds but partly wrong data that edge_fill() then
// overwrites.  No wait: stage_store consumes the registers.
template <int D, int T, int R, bool DEMOD, int NW, int NCH, Src SRC, bool CLAMP>
__device__ __forceinline__ void stage_load_impl(const TileRef& tr, long long n, int tid,
                                           float4 (&v0)[Geom<D, T, R, DEMOD, NW>::FULL + 1],
                                           float4 (&v1)[Geom<D, T, R, DEMOD, NW>::FULL + 1]) {
  using G = Geom<D, T, R, DEMOD, NW>;
  auto load4 = [&](int i, float4& a0, float4& a1) {
    long long p = tr.pb + 4LL * i;
    if constexpr (CLAMP) {
      const long long pmax = (n & ~3LL) - 4;  // last whole aligned chunk
      p = p < 0 ? 0 : (p > pmax ? pmax : p);
    }
    if constexpr (SRC == Src::F32) {
      a0 = ldg4_async(tr.x0 + p);
      if (NCH == 2) a1 = ldg4_async(tr.x1 + p);
    } else {
      const uint2 b = *reinterpret_cast<const uint2*>(tr.iq + 2 * p);
      a0 = make_float4(u8_byte_to_f32<0>(b.x), u8_byte_to_f32<2>(b.x), u8_byte_to_f32<0>(b.y),
                       u8_byte_to_f32<2>(b.y));
      a1 = make_float4(u8_byte_to_f32<1>(b.x), u8_byte_to_f32<3>(b.x), u8_byte_to_f32<1>(b.y),
                       u8_byte_to_f32<3>(b.y));
    }
  };
  // Issue order pinned (sched_barrier): the loop's prologue and body then
  // issue a tile's loads in the same order, so hipcc's waitcnt pass merges
  // equal histories at the loop head and waits for exactly the tile being
  // staged, not for the prefetch behind it.
  if (SDR_STAGE_PIN) __builtin_amdgcn_sched_barrier(0);
#pragma unroll
  for (int it = 0; it < G::FULL; ++it) {
    load4(tid + it * G::NTH, v0[it], v1[it]);
    if (SDR_STAGE_PIN) __builtin_amdgcn_sched_barrier(0);
  }
  // ragged last row: clamp the index (a redundant load) so every register
  // is defined and the arrays stay in VGPRs
  if (G::REM) load4(tid < G::REM ? tid + G::FULL * G::NTH : G::FULL * G::NTH - 1, v0[G::FULL], v1[G::FULL]);
  if (SDR_STAGE_PIN) __builtin_amdgcn_sched_barrier(0);
}

// Clamped loads only where the span leaves the block (workgroup-uniform).
template <int D, int T, int R, bool DEMOD, int NW, int NCH, Src SRC>
__device__ __forceinline__ void stage_load(const TileRef& tr, long long n, int tid,
                                           float4 (&v0)[Geom<D, T, R, DEMOD, NW>::FULL + 1],
                                           float4 (&v1)[Geom<D, T, R, DEMOD, NW>::FULL + 1]) {
  if (tr.pb >= 0 && tr.pb + Geom<D, T, R, DEMOD, NW>::LDS_LEN <= n)
    stage_load_impl<D, T, R, DEMOD, NW, NCH, SRC, false>(tr, n, tid, v0, v1);
  else
    stage_load_impl<D, T, R, DEMOD, NW, NCH, SRC, true>(tr, n, tid, v0, v1);
}

// Edge tiles (a stream's first tile, and the one holding the chunk that
// straddles n when n % 4 != 0): after the clamped vector fill, rewrite the
// span elements a stored output reads whose chunk was clamped -- the old
// state before the block, [pb, 0), and the true samples of the straddling
// chunk, [n & ~3, n).  With `strip`, also stage the block's last STRIP
// inputs (old state where p < 0) for tile 0's state carry.  The loads are
// issued in batches of four per thread before any LDS write, so an edge tile
// costs about one memory latency, not one per element.
template <int D, int T, int R, bool DEMOD, int NW, int NCH, Src SRC>
__device__ __forceinline__ void edge_fill(const TileRef& tr, int tid, long long n, int ns, float* lds0, float* lds1,
                                          bool strip, float* strip0, float* strip1) {
  using G = Geom<D, T, R, DEMOD, NW>;
  const long long n4 = n & ~3LL;
  const int lo_end = tr.pb < 0 ? (int)(-tr.pb < G::LDS_LEN ? -tr.pb : G::LDS_LEN) : 0;
  auto clampi = [](long long v, int lo, int hi) { return (int)(v < lo ? lo : (v > hi ? hi : v)); };
  const int hi_beg = clampi(n4 - tr.pb, lo_end, G::LDS_LEN);
  const int hi_end = clampi(n - tr.pb, hi_beg, G::LDS_LEN);
  const int nfix = lo_end + (hi_end - hi_beg);
  const int ntot = nfix + (strip ? G::STRIP : 0);
  for (int e0 = 0; e0 < ntot; e0 += 4 * G::NTH) {
    float v0[4], v1[4];
    float* d0[4];
    float* d1[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * G::NTH + tid;
      long long p;
      if (e < lo_end) {
        p = tr.pb + e;
        d0[u] = lds0 + e;
        d1[u] = lds1 + e;
      } else if (e < nfix) {
        const int i = hi_beg + (e - lo_end);
        p = tr.pb + i;
        d0[u] = lds0 + i;
        d1[u] = lds1 + i;
      } else {
        const int j = e - nfix;
        p = n - G::STRIP + j;
        d0[u] = strip0 + j;
        d1[u] = strip1 + j;
      }
      v0[u] = 0.0f;
      v1[u] = 0.0f;
      if (e < ntot) {
        v0[u] = edge_at<SRC>(tr.x0, tr.iq, 0, tr.st0, ns, n, p);
        if (NCH == 2) v1[u] = edge_at<SRC>(tr.x1, tr.iq, 1, tr.st1, ns, n, p);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      if (e0 + u * G::NTH + tid < ntot) {
        *d0[u] = v0[u];
        if (NCH == 2) *d1[u] = v1[u];
      }
    }
  }
  // Retire every edge load here.  Without this wait hipcc's waitcnt pass
  // merges the edge and interior paths conservatively and then drains the
  // whole vector-memory queue (vmcnt(0)) at the start of every tile's scan
  // -- including the next tiles' prefetch, which defeats the pipelining.
  if (SDR_EDGE_DRAIN) __builtin_amdgcn_s_waitcnt(0);
}

template <int D, int T, int R, bool DEMOD, int NW, int NCH>
__device__ __forceinline__ void stage_store(float* lds0, float* lds1, int tid,
                                            const float4 (&v0)[Geom<D, T, R, DEMOD, NW>::FULL + 1],
                                            const float4 (&v1)[Geom<D, T, R, DEMOD, NW>::FULL + 1]) {
  using G = Geom<D, T, R, DEMOD, NW>;
#pragma unroll
  for (int it = 0; it < G::FULL; ++it) {
    const int i = tid + it * G::NTH;
    *reinterpret_cast<float4*>(lds0 + 4 * i) = v0[it];
    if (NCH == 2) *reinterpret_cast<float4*>(lds1 + 4 * i) = v1[it];
  }
  if (G::REM && tid < G::REM) {
    const int i = tid + G::FULL * G::NTH;
    *reinterpret_cast<float4*>(lds0 + 4 * i) = v0[G::FULL];
    if (NCH == 2) *reinterpret_cast<float4*>(lds1 + 4 * i) = v1[G::FULL];
  }
}

// f(integral_constant<int, B>), f(<B+1>), ..., f(<E-1>): a fully unrolled
// loop whose index is a constant expression in the body.
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// The stream's carried prev_I / prev_Q (fmDemodArctan's state), read by a
// stream's tile 0 before its workgroup rewrites them.  Scalar loads: a
// vector load here would be a vmcnt event whose (conditional) destination
// makes hipcc's waitcnt pass drain the whole vector-memory queue -- the next
// tiles' prefetch included -- at the discriminator and at the next tile.
template <class TR>
__device__ __forceinline__ void load_prev(const FirLaunch& a, const TR& tr, float& pi, float& pq) {
  if (tr.t == 0) {  // workgroup-uniform
    using cf = const __attribute__((address_space(4))) float*;
    const int s = __builtin_amdgcn_readfirstlane(tr.s);
    pi = ((cf)a.prev0)[s];
    pq = ((cf)a.prev1)[s];
  }
}

// The FIR scan with taps as SGPR operands of the multiplies (no LDS tap
// traffic): this lane's R outputs of NCH channels, from its window w0/w1
// (LDS; window position 0 = output r's input HALO + D*r - k).
// FMA: the fused multiply-add arithmetic mode (SDR_ARITH_FMA) -- the same
// taps in the same order, one rounding per tap instead of two (not the
// reference's bits; within the stated fp32 tolerance).
template <int D, int T, int R, int NCH, class G, bool FMA = false>
__device__ __forceinline__ void scan_sgpr(const float* w0, const float* w1, const float* h, float (&acc0)[R],
                                          float (&acc1)[R], int ablate) {
  // Taps as SGPR operands of the multiplies: no LDS tap traffic.  All
  // T taps do not fit the SGPR file beside the addressing, so the
  // window is walked in NPASS passes over consecutive tap ranges
  // [k0, k1), each loading its taps once (scalar loads from the
  // constant address space, one wait) -- every output still visits
  // k = 0..T-1 in order, the passes only split its chain.
  constexpr int NPASS = 3, KP = (T + NPASS - 1) / NPASS;
  using hconst = const __attribute__((address_space(4))) float*;
  const hconst hc = (hconst)h;
  float hs[KP];
  static_for<0, NPASS>([&](auto pi) {
    constexpr int k0 = decltype(pi)::value * KP;
    constexpr int k1 = k0 + KP < T ? k0 + KP : T;
    // ablate 4 (timing only): one pass of three -- how much a cheaper scan buys
    if (ablate == 4 && k0 > 0) return;
#pragma unroll
    for (int i = 0; i < k1 - k0; ++i) hs[i] = hc[k0 + i];
#pragma unroll
    for (int i = 0; i < k1 - k0; ++i) asm volatile("" : "+s"(hs[i]));
    // window positions w = HALO + D r - k this pass touches
    constexpr int wlo = G::HALO - (k1 - 1) > 0 ? G::HALO - (k1 - 1) : 0;
    constexpr int whi = G::HALO + D * (R - 1) - k0;
    constexpr int clo = wlo / 4, chi = whi / 4;
    float4 q0 = *reinterpret_cast<const float4*>(w0 + 4 * chi);
    float4 q1 = q0;
    if (NCH == 2) q1 = *reinterpret_cast<const float4*>(w1 + 4 * chi);
    static_for<0, chi - clo + 1>([&](auto ci) {
      constexpr int c = chi - decltype(ci)::value;
      float4 n0 = q0, n1 = q1;
      if constexpr (c > clo) {
        n0 = *reinterpret_cast<const float4*>(w0 + 4 * (c - 1));
        if (NCH == 2) n1 = *reinterpret_cast<const float4*>(w1 + 4 * (c - 1));
      }
      const float e0[4] = {q0.x, q0.y, q0.z, q0.w};
      const float e1[4] = {q1.x, q1.y, q1.z, q1.w};
      static_for<0, 4>([&](auto ji) {
        constexpr int j = 3 - decltype(ji)::value;
        static_for<0, R>([&](auto ri) {
          constexpr int r = decltype(ri)::value;
          constexpr int k = G::HALO + D * r - (4 * c + j);
          if constexpr (k >= k0 && k < k1) {
            if constexpr (FMA) {
              acc0[r] = __builtin_fmaf(hs[k - k0], e0[j], acc0[r]);
              if (NCH == 2) acc1[r] = __builtin_fmaf(hs[k - k0], e1[j], acc1[r]);
            } else {
              acc0[r] = acc0[r] + hs[k - k0] * e0[j];
              if (NCH == 2) acc1[r] = acc1[r] + hs[k - k0] * e1[j];
            }
          }
        });
      });
      q0 = n0;
      q1 = n1;
#pragma unroll
      for (int r = 0; r < R; ++r) asm volatile("" : "+v"(acc0[r]), "+v"(acc1[r]));
      __builtin_amdgcn_sched_barrier(0);
    });
  });
}

// After the scan: the discriminator (fused launches) and the output stores
// of this lane's R outputs, then -- tile 0 of a stream only -- the carried
// prev_* and state.  old_pi/old_pq: the stream's prev_* read before any
// rewrite (tile 0, tid 1); strip0/1: the block's last STRIP inputs (tile 0).
// NTH: the threads sharing the state stores.
template <int D, int T, int R, int NW, int NCH, bool DEMOD, Src SRC, bool FMA = false>
__device__ __forceinline__ void tile_epilogue(const FirLaunch& a, const TileRef& tr, const float* h, int tid, int lane,
                                              int wave, long long n, long long nout, int ns, const float (&acc0)[R],
                                              const float (&acc1)[R], float old_pi, float old_pq, const float* strip0,
                                              const float* strip1) {
  using G = Geom<D, T, R, DEMOD, NW>;
  constexpr int NTH = G::NTH;
  const long long m0 = tr.m_start + (long long)wave * G::WADV + (long long)R * lane;  // this lane's first output
  if constexpr (DEMOD) {
    // ---- 3. discriminator in registers.  The decimated sample before
    // output r=0 is lane-1's last output (a wave shuffle); lane 0's
    // outputs are the wave's overlap and are not stored; at the start of
    // the stream (tile 0, wave 0, lane 1 -> output 0) it is the carried prev_*.
    float pI = __shfl_up(acc0[R - 1], 1, 64);
    float pQ = __shfl_up(acc1[R - 1], 1, 64);
    if (tr.t == 0 && tid == 1) {
      pI = old_pi;
      pQ = old_pq;
    }
    float d[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float ip = r ? acc0[r - 1] : pI;
      const float qp = r ? acc1[r - 1] : pQ;
      d[r] = demod_one(acc0[r], acc1[r], ip, qp);
    }
    float* o = a.out + (long long)tr.s * a.out_stride;
    // vector stores when the row keeps R-float groups aligned (uniform)
    const bool vec = ((reinterpret_cast<uintptr_t>(o) + 4ull * (unsigned long long)tr.m_start) % (4u * R)) == 0;
    // ablate 3 (timing only): no output stores unless the result is a
    // value it never is, so the scan still runs
    if (lane >= 1 && (a.ablate != 3 || d[0] == 12345.0f)) {
      if (vec && m0 + R <= nout) {
        if constexpr (R == 2) {
          *reinterpret_cast<float2*>(o + m0) = make_float2(d[0], d[1]);
        } else if constexpr (R == 4) {
          *reinterpret_cast<float4*>(o + m0) = make_float4(d[0], d[1], d[2], d[3]);
        } else {
#pragma unroll
          for (int r = 0; r < R; ++r) o[m0 + r] = d[r];
        }
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r)
          if (m0 + r < nout) o[m0 + r] = d[r];
      }
    }
  } else {
    float* o = a.y0 + (long long)tr.s * a.y_stride;
    const bool vec = ((reinterpret_cast<uintptr_t>(o) + 4ull * (unsigned long long)tr.m_start) % (4u * R)) == 0;
    if (vec && m0 + R <= nout) {
      if constexpr (R == 4) {
        *reinterpret_cast<float4*>(o + m0) = make_float4(acc0[0], acc0[1], acc0[2], acc0[3]);
      } else if constexpr (R == 2) {
        *reinterpret_cast<float2*>(o + m0) = make_float2(acc0[0], acc0[1]);
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) o[m0 + r] = acc0[r];
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (m0 + r < nout) o[m0 + r] = acc0[r];
    }
  }

  // ---- 4. state carry (tile 0 only; every read of the old values
  // happened before the barriers above)
  if (tr.t == 0) {
    if constexpr (DEMOD) {
      // prev_* <- last decimated I/Q of the block (src/filter.cpp:100-101),
      // recomputed in the reference's order from the staged strip:
      // input D*(nout-1) - k = n - D - k sits at strip index STRIP - D - k
      if (tid == 0) {
        float yi = 0.0f, yq = 0.0f;
        for (int k = 0; k < T; ++k) {
          const float hk = h[k];
          if constexpr (FMA) {  // the arithmetic of the scan that produced the outputs
            yi = __builtin_fmaf(hk, strip0[G::STRIP - D - k], yi);
            yq = __builtin_fmaf(hk, strip1[G::STRIP - D - k], yq);
          } else {
            yi = yi + hk * strip0[G::STRIP - D - k];
            yq = yq + hk * strip1[G::STRIP - D - k];
          }
        }
        a.prev0[tr.s] = yi;
        a.prev1[tr.s] = yq;
      }
    }
    // state <- last ns input samples (src/filter.cpp:139)
    if (ns <= G::STRIP) {
      for (int j = tid; j < ns; j += NTH) {
        tr.st0[j] = strip0[G::STRIP - ns + j];
        if (NCH == 2) tr.st1[j] = strip1[G::STRIP - ns + j];
      }
    } else {
      for (int j = tid; j < ns; j += NTH) {
        const long long p = n - ns + j;
        tr.st0[j] = in_at<SRC>(tr.x0, tr.iq, 0, p);
        if (NCH == 2) tr.st1[j] = in_at<SRC>(tr.x1, tr.iq, 1, p);
      }
    }
  }
}

}  // namespace
}  // namespace sdr
