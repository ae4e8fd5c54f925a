// fir_tile.hip -- gfx950 kernels for the reference's FIR / FIR+decimate /
// fused front end (src/filter.cpp:66-83, 85-102, 123-140, sequenced as in
// src/project.cpp:86-90).
//
// Arithmetic contract (bit-exact with the compiled reference):
//   y[m] = (...((0 + h[0]*x~[mD]) + h[1]*x~[mD-1]) + ...) + h[T-1]*x~[mD-T+1]
// with every product and sum rounded separately (no FMA contraction), taps
// visited in ascending k; x~[p] = x[p] for p >= 0, the saved tail state[ns+p]
// before the block.  The discriminator keeps the reference's double-precision
// envelope (std::pow(float,int) promotes, src/filter.cpp:88) and a correctly
// rounded fp32 divide.
//
// Tile kernel structure (fir_tile):
//   * a tile = NW waves x 64 lanes x R consecutive output samples of one
//     stream; its input span (D*64*NW*R samples plus a (T-1)-sample halo --
//     overlap-save) is staged in LDS with 16-B coalesced loads.  The halo of
//     a stream's first tile is the carried `state`;
//   * every lane slides down its own D*R-aligned window of the tile in 16-B
//     ds_read_b128 chunks (lane stride D*R dwords, 20 for D=10 R=2:
//     conflict-free) and keeps all R outputs of I and Q in registers; the
//     taps are SGPR operands of the multiplies, loaded once per pass over a
//     third of the taps (an earlier LDS tap-row mode for D = 1 lost its A/B:
//     31.4 vs 37.8 us per 1,024 x 5,120 block, scripts/d1bench.py);
//   * fused launches apply the discriminator in registers and write only the
//     demodulated stream: decimated I/Q never touch HBM.  Lane 0 of each wave
//     re-derives the R outputs before its span (E = R) so waves never wait on
//     each other;
//   * persistent workgroups walk a contiguous run of tiles; the loads of
//     tile i+1 are issued into registers before tile i is computed, so each
//     wave always has HBM reads in flight (software pipelining);
//   * state carry: only the first tile of a stream reads `state`/`prev`;
//     the workgroup that owns it rewrites them after its reads -- one kernel.
#include <algorithm>
#include <cstdio>
#include <cstdlib>
#include <type_traits>

#include "sdr_common.hpp"

#pragma clang fp contract(off)

// Build switches (same-box A/B with scripts/build_ab_tree.sh):
// SDR_FIR_NT / SDR_FIR_NT_U8: streamed span loads with the non-temporal
// hint (read once from HBM; the neighbour's halo re-read still hits L2).
// Measured (warm, same box): f32 -1..5 %, u8 wire +6 % -> f32 only.
#ifndef SDR_FIR_NT
#define SDR_FIR_NT 1
#endif
// SDR_NPASS: SGPR tap passes of the scan (3: 34 taps per pass fit the SGPR
// file beside the addressing; fewer passes re-read fewer window chunks).
#ifndef SDR_NPASS
#define SDR_NPASS 3
#endif
// SDR_FIR_DEFER: a tile's output stores wait until the next tile is staged
// SDR_SCAN_PF: chunks of a lane's window read from LDS ahead of the chunk
// being multiplied (its lgkmcnt wait covers the rest)
#ifndef SDR_SCAN_PF
#define SDR_SCAN_PF 1
#endif
#ifndef SDR_FIR_DEFER
#define SDR_FIR_DEFER 1
#endif
// SDR_OUT_NT: non-temporal hint on the demod output stores of the f32 path
// (warm same-box A/B: f32 -1..2 %, u8 neutral -> f32 only)
#ifndef SDR_OUT_NT
#define SDR_OUT_NT 1
#endif
#ifndef SDR_FIR_NT_U8
#define SDR_FIR_NT_U8 0
#endif
// SDR_FIR_BUF: the u8 wire path's interior span loads as raw buffer loads off
// a per-tile SGPR descriptor (one 32-bit lane offset, SGPR row offsets) instead
// of 64-bit per-load VALU addresses: cfg2u8 0.0764-0.0771 vs 0.0781-0.0799 ms,
// mono0 0.0836-0.0841 vs 0.0850-0.0857 (same box, profiles/r05c/ab_buf.txt).
// The f32 path measured 1.5 % slower that way (0.0978-0.1001 vs 0.0963-0.0977
// ms on cfg2) and keeps its global loads.
#ifndef SDR_FIR_BUF
#define SDR_FIR_BUF 1
#endif
// (Round 5: the wire-byte unpack with packed FMAs, v_pk_fma_f32 for two
// samples, measured neutral on cfg2u8 and -1.5 % on mono0; code at 821f6db.)
// SDR_SC_T0PRE: fir_tile_sc's tile 0 issues its extra loads (carried state,
// block tail, side copy) with the span's (one memory latency, not three);
// f32 front end: cfg2 0.0954-0.0959 vs 0.0959-0.0963 ms (profiles/r05u/)
#ifndef SDR_SC_T0PRE
#define SDR_SC_T0PRE 1
#endif
// SDR_SCAN_VCONST (timing builds only, wrong outputs): fir_tile_sc's scan
// with a VGPR in place of the SGPR taps
#ifndef SDR_SCAN_VCONST
#define SDR_SCAN_VCONST 0
#endif

namespace sdr {
namespace {
typedef float nf4 __attribute__((ext_vector_type(4)));
__device__ __forceinline__ nf4 ldg_stream_n(const float4* p) {
#if SDR_FIR_NT
  return __builtin_nontemporal_load(reinterpret_cast<const nf4*>(p));
#else
  return *reinterpret_cast<const nf4*>(p);
#endif
}
__device__ __forceinline__ void set_chunk(float4& d, const nf4& v) { d = make_float4(v.x, v.y, v.z, v.w); }
__device__ __forceinline__ uint2 ldg_stream(const uint2* p) {
#if SDR_FIR_NT_U8
  typedef unsigned u2 __attribute__((ext_vector_type(2)));
  const u2 v = __builtin_nontemporal_load(reinterpret_cast<const u2*>(p));
  return make_uint2(v.x, v.y);
#else
  return *p;
#endif
}
}  // namespace
}  // namespace sdr

#ifdef SDR_FIR_TRACE
// Diagnostic builds only (scripts/build_ab_tree.sh trace -DSDR_FIR_TRACE):
// per-workgroup timeline of fir_tile's first tile, read back by
// tools/fir_trace.py through sdr_debug_fir_trace().  Never in the product
// library.  Per workgroup, 8 words: HW_ID | XCC_ID << 32, s_memrealtime at
// entry, then s_memtime sums over the workgroup's tiles of: the wait for a
// tile's loads (top of the tile -> landed), staging, scan, epilogue; the
// tile count; s_memrealtime at the end; s_memtime at entry and at the end
// (their ratio to the realtime span is the shader clock).
constexpr int kTraceWG = 1 << 17;
constexpr int kTraceW = 10;  // words per record
__device__ unsigned long long g_fir_trace[kTraceWG * kTraceW];
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
  static constexpr int SPAN4 = 4 * NCHUNK;                         // a lane window, whole chunks
  static constexpr int LDS_LEN = D * ((NW - 1) * WADV + 63 * R) + SPAN4;  // floats per channel
  static constexpr int LDS4 = LDS_LEN / 4;
  static constexpr int FULL = LDS4 / NTH, REM = LDS4 % NTH;        // staging rows per thread
  // the block's last STRIP inputs per channel, staged by tile 0: the
  // prev_* recompute (D+T-1 inputs) and the new state (ns <= STRIP)
  static constexpr int STRIP = ((D + T - 1 > 128 ? D + T - 1 : 128) + 3) / 4 * 4;
  // LDS floats: the channels (the two tail strips reuse them)
  // (the strips reuse the channel buffers after tile 0's scan: LDS per
  // wave sets the occupancy, 13 -> 14 one-wave workgroups per CU at D = 10)
  static_assert(STRIP <= LDS_LEN, "strip staged into the channel buffers");
  static constexpr int SMEM = 2 * LDS_LEN;
};

__device__ __forceinline__ float demod_one(float I, float Q, float ip, float qp) {
  // src/filter.cpp:88-98
  const float env = (float)((double)I * (double)I + (double)Q * (double)Q);
  if (env == 0.0f) return 0.0f;
  const float a = I * (Q - qp);
  const float b = Q * (I - ip);
  return (a - b) / env;
}

// FirLaunch's side copy for stream s, by the stream's tile-0 workgroup
// (threads tid of nth, side_n <= kSideMax * nth, checked by the C API): the
// loads go out in the same batch as that tile's state-carry loads and the
// stores after their s_waitcnt(0) -- one memory latency for both, not two.
constexpr int kSideMax = 4;
__device__ __forceinline__ void side_load(const FirLaunch& a, int s, int tid, int nth, float (&v)[kSideMax]) {
  if (a.side_n <= 0) return;  // launch-uniform
  const float* src = a.side_src + (long long)s * a.side_src_stride;
  // unguarded loads at clamped indices (side_store skips the extra lanes): an
  // exec-masked load's merge would make the compiler wait for it right here
#pragma unroll
  for (int u = 0; u < kSideMax; ++u) v[u] = src[min(tid + u * nth, a.side_n - 1)];
}
__device__ __forceinline__ void side_store(const FirLaunch& a, int s, int tid, int nth, const float (&v)[kSideMax]) {
  float* dst = a.side_dst + (long long)s * a.side_dst_stride;
#pragma unroll
  for (int u = 0; u < kSideMax; ++u) {
    const int j = tid + u * nth;
    if (j < a.side_n) dst[j] = v[u];
  }
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

// Where one tile lives.
struct TileRef {
  int s;              // stream
  int t;              // tile within the stream
  long long m_start;  // first output the tile computes (t*ADV; tiles t >= 1 recompute their first E)
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
  // Tile t computes outputs [t*ADV, t*ADV + NW*64*R).  Its first E outputs
  // (lane 0 of each wave) are the previous wave's last E, recomputed so no
  // wave waits for another; tile 0 has no predecessor: its lane 0 outputs
  // are the stream's first and are stored, with the carried prev_*.  So
  // tiles_per_stream = ceil((nout - E) / ADV): at cfg2 (6,554 outputs,
  // ADV 126, E 2) exactly 52 tiles, none partial.
  r.m_start = (long long)r.t * G::ADV;
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
template <int D, int T, int R, bool DEMOD, int NW, int NCH, Src SRC, bool CLAMP, class V>
__device__ __forceinline__ void stage_load_impl(const TileRef& tr, long long n, int tid,
                                           V (&v0)[Geom<D, T, R, DEMOD, NW>::FULL + 1],
                                           V (&v1)[Geom<D, T, R, DEMOD, NW>::FULL + 1]) {
  using G = Geom<D, T, R, DEMOD, NW>;
  auto load4 = [&](int i, V& a0, V& a1) {
    long long p = tr.pb + 4LL * i;
    if constexpr (CLAMP) {
      const long long pmax = (n & ~3LL) - 4;  // last whole aligned chunk
      p = p < 0 ? 0 : (p > pmax ? pmax : p);
    }
    if constexpr (SRC == Src::F32) {
      set_chunk(a0, ldg_stream_n(reinterpret_cast<const float4*>(tr.x0 + p)));
      if (NCH == 2) set_chunk(a1, ldg_stream_n(reinterpret_cast<const float4*>(tr.x1 + p)));
    } else {
      const uint2 b = ldg_stream(reinterpret_cast<const uint2*>(tr.iq + 2 * p));
      // the raw wire bytes stay in the prefetch registers (2 VGPRs per
      // chunk); stage_store unpacks them.  Unpacking here would consume the
      // load right after issuing it -- an immediate vmcnt wait, i.e. no
      // prefetch at all.
      a0.x = __uint_as_float(b.x);
      a0.y = __uint_as_float(b.y);
    }
  };
#if SDR_FIR_BUF
  if constexpr (!CLAMP && SRC == Src::U8) {
    // interior span: raw buffer loads off a per-tile SGPR descriptor, a 32-bit
    // lane offset and an SGPR row offset -- no 64-bit VALU address per load
    constexpr int kAux = SRC == Src::F32 ? (SDR_FIR_NT ? 2 : 0) : (SDR_FIR_NT_U8 ? 2 : 0);  // 2: nt
    constexpr int EB = SRC == Src::F32 ? 16 : 8;  // bytes per chunk
    auto rsrc = [&](const void* base) __attribute__((always_inline)) {
      return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, G::LDS4 * EB, 0x00020000);
    };
    // row `row` (wave-uniform: the SGPR offset), lane chunk `col`
    auto ld = [&](int row, int col, V& a0, V& a1, auto r0, auto r1) __attribute__((always_inline)) {
      const int vo = EB * col, so = EB * G::NTH * row;
      if constexpr (SRC == Src::F32) {
        typedef float f4v __attribute__((ext_vector_type(4)));
        const f4v x = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r0, vo, so, kAux));
        a0 = make_float4(x.x, x.y, x.z, x.w);
        if (NCH == 2) {
          const f4v y = __builtin_bit_cast(f4v, __builtin_amdgcn_raw_buffer_load_b128(r1, vo, so, kAux));
          a1 = make_float4(y.x, y.y, y.z, y.w);
        }
      } else {
        typedef unsigned u2v __attribute__((ext_vector_type(2)));
        const u2v b = __builtin_amdgcn_raw_buffer_load_b64(r0, vo, so, kAux);
        a0.x = __uint_as_float(b.x);
        a0.y = __uint_as_float(b.y);
      }
    };
    if constexpr (SRC == Src::F32) {
      const auto r0 = rsrc(tr.x0 + tr.pb);
      const auto r1 = rsrc(NCH == 2 ? tr.x1 + tr.pb : tr.x0 + tr.pb);
#pragma unroll
      for (int it = 0; it < G::FULL; ++it) ld(it, tid, v0[it], v1[it], r0, r1);
      // ragged last row: lanes past REM re-load its last chunk (the row offset
      // stays uniform -- a lane-dependent one is a readfirstlane loop)
      if (G::REM) ld(G::FULL, tid < G::REM ? tid : G::REM - 1, v0[G::FULL], v1[G::FULL], r0, r1);
    } else {
      const auto r0 = rsrc(tr.iq + 2 * tr.pb);
#pragma unroll
      for (int it = 0; it < G::FULL; ++it) ld(it, tid, v0[it], v1[it], r0, r0);
      if (G::REM) ld(G::FULL, tid < G::REM ? tid : G::REM - 1, v0[G::FULL], v1[G::FULL], r0, r0);
    }
    return;
  }
#endif
#pragma unroll
  for (int it = 0; it < G::FULL; ++it) load4(tid + it * G::NTH, v0[it], v1[it]);
  // ragged last row: clamp the index (a redundant load) so every register
  // is defined and the arrays stay in VGPRs
  if (G::REM) load4(tid < G::REM ? tid + G::FULL * G::NTH : G::FULL * G::NTH - 1, v0[G::FULL], v1[G::FULL]);
}

// Clamped loads only where the span leaves the block (workgroup-uniform).
template <int D, int T, int R, bool DEMOD, int NW, int NCH, Src SRC, class V>
__device__ __forceinline__ void stage_load(const TileRef& tr, long long n, int tid,
                                           V (&v0)[Geom<D, T, R, DEMOD, NW>::FULL + 1],
                                           V (&v1)[Geom<D, T, R, DEMOD, NW>::FULL + 1]) {
  if (tr.pb >= 0 && tr.pb + Geom<D, T, R, DEMOD, NW>::LDS_LEN <= n)
    stage_load_impl<D, T, R, DEMOD, NW, NCH, SRC, false>(tr, n, tid, v0, v1);
  else
    stage_load_impl<D, T, R, DEMOD, NW, NCH, SRC, true>(tr, n, tid, v0, v1);
}

// Edge tiles (a stream's first tile, and the one holding the chunk that
// straddles n when n % 4 != 0): after the clamped vector fill, rewrite the
// span elements a stored output reads whose chunk was clamped -- the old
// state before the block, [pb, 0), and the true samples of the straddling
// chunk, [n & ~3, n).  put(i, v0, v1) stores span element i of the two
// channels in the kernel's LDS layout.  The loads are issued in batches of
// four per thread before any LDS write, so an edge tile costs about one
// memory latency, not one per element.
template <int D, int T, int R, bool DEMOD, int NW, int NCH, Src SRC, class Put>
__device__ __forceinline__ void edge_fill(const TileRef& tr, int tid, long long n, int ns, Put&& put, int c0 = 0) {
  using G = Geom<D, T, R, DEMOD, NW>;
  const long long n4 = n & ~3LL;
  const int lo_end = tr.pb < 0 ? (int)(-tr.pb < G::LDS_LEN ? -tr.pb : G::LDS_LEN) : 0;
  auto clampi = [](long long v, int lo, int hi) { return (int)(v < lo ? lo : (v > hi ? hi : v)); };
  const int hi_beg = clampi(n4 - tr.pb, lo_end, G::LDS_LEN);
  const int hi_end = clampi(n - tr.pb, hi_beg, G::LDS_LEN);
  const int nfix = lo_end + (hi_end - hi_beg);
  for (int e0 = 0; e0 < nfix; e0 += 4 * G::NTH) {
    float v0[4], v1[4];
    int idx[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int e = e0 + u * G::NTH + tid;
      idx[u] = e < lo_end ? e : hi_beg + (e - lo_end);
      const long long p = tr.pb + idx[u];
      v0[u] = 0.0f;
      v1[u] = 0.0f;
      if (e < nfix) {
        v0[u] = edge_at<SRC>(tr.x0, tr.iq, c0, tr.st0, ns, n, p);
        if (NCH == 2) v1[u] = edge_at<SRC>(tr.x1, tr.iq, 1, tr.st1, ns, n, p);
      }
    }
#pragma unroll
    for (int u = 0; u < 4; ++u)
      if (e0 + u * G::NTH + tid < nfix) put(idx[u], v0[u], v1[u]);
  }
  // Retire the edge loads inside the (rare) edge path.  Left pending, they
  // make hipcc's waitcnt pass merge the edge and interior paths
  // conservatively and drain the whole vector-memory queue (vmcnt(0)) at
  // every tile's scan -- the next tiles' prefetch included.
  __builtin_amdgcn_s_waitcnt(0);
}

template <int D, int T, int R, bool DEMOD, int NW, int NCH, Src SRC>
__device__ __forceinline__ void stage_store(float* lds0, float* lds1, int tid,
                                            const float4 (&v0)[Geom<D, T, R, DEMOD, NW>::FULL + 1],
                                            const float4 (&v1)[Geom<D, T, R, DEMOD, NW>::FULL + 1]) {
  using G = Geom<D, T, R, DEMOD, NW>;
  // u8: v0[i].x/.y hold 8 raw interleaved wire bytes (I0 Q0 I1 Q1 | I2 Q2 I3 Q3)
  auto put = [&](int i, const float4& a0, const float4& a1) {
    if constexpr (SRC == Src::U8) {
      const uint32_t bx = __float_as_uint(a0.x), by = __float_as_uint(a0.y);
      *reinterpret_cast<float4*>(lds0 + 4 * i) = make_float4(u8_byte_to_f32<0>(bx), u8_byte_to_f32<2>(bx),
                                                             u8_byte_to_f32<0>(by), u8_byte_to_f32<2>(by));
      *reinterpret_cast<float4*>(lds1 + 4 * i) = make_float4(u8_byte_to_f32<1>(bx), u8_byte_to_f32<3>(bx),
                                                             u8_byte_to_f32<1>(by), u8_byte_to_f32<3>(by));
    } else {
      *reinterpret_cast<float4*>(lds0 + 4 * i) = a0;
      if (NCH == 2) *reinterpret_cast<float4*>(lds1 + 4 * i) = a1;
    }
  };
#pragma unroll
  for (int it = 0; it < G::FULL; ++it) put(tid + it * G::NTH, v0[it], v1[it]);
  if (G::REM && tid < G::REM) put(tid + G::FULL * G::NTH, v0[G::FULL], v1[G::FULL]);
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

// TM = where the taps live: 1 SGPRs (NPASS passes), the only mode built.
// The loads of tile i+1 are issued into registers before tile i is computed
// (prefetch depth 1).
// FMA = the fused multiply-add arithmetic mode (SDR_ARITH_FMA, SGPR taps
// only): same taps, same order, one rounding per tap instead of two -- not
// the reference's bits, within the fp32 tolerance of DESIGN.md 2.
// fir_tile: one workgroup of NW waves per tile, the tiles walked statically
// (walk 0: a contiguous run per workgroup; walk 1: XCD slabs, one tile per
// workgroup in practice -- the dispatcher interleaves them).  The fused f32
// front end's kernel: fir_tile_grp's persistent groups lost 13 % on cfg2
// (DESIGN.md 5.2).
template <int D, int T, int R, int NW, int NCH, bool DEMOD, Src SRC, int TM, bool FMA = false>
__global__ __launch_bounds__(64 * NW) void fir_tile(FirLaunch a, const float* __restrict__ h) {
  using G = Geom<D, T, R, DEMOD, NW>;
  constexpr int NTH = G::NTH;
  static_assert(NCH == 2 || !DEMOD, "the discriminator needs I and Q");
  static_assert(SRC == Src::F32 || NCH == 2, "u8 wire format carries I and Q");
  static_assert(TM == 1, "taps as SGPR operands");

  extern __shared__ __attribute__((aligned(16))) float smem[];
  float* lds0 = smem;
  float* lds1 = smem + G::LDS_LEN;
  float* strip0 = lds0;                 // the block's last inputs (tile 0, after its scan)
  float* strip1 = lds1;

  const int tid = threadIdx.x;
  const int lane = tid & 63, wave = tid >> 6;
  const long long n = a.n;
  const long long nout = n / D;
  const int ns = a.ns;
  const int total = a.nstreams * a.tiles_per_stream;
  // The tiles this workgroup walks: first, first + step, ... < last.
  //  walk 0: a contiguous run of tiles_per_wg tiles;
  //  walk 1: workgroups are dispatched to the 8 XCDs round-robin, so
  //    XCD x = blockIdx % 8 owns the x-th eighth of all tiles and its
  //    workgroups interleave through it: at any moment the resident
  //    workgroups of one XCD stream adjacent tiles (DRAM page locality, and
  //    each halo is the neighbour's tail, in the same L2).
  int first, step, last;
  if (a.walk == 0) {
    first = blockIdx.x * a.tiles_per_wg;
    step = 1;
    last = min(first + a.tiles_per_wg, total);
  } else {
    const int per_xcd = (total + 7) / 8;
    const int x = blockIdx.x & 7;
    step = gridDim.x >> 3;
    first = x * per_xcd + (blockIdx.x >> 3);
    last = min((x + 1) * per_xcd, total);
  }
  if (first >= last) return;
#ifdef SDR_FIR_TRACE
  unsigned long long tr_sum[4] = {}, tr_last = 0, tr_n = 0, tr_r0 = __builtin_amdgcn_s_memrealtime(), tr_m0 = __builtin_amdgcn_s_memtime();
#define SDR_TRACE_AT(i)                                        \
  {                                                            \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    if ((i) > 0) tr_sum[(i) - 1] += now_ - tr_last;            \
    tr_last = now_;                                            \
  }
#else
#define SDR_TRACE_AT(i)
#endif

  using Stage = float4[G::FULL + 1];
  Stage sa0, sa1;
#pragma unroll
  for (int i = 0; i <= G::FULL; ++i) sa0[i] = sa1[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (SDR_ABL(a.ablate) != 1)
    stage_load<D, T, R, DEMOD, NW, NCH, SRC>(tile_ref<D, T, R, DEMOD, NW, NCH, SRC>(a, first), n, tid, sa0, sa1);

  auto tile = [&](const int lin, Stage& v0, Stage& v1) __attribute__((always_inline)) {
    const TileRef tr = tile_ref<D, T, R, DEMOD, NW, NCH, SRC>(a, lin);
    // Old prev_I/prev_Q, read before this workgroup rewrites them at the
    // end of the iteration (tile 0 only).
    float old_pi = 0.0f, old_pq = 0.0f;
    if constexpr (DEMOD) {
      // scalar loads (lgkmcnt, not vmcnt): a conditional vector load here
      // makes the waitcnt pass drain the prefetch queue at the scan.  The
      // value is the launch's input: only this workgroup rewrites it, after
      // this read.
      if (tr.t == 0) {  // workgroup-uniform
        using cf = const __attribute__((address_space(4))) float*;
        const int s = __builtin_amdgcn_readfirstlane(tr.s);
        old_pi = ((cf)a.prev0)[s];
        old_pq = ((cf)a.prev1)[s];
      }
    }

    // ---- 1. registers -> LDS (after every read of the previous tile), then
    // prefetch the next tile into the registers just freed.  Tile 0 also
    // stages the block's last STRIP inputs (old state where p < 0: the
    // D*(nout-1) - k >= -(T-1) >= -ns inputs of the last output) before it
    // rewrites the state below.
    SDR_TRACE_AT(0);
    __syncthreads();
#ifdef SDR_FIR_TRACE
    __builtin_amdgcn_s_waitcnt(0);
    SDR_TRACE_AT(1);
#endif
    stage_store<D, T, R, DEMOD, NW, NCH, SRC>(lds0, lds1, tid, v0, v1);
    if (tr.t == 0 || !interior<D, T, R, DEMOD, NW>(tr, n)) {  // workgroup-uniform
      __syncthreads();
      edge_fill<D, T, R, DEMOD, NW, NCH, SRC>(tr, tid, n, ns, [&](int i, float v0, float v1) {
        lds0[i] = v0;
        if (NCH == 2) lds1[i] = v1;
      });
    }
    __syncthreads();
    SDR_TRACE_AT(2);
    if (lin + step < last && SDR_ABL(a.ablate) != 1)
      stage_load<D, T, R, DEMOD, NW, NCH, SRC>(tile_ref<D, T, R, DEMOD, NW, NCH, SRC>(a, lin + step), n, tid, v0, v1);

    // ---- 2. slide down this lane's window, R outputs x NCH channels in registers
    // Lane (wave, lane) owns outputs m_start + wave*WADV + R*lane + r.  Per
    // 4-position chunk c it reads NCH input float4s of its own window; the
    // next chunk is prefetched, and the sched_barrier keeps the scheduler from
    // hoisting every LDS read of the unrolled loop (registers -> occupancy).
    const int lbase = D * (wave * G::WADV + R * lane);  // LDS index of this lane's window
    float acc0[R], acc1[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      acc0[r] = 0.0f;
      acc1[r] = 0.0f;
    }
    if (SDR_ABL(a.ablate) == 2) {
      acc0[0] = lds0[lbase];
      if (NCH == 2) acc1[0] = lds1[lbase];
    } else {
      const float* w0 = lds0 + lbase;
      const float* w1 = lds1 + lbase;
      {
        // Taps as SGPR operands of the multiplies: no LDS tap traffic.  All
        // T taps do not fit the SGPR file beside the addressing, so the
        // window is walked in NPASS passes over consecutive tap ranges
        // [k0, k1), each loading its taps once (scalar loads from the
        // constant address space, one wait) -- every output still visits
        // k = 0..T-1 in order, the passes only split its chain.
        constexpr int NPASS = SDR_NPASS, KP = (T + NPASS - 1) / NPASS;
        using hconst = const __attribute__((address_space(4))) float*;
        const hconst hc = (hconst)h;
        float hs[KP];
        static_for<0, NPASS>([&](auto pi) {
          constexpr int k0 = decltype(pi)::value * KP;
          constexpr int k1 = k0 + KP < T ? k0 + KP : T;
          // ablate 4 (timing only): one pass of three -- how much a cheaper scan buys
          if (SDR_ABL(a.ablate) == 4 && k0 > 0) return;
#pragma unroll
          for (int i = 0; i < k1 - k0; ++i) hs[i] = hc[k0 + i];
#pragma unroll
          for (int i = 0; i < k1 - k0; ++i) asm volatile("" : "+s"(hs[i]));
          // window positions w = HALO + D r - k this pass touches
          constexpr int wlo = G::HALO - (k1 - 1) > 0 ? G::HALO - (k1 - 1) : 0;
          constexpr int whi = G::HALO + D * (R - 1) - k0;
          constexpr int clo = wlo / 4, chi = whi / 4;
          // SDR_SCAN_PF chunks of LDS reads in flight ahead of the one in use
          constexpr int PF = SDR_SCAN_PF;
          float4 pf0[PF + 1], pf1[PF + 1];
          static_for<0, PF>([&](auto ui) {
            constexpr int u = decltype(ui)::value;
            if constexpr (chi - u >= clo) {
              pf0[u] = *reinterpret_cast<const float4*>(w0 + 4 * (chi - u));
              pf1[u] = pf0[u];
              if (NCH == 2) pf1[u] = *reinterpret_cast<const float4*>(w1 + 4 * (chi - u));
            }
          });
          static_for<0, chi - clo + 1>([&](auto ci) {
            constexpr int c = chi - decltype(ci)::value;
            if constexpr (c - PF >= clo) {
              pf0[PF] = *reinterpret_cast<const float4*>(w0 + 4 * (c - PF));
              if (NCH == 2) pf1[PF] = *reinterpret_cast<const float4*>(w1 + 4 * (c - PF));
            }
            const float4 q0 = pf0[0], q1 = NCH == 2 ? pf1[0] : pf0[0];
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
#pragma unroll
            for (int u = 0; u < PF; ++u) {
              pf0[u] = pf0[u + 1];
              pf1[u] = pf1[u + 1];
            }
#pragma unroll
            for (int r = 0; r < R; ++r) asm volatile("" : "+v"(acc0[r]), "+v"(acc1[r]));
            __builtin_amdgcn_sched_barrier(0);
          });
        });
      }
    }

    SDR_TRACE_AT(3);
    const long long m0 = tr.m_start + (long long)wave * G::WADV + (long long)R * lane;  // this lane's first output
    if constexpr (DEMOD) {
      // ---- 3. discriminator in registers.  The decimated sample before
      // output r=0 is lane-1's last output (a wave shuffle); lane 0's
      // outputs are the wave's overlap and are not stored, except at the
      // start of the stream (tile 0, wave 0, lane 0 -> outputs 0..R-1),
      // whose predecessor is the carried prev_*.
      float pI = __shfl_up(acc0[R - 1], 1, 64);
      float pQ = __shfl_up(acc1[R - 1], 1, 64);
      const bool first = tr.t == 0 && tid == 0;
      if (first) {
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
      if (lane >= 1 || first) {
        if (vec && m0 + R <= nout) {
          if constexpr (R == 2) {
            if constexpr (SDR_OUT_NT && SRC == Src::F32) {
              typedef float f2 __attribute__((ext_vector_type(2)));
              __builtin_nontemporal_store(f2{d[0], d[1]}, reinterpret_cast<f2*>(o + m0));
            } else {
              *reinterpret_cast<float2*>(o + m0) = make_float2(d[0], d[1]);
            }
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
      // stage the block's last STRIP inputs (old state where p < 0: the
      // D*(nout-1) - k >= -(T-1) >= -ns inputs of the last output) into the
      // channel buffers, free once every lane's scan has read them
      __syncthreads();
      for (int j0 = 0; j0 < G::STRIP; j0 += 4 * NTH) {
        float v0[4], v1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = j0 + u * NTH + tid;
          const long long p = n - G::STRIP + j;
          v0[u] = v1[u] = 0.0f;
          if (j < G::STRIP) {
            v0[u] = edge_at<SRC>(tr.x0, tr.iq, 0, tr.st0, ns, n, p);
            if (NCH == 2) v1[u] = edge_at<SRC>(tr.x1, tr.iq, 1, tr.st1, ns, n, p);
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = j0 + u * NTH + tid;
          if (j < G::STRIP) {
            strip0[j] = v0[u];
            if (NCH == 2) strip1[j] = v1[u];
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0);  // as in edge_fill: keep the waitcnt pass from draining at the next scan
      __syncthreads();
      if constexpr (DEMOD) {
        // prev_* <- last decimated I/Q of the block (src/filter.cpp:100-101),
        // recomputed in the reference's order from the staged strip:
        // input D*(nout-1) - k = n - D - k sits at strip index STRIP - D - k
        // (lane c < 2 runs channel c; groups of 8 LDS reads in flight -- a
        // full unroll would hold all T reads live and cost a wave per SIMD
        // of occupancy for the whole kernel)
        if (tid < 2) {
          using hconst = const __attribute__((address_space(4))) float*;
          const hconst hc = (hconst)h;
          const float* sp = (tid == 0 ? strip0 : strip1) + (G::STRIP - D);
          float y = 0.0f;
#pragma unroll 8
          for (int k = 0; k < T; ++k) y = y + hc[k] * sp[-k];
          (tid == 0 ? a.prev0 : a.prev1)[tr.s] = y;
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
  };

#ifdef SDR_FIR_TRACE
  for (int lin = first; lin < last; lin += step) {
    tile(lin, sa0, sa1);
    SDR_TRACE_AT(4);
    ++tr_n;
  }
  if (tid == 0 && blockIdx.x < kTraceWG) {
    unsigned long long* o = g_fir_trace + (unsigned long long)kTraceW * blockIdx.x;
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    o[0] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
    o[1] = tr_r0;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[2 + i] = tr_sum[i];
    o[6] = tr_n;
    o[7] = __builtin_amdgcn_s_memrealtime();
    o[8] = tr_m0;
    o[9] = __builtin_amdgcn_s_memtime();
  }
#else
  for (int lin = first; lin < last; lin += step) tile(lin, sa0, sa1);
#endif
}
#undef SDR_TRACE_AT


// A wave's own LDS slice is published to its other lanes: LDS operations of
// one wave execute in order, so the wait and a compiler barrier suffice (the
// workgroup's other waves work on other tiles and are never waited for).
__device__ __forceinline__ void wave_sync() {
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_wave_barrier();
}

// Launch shape: persistent workgroups (a group each, one or two per CU),
// blockDim.x / 64 waves each.  Every wave owns one LDS slice of grp_slice()
// floats and works through the group's tiles on its own, claiming the next
// one from a counter in LDS when its staging is done, so the waves on a
// lightly loaded SIMD take more tiles than those sharing a SIMD with more
// waves.  The group's k-th claim is tile  slab + j + k * groups_per_slab
// (walk 1: group g = 8j + x works in XCD slab x, a contiguous eighth of the
// tiles; walk 0: one slab): the chip streams through a contiguous window of
// each slab, as one workgroup per tile dispatched in order did, and a
// tile's halo -- its neighbour's tail -- is read in the same XCD's L2 (round
// robin placement; speed only).  One workgroup per tile, the round-2 shape,
// left a CU with 10-11 of its 14 workgroup slots occupied on average:
// workgroup dispatch, not HBM, set the rate (tools/fir_trace.py); a static
// persistent walk lost the difference in its tail; giving each group a
// contiguous run of tiles instead (256 separate read cursors) cost 13 % on
// cfg2.
#ifndef SDR_FIR_LB
#define SDR_FIR_LB 1024
#endif
// SDR_GRP_T0PRE: fir_tile_grp's one-channel f32 tile 0 loads its extra inputs
// (carried state, new state, side copy) before the span's wait
#ifndef SDR_GRP_T0PRE
#define SDR_GRP_T0PRE 1
#endif
// fir_tile_grp's LDS floats per wave: one span per channel (a one-channel
// FIR needs half of fir_tile's two-channel slice: 16 waves of the D = 5 / 1
// FIRs fit a CU instead of 14, one round of tiles instead of two)
#ifndef SDR_GRP_CH_SLICE
#define SDR_GRP_CH_SLICE 1  // 0: two spans per wave whatever NCH (the round-4 layout, A/B)
#endif
template <int D, int T, int R, bool DEMOD, int NCH>
constexpr int grp_slice() {
  return (SDR_GRP_CH_SLICE ? NCH : 2) * Geom<D, T, R, DEMOD, 1>::LDS_LEN;
}
template <int D, int T, int R, int NW, int NCH, bool DEMOD, Src SRC, int TM, bool FMA = false>
__global__ __launch_bounds__(SDR_FIR_LB) void fir_tile_grp(FirLaunch a, const float* __restrict__ h) {
  using G = Geom<D, T, R, DEMOD, NW>;
  constexpr int NTH = G::NTH;
  static_assert(NW == 1, "one wave per tile");
  static_assert(NCH == 2 || !DEMOD, "the discriminator needs I and Q");
  static_assert(SRC == Src::F32 || NCH == 2, "u8 wire format carries I and Q");
  static_assert(TM == 1, "taps as SGPR operands");

  extern __shared__ __attribute__((aligned(16))) float smem[];
  __shared__ int next_tile;  // the group's claim counter
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
  float* lds0 = smem + wv * grp_slice<D, T, R, DEMOD, NCH>();  // this wave's slice
  float* lds1 = lds0 + G::LDS_LEN;
  float* strip0 = lds0;  // the block's last inputs (tile 0, after its scan)
  float* strip1 = lds1;

  const int tid = threadIdx.x & 63;
  const int lane = tid, wave = 0;
  const long long n = a.n;
  const long long nout = n / D;
  const int ns = a.ns;
  const int total = a.nstreams * a.tiles_per_stream;
  // group b: slab x = b % 8 (walk 1; workgroups are dealt to the XCDs round
  // robin, so a slab's groups share an L2: speed only), the j-th run of
  // a.tiles_per_wg consecutive tiles in it
  // the group's k-th tile is slab start + j + k * (groups per slab): all
  // groups of a slab advance through one window of it (a.walk: 8 slabs)
  const int sh = a.walk ? 3 : 0;
  const int x = blockIdx.x & ((1 << sh) - 1), j = blockIdx.x >> sh, gps = gridDim.x >> sh;
  const int s_lo = x * a.slab, s_hi = min(s_lo + a.slab, total);
  if (threadIdx.x == 0) next_tile = 0;
  __syncthreads();  // the only workgroup barrier
  // one LDS atomic per claim (lgkmcnt: never waits on vector memory)
  auto claim = [&]() __attribute__((always_inline)) {
    int v = 0;
    if (tid == 0) v = atomicAdd(&next_tile, 1);
    v = s_lo + j + __builtin_amdgcn_readfirstlane(v) * gps;
    return v < s_hi ? v : -1;
  };
  const int first = claim();
  if (first < 0) return;
#ifdef SDR_FIR_TRACE
  unsigned long long tr_sum[4] = {}, tr_last = 0, tr_n = 0, tr_r0 = __builtin_amdgcn_s_memrealtime(), tr_m0 = __builtin_amdgcn_s_memtime();
#define SDR_TRACE_AT(i)                                        \
  {                                                            \
    const unsigned long long now_ = __builtin_amdgcn_s_memtime(); \
    if ((i) > 0) tr_sum[(i) - 1] += now_ - tr_last;            \
    tr_last = now_;                                            \
  }
#else
#define SDR_TRACE_AT(i)
#endif

  using Stage = float4[G::FULL + 1];
  Stage sa0, sa1;
#pragma unroll
  for (int i = 0; i <= G::FULL; ++i) sa0[i] = sa1[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (SDR_ABL(a.ablate) != 1)
    stage_load<D, T, R, DEMOD, NW, NCH, SRC>(tile_ref<D, T, R, DEMOD, NW, NCH, SRC>(a, first), n, tid, sa0, sa1);

  // A tile's outputs wait in registers and are stored after the next tile's
  // loads have been waited for: stored at the end of their own tile, they
  // were the youngest vector-memory operations when the next tile's staging
  // waited (vmcnt counts loads and stores in issue order), so every tile paid
  // its stores' write latency on top of its loads'.
  float pend[R];
  float* pend_row = nullptr;
  int16_t* pend_pcm = nullptr;  // FIR-only launches with a.pcm: the s16 row
  long long pend_m0 = nout;  // nout: nothing pending in this lane
  bool pend_vec = false;
  auto flush = [&]() __attribute__((always_inline)) {
    if constexpr (!DEMOD) {
      if (a.pcm) {  // launch-uniform: s16 PCM (src/project.cpp:311-314) instead of f32
        int16_t* o = pend_pcm;
        if (pend_vec && pend_m0 + R <= nout) {
          if constexpr (R == 4) {
            typedef short s4 __attribute__((ext_vector_type(4)));
            *reinterpret_cast<s4*>(o + pend_m0) = s4{pcm_quantise(pend[0]), pcm_quantise(pend[1]),
                                                     pcm_quantise(pend[2]), pcm_quantise(pend[3])};
          } else {
#pragma unroll
            for (int r = 0; r < R; ++r) o[pend_m0 + r] = pcm_quantise(pend[r]);
          }
        } else {
#pragma unroll
          for (int r = 0; r < R; ++r)
            if (pend_m0 + r < nout) o[pend_m0 + r] = pcm_quantise(pend[r]);
        }
        pend_m0 = nout;
        return;
      }
    }
    float* o = pend_row;
    if (pend_vec && pend_m0 + R <= nout) {
      if constexpr (R == 2) {
        typedef float f2 __attribute__((ext_vector_type(2)));
        if constexpr (SDR_OUT_NT && SRC == Src::F32 && DEMOD)
          __builtin_nontemporal_store(f2{pend[0], pend[1]}, reinterpret_cast<f2*>(o + pend_m0));
        else
          *reinterpret_cast<f2*>(o + pend_m0) = f2{pend[0], pend[1]};
      } else if constexpr (R == 4) {
        *reinterpret_cast<float4*>(o + pend_m0) = make_float4(pend[0], pend[1], pend[2], pend[3]);
      } else {
#pragma unroll
        for (int r = 0; r < R; ++r) o[pend_m0 + r] = pend[r];
      }
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r)
        if (pend_m0 + r < nout) o[pend_m0 + r] = pend[r];
    }
    pend_m0 = nout;
  };
  // nxt(): the tile to prefetch after this one's staging (-1: none)
  auto tile = [&](const int lin, auto&& nxt, Stage& v0, Stage& v1) __attribute__((always_inline)) {
    const TileRef tr = tile_ref<D, T, R, DEMOD, NW, NCH, SRC>(a, lin);
    // Old prev_I/prev_Q, read before this workgroup rewrites them at the
    // end of the iteration (tile 0 only).
    float old_pi = 0.0f, old_pq = 0.0f;
    if constexpr (DEMOD) {
      // scalar loads (lgkmcnt, not vmcnt): a conditional vector load here
      // makes the waitcnt pass drain the prefetch queue at the scan.  The
      // value is the launch's input: only this workgroup rewrites it, after
      // this read.
      if (tr.t == 0) {  // workgroup-uniform
        using cf = const __attribute__((address_space(4))) float*;
        const int s = __builtin_amdgcn_readfirstlane(tr.s);
        old_pi = ((cf)a.prev0)[s];
        old_pq = ((cf)a.prev1)[s];
      }
    }

    // ---- 1. registers -> LDS (after every read of the previous tile), then
    // prefetch the next tile into the registers just freed.  Tile 0 also
    // stages the block's last STRIP inputs (old state where p < 0: the
    // D*(nout-1) - k >= -(T-1) >= -ns inputs of the last output) before it
    // rewrites the state below.
    SDR_TRACE_AT(0);
    // A one-channel f32 FIR's tile 0 (SDR_GRP_T0PRE): the carried state under
    // the span's head, the new state (the block's last ns inputs) and the side
    // copy as unguarded loads at clamped indices here, before the span's wait
    // -- instead of an edge pass after it and the tail loads after the scan
    constexpr int kPre = (G::HALO > 64 * kSideMax ? G::HALO : 64 * kSideMax) / 64 + 1;
    float e_pre[kPre], n_pre[kPre], side[kSideMax];
    const bool t0pre = SDR_GRP_T0PRE && !DEMOD && NCH == 1 && SRC == Src::F32 && tr.t == 0 && ns >= (int)-tr.pb &&
                       ns <= 64 * kPre && n >= ns && ((n & 3) == 0 || tr.pb + G::LDS_LEN <= (n & ~3LL));
    if (t0pre) {
#pragma unroll
      for (int u = 0; u < kPre; ++u) {
        const int i = tid + 64 * u;
        e_pre[u] = tr.st0[ns + tr.pb + min(i, (int)-tr.pb - 1)];
        n_pre[u] = tr.x0[n - ns + min(i, ns - 1)];
      }
      side_load(a, tr.s, tid, NTH, side);
    }
    wave_sync();
#ifdef SDR_FIR_TRACE
    __builtin_amdgcn_s_waitcnt(0);
    SDR_TRACE_AT(1);
#endif
    stage_store<D, T, R, DEMOD, NW, NCH, SRC>(lds0, lds1, tid, v0, v1);
    if (t0pre) {
#pragma unroll
      for (int u = 0; u < kPre; ++u)
        if (tid + 64 * u < (int)-tr.pb) lds0[tid + 64 * u] = e_pre[u];
    } else if (tr.t == 0 || !interior<D, T, R, DEMOD, NW>(tr, n)) {  // workgroup-uniform
      wave_sync();
      edge_fill<D, T, R, DEMOD, NW, NCH, SRC>(tr, tid, n, ns, [&](int i, float v0, float v1) {
        lds0[i] = v0;
        if (NCH == 2) lds1[i] = v1;
      });
    }
    wave_sync();
    SDR_TRACE_AT(2);
    const int next = nxt();
    if constexpr (SDR_FIR_DEFER) flush();  // the previous tile's outputs
    if (next >= 0 && SDR_ABL(a.ablate) != 1)
      stage_load<D, T, R, DEMOD, NW, NCH, SRC>(tile_ref<D, T, R, DEMOD, NW, NCH, SRC>(a, next), n, tid, v0, v1);

    // ---- 2. slide down this lane's window, R outputs x NCH channels in registers
    // Lane (wave, lane) owns outputs m_start + wave*WADV + R*lane + r.  Per
    // 4-position chunk c it reads NCH input float4s of its own window; the
    // next chunk is prefetched, and the sched_barrier keeps the scheduler from
    // hoisting every LDS read of the unrolled loop (registers -> occupancy).
    const int lbase = D * (wave * G::WADV + R * lane);  // LDS index of this lane's window
    float acc0[R], acc1[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      acc0[r] = 0.0f;
      acc1[r] = 0.0f;
    }
    if (SDR_ABL(a.ablate) == 2) {
      acc0[0] = lds0[lbase];
      if (NCH == 2) acc1[0] = lds1[lbase];
    } else {
      const float* w0 = lds0 + lbase;
      const float* w1 = lds1 + lbase;
      {
        // Taps as SGPR operands of the multiplies: no LDS tap traffic.  All
        // T taps do not fit the SGPR file beside the addressing, so the
        // window is walked in NPASS passes over consecutive tap ranges
        // [k0, k1), each loading its taps once (scalar loads from the
        // constant address space, one wait) -- every output still visits
        // k = 0..T-1 in order, the passes only split its chain.
        constexpr int NPASS = SDR_NPASS, KP = (T + NPASS - 1) / NPASS;
        using hconst = const __attribute__((address_space(4))) float*;
        const hconst hc = (hconst)h;
        float hs[KP];
        static_for<0, NPASS>([&](auto pi) {
          constexpr int k0 = decltype(pi)::value * KP;
          constexpr int k1 = k0 + KP < T ? k0 + KP : T;
          // ablate 4 (timing only): one pass of three -- how much a cheaper scan buys
          if (SDR_ABL(a.ablate) == 4 && k0 > 0) return;
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
    }

    SDR_TRACE_AT(3);
    // ---- 3. the tile's outputs, kept in registers (pend) and stored after
    // the NEXT tile's staging -- see flush()
    const long long m0 = tr.m_start + (long long)wave * G::WADV + (long long)R * lane;  // this lane's first output
    if constexpr (DEMOD) {
      // discriminator in registers.  The decimated sample before output r=0
      // is lane-1's last output (a wave shuffle); lane 0's outputs are the
      // wave's overlap and are not stored, except at the start of the stream
      // (tile 0, wave 0, lane 0 -> outputs 0..R-1), whose predecessor is the
      // carried prev_*.
      float pI = __shfl_up(acc0[R - 1], 1, 64);
      float pQ = __shfl_up(acc1[R - 1], 1, 64);
      const bool first = tr.t == 0 && tid == 0;
      if (first) {
        pI = old_pi;
        pQ = old_pq;
      }
#pragma unroll
      for (int r = 0; r < R; ++r) {
        const float ip = r ? acc0[r - 1] : pI;
        const float qp = r ? acc1[r - 1] : pQ;
        pend[r] = demod_one(acc0[r], acc1[r], ip, qp);
      }
      pend_row = a.out + (long long)tr.s * a.out_stride;
      pend_m0 = (lane >= 1 || first) ? m0 : nout;  // lane 0 of a later tile: recomputed overlap, not stored
    } else {
#pragma unroll
      for (int r = 0; r < R; ++r) pend[r] = acc0[r];
      pend_m0 = m0;
      if (a.pcm) pend_pcm = a.pcm + (long long)tr.s * a.pcm_stride;
      else pend_row = a.y0 + (long long)tr.s * a.y_stride;
    }
    // vector stores when the row keeps R-element groups aligned (uniform)
    if (!DEMOD && a.pcm)
      pend_vec = ((reinterpret_cast<uintptr_t>(pend_pcm) + 2ull * (unsigned long long)tr.m_start) % (2u * R)) == 0;
    else
      pend_vec = ((reinterpret_cast<uintptr_t>(pend_row) + 4ull * (unsigned long long)tr.m_start) % (4u * R)) == 0;
    if constexpr (!SDR_FIR_DEFER) flush();

    // ---- 4. state carry (tile 0 only; every read of the old values
    // happened before the barriers above)
    if (t0pre) {
      // the new state and the side copy straight from registers (no strip)
      side_store(a, tr.s, tid, NTH, side);
#pragma unroll
      for (int u = 0; u < kPre; ++u)
        if (tid + 64 * u < ns) tr.st0[tid + 64 * u] = n_pre[u];
    } else if (tr.t == 0) {
      side_load(a, tr.s, tid, NTH, side);
      // stage the block's last STRIP inputs (old state where p < 0: the
      // D*(nout-1) - k >= -(T-1) >= -ns inputs of the last output) into the
      // channel buffers, free once every lane's scan has read them
      wave_sync();
      for (int j0 = 0; j0 < G::STRIP; j0 += 4 * NTH) {
        float v0[4], v1[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = j0 + u * NTH + tid;
          const long long p = n - G::STRIP + j;
          v0[u] = v1[u] = 0.0f;
          if (j < G::STRIP) {
            v0[u] = edge_at<SRC>(tr.x0, tr.iq, 0, tr.st0, ns, n, p);
            if (NCH == 2) v1[u] = edge_at<SRC>(tr.x1, tr.iq, 1, tr.st1, ns, n, p);
          }
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = j0 + u * NTH + tid;
          if (j < G::STRIP) {
            strip0[j] = v0[u];
            if (NCH == 2) strip1[j] = v1[u];
          }
        }
      }
      __builtin_amdgcn_s_waitcnt(0);  // as in edge_fill: keep the waitcnt pass from draining at the next scan
      side_store(a, tr.s, tid, NTH, side);
      wave_sync();
      if constexpr (DEMOD) {
        // prev_* <- last decimated I/Q of the block (src/filter.cpp:100-101),
        // recomputed in the reference's order from the staged strip:
        // input D*(nout-1) - k = n - D - k sits at strip index STRIP - D - k
        // (lane c < 2 runs channel c; groups of 8 LDS reads in flight -- a
        // full unroll would hold all T reads live and cost a wave per SIMD
        // of occupancy for the whole kernel)
        if (tid < 2) {
          using hconst = const __attribute__((address_space(4))) float*;
          const hconst hc = (hconst)h;
          const float* sp = (tid == 0 ? strip0 : strip1) + (G::STRIP - D);
          float y = 0.0f;
#pragma unroll 8
          for (int k = 0; k < T; ++k) y = y + hc[k] * sp[-k];
          (tid == 0 ? a.prev0 : a.prev1)[tr.s] = y;
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
  };

#ifdef SDR_FIR_TRACE
#define SDR_TRACE_TILE() \
  SDR_TRACE_AT(4);       \
  ++tr_n
#else
#define SDR_TRACE_TILE()
#endif
  for (int lin = first; lin >= 0;) {
    int next = -1;
    tile(lin, [&]() __attribute__((always_inline)) {
      next = claim();
      return next;
    }, sa0, sa1);
    SDR_TRACE_TILE();
    lin = next;
  }
  flush();
#undef SDR_TRACE_TILE
#ifdef SDR_FIR_TRACE
  if (tid == 0 && blockIdx.x * 16 + wv < kTraceWG) {  // one record per wave
    unsigned long long* o = g_fir_trace + (unsigned long long)kTraceW * (blockIdx.x * 16 + wv);
    const unsigned hw = __builtin_amdgcn_s_getreg((31 << 11) | 4);    // HW_REG_HW_ID
    const unsigned xcc = __builtin_amdgcn_s_getreg((31 << 11) | 20);  // HW_REG_XCC_ID
    o[0] = (unsigned long long)hw | ((unsigned long long)xcc << 32);
    o[1] = tr_r0;
#pragma unroll
    for (int i = 0; i < 4; ++i) o[2 + i] = tr_sum[i];
    o[6] = tr_n;
    o[7] = __builtin_amdgcn_s_memrealtime();
    o[8] = tr_m0;
    o[9] = __builtin_amdgcn_s_memtime();
  }
#endif
}
#undef SDR_TRACE_AT

// ------------------------------------------------ split-channel front end --
// One channel of a lane's window: acc[r] = sum_k h[k] * w[HALO + D r - k] in
// the reference's order (k ascending, product and sum rounded separately),
// taps as SGPR operands in NPASS passes -- fir_tile's scan, one channel.
template <int D, int T, int R, bool FMA>
__device__ __forceinline__ void scan_one(const float* w, float (&acc)[R], const float* h) {
  using G = Geom<D, T, R, true, 1>;
  constexpr int NPASS = SDR_NPASS, KP = (T + NPASS - 1) / NPASS;
  using hconst = const __attribute__((address_space(4))) float*;
  const hconst hc = (hconst)h;
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0f;
  float hs[KP];
  static_for<0, NPASS>([&](auto pi) {
    constexpr int k0 = decltype(pi)::value * KP;
    constexpr int k1 = k0 + KP < T ? k0 + KP : T;
#pragma unroll
    for (int i = 0; i < k1 - k0; ++i) hs[i] = hc[k0 + i];
#pragma unroll
    for (int i = 0; i < k1 - k0; ++i) asm volatile("" : "+s"(hs[i]));
#if SDR_SCAN_VCONST
    // timing ablation only (wrong outputs): every multiply of the pass takes
    // one VGPR operand instead of its SGPR tap
    float hvc[R];  // one per output, so no two products are the same value (no CSE)
#pragma unroll
    for (int r = 0; r < R; ++r) {
      hvc[r] = hs[r];
      asm volatile("" : "+v"(hvc[r]));
    }
#endif
    constexpr int wlo = G::HALO - (k1 - 1) > 0 ? G::HALO - (k1 - 1) : 0;
    constexpr int whi = G::HALO + D * (R - 1) - k0;
    constexpr int clo = wlo / 4, chi = whi / 4;
    float4 q0 = *reinterpret_cast<const float4*>(w + 4 * chi);
    float4 q1 = q0;
    if constexpr (chi - 1 >= clo) q1 = *reinterpret_cast<const float4*>(w + 4 * (chi - 1));
    static_for<0, chi - clo + 1>([&](auto ci) {
      constexpr int c = chi - decltype(ci)::value;
      float4 n2 = q1;
      if constexpr (c - 2 >= clo) n2 = *reinterpret_cast<const float4*>(w + 4 * (c - 2));
      const float e[4] = {q0.x, q0.y, q0.z, q0.w};
      static_for<0, 4>([&](auto ji) {
        constexpr int j = 3 - decltype(ji)::value;
        static_for<0, R>([&](auto ri) {
          constexpr int r = decltype(ri)::value;
          constexpr int k = G::HALO + D * r - (4 * c + j);
          if constexpr (k >= k0 && k < k1) {
#if SDR_SCAN_VCONST
            const float tap = hvc[r];
#else
            const float tap = hs[k - k0];
#endif
            if constexpr (FMA)
              acc[r] = __builtin_fmaf(tap, e[j], acc[r]);
            else
              acc[r] = acc[r] + tap * e[j];
          }
        });
      });
      q0 = q1;
      q1 = n2;
#pragma unroll
      for (int r = 0; r < R; ++r) asm volatile("" : "+v"(acc[r]));
      __builtin_amdgcn_sched_barrier(0);
    });
  });
}

// fir_tile_sc: the fused f32 front end with the two channels of a tile on
// two waves.  Wave 0 stages and scans I, wave 1 stages and scans Q, each in
// its own 5,488-B slice; wave 1 hands its R outputs per lane to wave 0
// through LDS (one barrier), wave 0 runs the discriminator and stores.  A
// workgroup lives about as long as one channel's scan instead of two, with
// half the staging registers per wave.  Same tiles, arithmetic, order,
// outputs and state as fir_tile (src/filter.cpp:123-140, 85-102).
template <int D, int T, int R, Src SRC, bool FMA = false>
__global__ __launch_bounds__(128) void fir_tile_sc(FirLaunch a, const float* __restrict__ h) {
  constexpr int NW = 1, NTH = 64;
  constexpr bool DEMOD = true;
  using G = Geom<D, T, R, DEMOD, NW>;
  extern __shared__ __attribute__((aligned(16))) float smem[];
  const int c = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);  // channel of this wave
  const int lane = threadIdx.x & 63;
  float* lds = smem + c * G::LDS_LEN;  // this channel's span
  float* xch = smem + 2 * G::LDS_LEN;  // wave 1's outputs for wave 0
  const long long n = a.n;
  const long long nout = n / D;
  const int ns = a.ns;
  const int total = a.nstreams * a.tiles_per_stream;
  // XCD slabs (fir_tile walk 1): workgroup b runs on XCD b % 8
  const int per_xcd = (total + 7) / 8;
  const int x = blockIdx.x & 7;
  const int lin = x * per_xcd + (blockIdx.x >> 3);
  if (lin >= min((x + 1) * per_xcd, total)) return;
  TileRef tr = tile_ref<D, T, R, DEMOD, NW, 2, SRC>(a, lin);
  if (c) {
    tr.x0 = tr.x1;
    tr.st0 = tr.st1;
  }
  float old_pi = 0.0f, old_pq = 0.0f;
  // (timing ablation 9: tile 0 without its extra work -- wrong outputs; how
  // much the streams' first tiles cost the launch)
  const bool t0x = tr.t == 0 && SDR_ABL(a.ablate) != 9;
  if (c == 0 && t0x) {
    using cf = const __attribute__((address_space(4))) float*;
    const int s = __builtin_amdgcn_readfirstlane(tr.s);
    old_pi = ((cf)a.prev0)[s];
    old_pq = ((cf)a.prev1)[s];
#if !SDR_SC_T0PRE
    // both read before the barrier below: wave 1 rewrites prev_Q after it
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
  }
  using Stage = float4[G::FULL + 1];
  Stage v;
#pragma unroll
  for (int i = 0; i <= G::FULL; ++i) v[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  if (SDR_ABL(a.ablate) != 1) stage_load<D, T, R, DEMOD, NW, 1, SRC>(tr, n, lane, v, v);
  // Tile 0's own inputs go out in the span's load batch (SDR_SC_T0PRE): the
  // carried state under the span's head, the block's last STRIP inputs (the
  // prev_* recompute and the new state) and the side copy -- one memory
  // latency for the tile instead of three (edge loads after the span landed,
  // strip loads after the scan).  Needs the span's top inside the block
  // (t0pre); else tile 0 takes edge_fill and the strip loads as before.
  constexpr int kPre = (G::STRIP > G::HALO ? G::STRIP : G::HALO) / 64 + 1;
  constexpr int kTp = (T + 63) / 64;  // taps per lane for the prev_* recompute's products
  float e_pre[kPre], s_pre[kPre], side[kSideMax], h_pre[kTp];
  // (f32 only: on the u8 wire path it measured 0.5-1 % slower -- its byte
  // loads of the tail; profiles/r05u/ab_t0pre.txt)
  const bool t0pre = SDR_SC_T0PRE && SRC == Src::F32 && t0x && ns <= G::STRIP && ns >= (int)-tr.pb &&
                     n >= G::STRIP &&
                     ((n & 3) == 0 || tr.pb + G::LDS_LEN <= (n & ~3LL));  // workgroup-uniform
  if (t0pre) {
#pragma unroll
    // unguarded loads at clamped indices (the extra lanes' values are never
    // used): no exec-masked load whose merge would make the compiler wait
    for (int u = 0; u < kPre; ++u) {
      const int i = lane + 64 * u;
      e_pre[u] = tr.st0[ns + tr.pb + min(i, (int)-tr.pb - 1)];  // pb = -HALO >= -ns (t0pre)
      // the block's tail (n >= STRIP: inside the block): raw loads, converted
      // where they are stored (a u8 conversion here would wait on each load)
      const long long pt = n - G::STRIP + min(i, G::STRIP - 1);
      if constexpr (SRC == Src::F32)
        s_pre[u] = tr.x0[pt];
      else
        s_pre[u] = __uint_as_float((uint32_t)tr.iq[2 * pt + c]);
    }
    if (c == 0) side_load(a, tr.s, lane, 64, side);
#pragma unroll
    for (int u = 0; u < kTp; ++u) h_pre[u] = h[min(lane + 64 * u, T - 1)];
  }
  if constexpr (SRC == Src::F32) {
    stage_store<D, T, R, DEMOD, NW, 1, SRC>(lds, lds, lane, v, v);
  } else {
    // u8 wire format: both waves load the interleaved bytes (I0 Q0 I1 Q1 | I2 Q2 I3 Q3
    // per chunk; the second read hits L2) and unpack their own channel
    auto put = [&](int i, const float4& w) __attribute__((always_inline)) {
      const uint32_t bx = __float_as_uint(w.x), by = __float_as_uint(w.y);
      if (c == 0)
        *reinterpret_cast<float4*>(lds + 4 * i) = make_float4(u8_byte_to_f32<0>(bx), u8_byte_to_f32<2>(bx),
                                                              u8_byte_to_f32<0>(by), u8_byte_to_f32<2>(by));
      else
        *reinterpret_cast<float4*>(lds + 4 * i) = make_float4(u8_byte_to_f32<1>(bx), u8_byte_to_f32<3>(bx),
                                                              u8_byte_to_f32<1>(by), u8_byte_to_f32<3>(by));
    };
#pragma unroll
    for (int it = 0; it < G::FULL; ++it) put(lane + it * NTH, v[it]);
    if (G::REM && lane < G::REM) put(lane + G::FULL * NTH, v[G::FULL]);
  }
  if (t0pre) {
    // the span's head: the carried state (the clamped chunks there loaded
    // block data), written after this wave's chunk stores to the same slice
#pragma unroll
    for (int u = 0; u < kPre; ++u)
      if (lane + 64 * u < (int)-tr.pb) lds[lane + 64 * u] = e_pre[u];
  } else if (t0x || (tr.t != 0 && !interior<D, T, R, DEMOD, NW>(tr, n))) {
    wave_sync();
    edge_fill<D, T, R, DEMOD, NW, 1, SRC>(tr, lane, n, ns, [&](int i, float v0, float) { lds[i] = v0; }, c);
  }
  wave_sync();  // a wave reads only its own slice
  const int lbase = D * R * lane;
  float acc[R];
  if (SDR_ABL(a.ablate) == 2) {
#pragma unroll
    for (int r = 0; r < R; ++r) acc[r] = lds[lbase + r];
  } else {
    scan_one<D, T, R, FMA>(lds + lbase, acc, h);
  }
  if (c == 1) {
#pragma unroll
    for (int r = 0; r < R; ++r) xch[r * 64 + lane] = acc[r];
  }
#if SDR_SC_T0PRE
  // prev_I / prev_Q read before the barrier: wave 1 rewrites prev_Q after it
  if (c == 0 && t0x) asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
#endif
  __syncthreads();
  if (c == 0) {
    float accQ[R];
#pragma unroll
    for (int r = 0; r < R; ++r) accQ[r] = xch[r * 64 + lane];
    float pI = __shfl_up(acc[R - 1], 1, 64);
    float pQ = __shfl_up(accQ[R - 1], 1, 64);
    const bool first = tr.t == 0 && lane == 0;
    if (first) {
      pI = old_pi;
      pQ = old_pq;
    }
    float d[R];
#pragma unroll
    for (int r = 0; r < R; ++r) {
      const float ip = r ? acc[r - 1] : pI;
      const float qp = r ? accQ[r - 1] : pQ;
      d[r] = demod_one(acc[r], accQ[r], ip, qp);
    }
    const long long m0 = tr.m_start + (long long)R * lane;
    float* o = a.out + (long long)tr.s * a.out_stride;
    const bool vec = ((reinterpret_cast<uintptr_t>(o) + 4ull * (unsigned long long)tr.m_start) % (4u * R)) == 0;
    if (lane >= 1 || first) {
      if (vec && m0 + R <= nout) {
        if constexpr (R == 2) {
          typedef float f2 __attribute__((ext_vector_type(2)));
          if constexpr (SDR_OUT_NT)
            __builtin_nontemporal_store(f2{d[0], d[1]}, reinterpret_cast<f2*>(o + m0));
          else
            *reinterpret_cast<f2*>(o + m0) = f2{d[0], d[1]};
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
  }
  // state carry (tile 0): each wave its own channel, after every read of the old values
  if (t0x) {
    float* strip = lds;  // the scan is done with it
    if (t0pre) {
#pragma unroll
      for (int u = 0; u < kPre; ++u)
        if (lane + 64 * u < G::STRIP)
          strip[lane + 64 * u] = SRC == Src::F32 ? s_pre[u] : u8_to_f32(__float_as_uint(s_pre[u]));
    } else {
      if (c == 0) side_load(a, tr.s, lane, 64, side);
      for (int j0 = 0; j0 < G::STRIP; j0 += 4 * NTH) {
        float w[4];
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = j0 + u * NTH + lane;
          w[u] = j < G::STRIP ? edge_at<SRC>(tr.x0, tr.iq, c, tr.st0, ns, n, n - G::STRIP + j) : 0.0f;
        }
#pragma unroll
        for (int u = 0; u < 4; ++u) {
          const int j = j0 + u * NTH + lane;
          if (j < G::STRIP) strip[j] = w[u];
        }
      }
      __builtin_amdgcn_s_waitcnt(0);
    }
    // (t0pre: no load is outstanding here -- no drain, which would also wait
    // out the tile's output stores just issued)
    if (c == 0) side_store(a, tr.s, lane, 64, side);
    wave_sync();
    {
      // prev_c <- this channel's last decimated output (src/filter.cpp:100-101),
      // recomputed in the reference's order from the strip: the T products
      // h[k] * x[n-D-k] by all lanes at once (each rounded as the reference
      // rounds it), then lane 0 sums them for k = 0..T-1 -- the chain is the
      // adds alone
      static_assert(T <= G::LDS_LEN - G::STRIP, "the products fit the slice after the strip");
      float* prod = strip + G::STRIP;
      const float* sp = strip + (G::STRIP - D);
      if (!t0pre) {
#pragma unroll
        for (int u = 0; u < kTp; ++u) h_pre[u] = lane + 64 * u < T ? h[lane + 64 * u] : 0.0f;
      }
#pragma unroll
      for (int u = 0; u < kTp; ++u) {
        const int k = lane + 64 * u;
        if (k < T) prod[k] = h_pre[u] * sp[-k];
      }
      wave_sync();
      if (lane == 0) {
        float y = 0.0f;
#pragma unroll 8
        for (int k = 0; k < T; ++k) y = y + prod[k];
        (c ? a.prev1 : a.prev0)[tr.s] = y;
      }
    }
    if (ns <= G::STRIP) {
      for (int j = lane; j < ns; j += NTH) tr.st0[j] = strip[G::STRIP - ns + j];
    } else {
      for (int j = lane; j < ns; j += NTH) tr.st0[j] = in_at<SRC>(tr.x0, tr.iq, c, n - ns + j);
    }
  }
}

// ---------------------------------------------------------- generic path --
// Any D / T / ns the tiled kernel is not instantiated for.  One thread per
// output sample, same operation order; x~ read straight from global memory.
template <Src SRC>
__global__ __launch_bounds__(kWG) void fir_generic(FirLaunch a, const float* __restrict__ h, int nch,
                                                   float* y0, float* y1, long long y_stride) {
  const int s = blockIdx.y;
  const long long m = (long long)blockIdx.x * kWG + threadIdx.x;
  const long long nout = a.n / a.D;
  if (m >= nout) return;
  const float* x0 = SRC == Src::F32 ? a.x0 + (long long)s * a.x_stride : nullptr;
  const float* x1 = SRC == Src::F32 && nch == 2 ? a.x1 + (long long)s * a.x_stride : nullptr;
  const uint8_t* iq = SRC == Src::U8 ? a.iq + (long long)s * a.x_stride : nullptr;
  const float* st0 = a.state0 + (long long)s * a.ns;
  const float* st1 = nch == 2 ? a.state1 + (long long)s * a.ns : nullptr;
  const long long P = (long long)a.D * m;
  float acc0 = 0.0f, acc1 = 0.0f;
  for (int k = 0; k < a.ntaps; ++k) {
    const long long p = P - k;
    const float hk = h[k];
    const float v0 = p >= 0 ? in_at<SRC>(x0, iq, 0, p) : st0[a.ns + p];
    acc0 = acc0 + hk * v0;
    if (nch == 2) {
      const float v1 = p >= 0 ? in_at<SRC>(x1, iq, 1, p) : st1[a.ns + p];
      acc1 = acc1 + hk * v1;
    }
  }
  y0[(long long)s * y_stride + m] = acc0;
  if (nch == 2) y1[(long long)s * y_stride + m] = acc1;
}

// state <- last ns inputs; a separate launch after fir_generic (whose
// threads may still be reading the old state otherwise).
template <Src SRC>
__global__ __launch_bounds__(kWG) void commit_state(FirLaunch a, int nch) {
  const int s = blockIdx.y;
  const int j = blockIdx.x * kWG + threadIdx.x;
  if (j >= a.ns) return;
  const float* x0 = SRC == Src::F32 ? a.x0 + (long long)s * a.x_stride : nullptr;
  const float* x1 = SRC == Src::F32 && nch == 2 ? a.x1 + (long long)s * a.x_stride : nullptr;
  const uint8_t* iq = SRC == Src::U8 ? a.iq + (long long)s * a.x_stride : nullptr;
  const long long p = a.n - a.ns + j;
  a.state0[(long long)s * a.ns + j] = in_at<SRC>(x0, iq, 0, p);
  if (nch == 2) a.state1[(long long)s * a.ns + j] = in_at<SRC>(x1, iq, 1, p);
}

// fmDemodArctan over nstreams x n decimated samples (src/filter.cpp:85-102).
// Thread 0 of a stream is the only reader of prev_* and rewrites them.
__global__ __launch_bounds__(kWG) void demod_kernel(const float* I, const float* Q, long long n, long long stride,
                                                    float* prev_i, float* prev_q, float* out, long long out_stride) {
  const int s = blockIdx.y;
  const long long k = (long long)blockIdx.x * kWG + threadIdx.x;
  if (k >= n) return;
  const float* Is = I + (long long)s * stride;
  const float* Qs = Q + (long long)s * stride;
  float ip, qp;
  if (k == 0) {
    ip = prev_i[s];
    qp = prev_q[s];
  } else {
    ip = Is[k - 1];
    qp = Qs[k - 1];
  }
  out[(long long)s * out_stride + k] = demod_one(Is[k], Qs[k], ip, qp);
  if (k == 0) {
    prev_i[s] = Is[n - 1];
    prev_q[s] = Qs[n - 1];
  }
}

// ------------------------------------------------------------ dispatch ----
// persist = false: fir_tile, about `wpc` one-wave workgroups per CU
// requested (64 for the fused f32 front end: one tile each),
// walking XCD slabs.  persist = true: fir_tile_grp, one workgroup per CU (or
// as many as LDS and 32 waves allow) of as many waves as the CU's LDS holds
// slices (<= 16: the 4 waves per SIMD that <= 128 VGPRs allow), the groups
// claiming interleaved tiles of XCD slabs.
template <int D, int T, int R, int NW, int NCH, bool DEMOD, Src SRC, int TM, bool FMA = false>
hipError_t run_tile(const FirLaunch& a0, const float* h, hipStream_t st, bool persist, int wpc) {
  using G = Geom<D, T, R, DEMOD, NW>;
  FirLaunch a = a0;
  const long long nout = a.n / D;
  a.tiles_per_stream = nout > G::E ? (int)((nout - G::E + G::ADV - 1) / G::ADV) : 1;
  const long long total = (long long)a.tiles_per_stream * a.nstreams;
  if (total <= 0 || total > 0x7fffffffLL) return hipErrorInvalidValue;
  const long long ncu = device_cu_count();
  static const int ablate = SDR_TIMING_ENV("SDR_ABLATE", 0);  // timing builds only
  a.ablate = ablate;
  static const int persist_env = SDR_TIMING_ENV("SDR_FIR_PERSIST", -1);  // A/B, timing builds
  if (persist_env >= 0) persist = persist_env != 0;
  if (a.pcm || a.side_n > 0) persist = true;  // only fir_tile_grp implements them
  if (persist) {
    // a CU's LDS (160 KiB on gfx950, read from the device), less the claim counter
    const long long kLds = (long long)device_lds_bytes() - 64;
    constexpr long long slice = (long long)grp_slice<D, T, R, DEMOD, NCH>() * sizeof(float);
    if (kLds < slice) return hipErrorInvalidConfiguration;
    static const int wpg_env = SDR_TIMING_ENV("SDR_FIR_WPG", 0);  // timing builds
    long long wpg = std::min<long long>(16, kLds / slice);
    if (wpg_env > 0) wpg = std::min<long long>(wpg, wpg_env);
    const long long wg_per_cu = std::max<long long>(1, std::min<long long>(32 / wpg, kLds / (wpg * slice)));
    long long groups = std::min<long long>(ncu * wg_per_cu, (total + wpg - 1) / wpg);
    // timing experiments: about k tiles per wave, as many groups as that takes
    static const int wave_tiles = SDR_TIMING_ENV("SDR_FIR_WAVE_TILES", 0);
    if (wave_tiles > 0) groups = std::max<long long>(8, (total + wpg * wave_tiles - 1) / (wpg * wave_tiles) + 7);
    if (total >= 64 && groups >= 8) {
      groups -= groups % 8;
      a.walk = 1;
      a.slab = (int)((total + 7) / 8);
    } else {
      a.walk = 0;
      a.slab = (int)total;
    }
    const long long per = (a.slab + (groups >> (a.walk ? 3 : 0)) - 1) / (groups >> (a.walk ? 3 : 0));
    wpg = std::max<long long>(1, std::min<long long>(wpg, per));
    hipLaunchKernelGGL((fir_tile_grp<D, T, R, NW, NCH, DEMOD, SRC, TM, FMA>), dim3((unsigned)groups),
                       dim3((unsigned)(64 * wpg)), (size_t)(wpg * slice), st, a, h);
    return hipGetLastError();
  }
  static const int per_cu_env = SDR_TIMING_ENV("SDR_WG_PER_CU", 0);
  const int per_cu = per_cu_env > 0 ? per_cu_env : wpc;
  const long long slots = ncu * per_cu * 4 / NW;  // ~per_cu waves per CU
  long long blocks;
  if (total >= 8 * 8) {
    // a multiple of 8 workgroups, none of them idle
    a.walk = 1;
    const long long per_xcd = (total + 7) / 8;
    const long long g = (slots < per_xcd * 8 ? slots : per_xcd * 8) / 8;
    blocks = 8 * (g > 0 ? g : 1);
    a.tiles_per_wg = (int)((per_xcd + blocks / 8 - 1) / (blocks / 8));
  } else {
    a.walk = 0;
    const long long grid = total < slots ? total : slots;
    a.tiles_per_wg = (int)((total + grid - 1) / grid);
    blocks = (total + a.tiles_per_wg - 1) / a.tiles_per_wg;
  }
  const size_t lds = (size_t)G::SMEM * sizeof(float);
  hipLaunchKernelGGL((fir_tile<D, T, R, NW, NCH, DEMOD, SRC, TM, FMA>), dim3((unsigned)blocks), dim3(G::NTH), lds, st,
                     a, h);
  return hipGetLastError();
}

// fir_tile_sc launch: one two-wave workgroup per tile, XCD slabs
template <int D, int T, int R, Src SRC, bool FMA = false>
hipError_t run_tile_sc(const FirLaunch& a0, const float* h, hipStream_t st) {
  using G = Geom<D, T, R, true, 1>;
  FirLaunch a = a0;
  const long long nout = a.n / D;
  a.tiles_per_stream = nout > G::E ? (int)((nout - G::E + G::ADV - 1) / G::ADV) : 1;
  const long long total = (long long)a.tiles_per_stream * a.nstreams;
  if (total <= 0 || total > 0x7fffffffLL - 8) return hipErrorInvalidValue;
  static const int ablate = SDR_TIMING_ENV("SDR_ABLATE", 0);  // timing builds only
  a.ablate = ablate;
  const long long per_xcd = (total + 7) / 8;
  const size_t lds = (size_t)(2 * G::LDS_LEN + 64 * R) * sizeof(float);
  hipLaunchKernelGGL((fir_tile_sc<D, T, R, SRC, FMA>), dim3((unsigned)(8 * per_xcd)), dim3(128), lds, st, a, h);
  return hipGetLastError();
}

// The fused f32 front end runs fir_tile_sc (same box: 0.0978-0.0990 vs
// 0.1015-0.1056 ms on cfg2, profiles/r03_ab/cfg2_split_channel.txt);
// switch SDR_FIR_SC=0 selects fir_tile (the tests run both)
bool sc_enabled() { return sw(kSwFirSc) != 0; }
// the u8 wire path on fir_tile_sc too (cfg2u8 0.0806-0.0813 -> 0.0785-0.0788
// ms, mono0 -1 % on one box); SDR_FIR_SC_U8=0 selects the persistent
// fir_tile_grp (switch SDR_FIR_SC_U8; the tests run both)
bool sc_u8_enabled() { return sw(kSwFirScU8) != 0; }

// Tile shape per decimation factor: R outputs per lane, one wave per
// workgroup, taps in SGPRs (TM 1), waves per CU.  D*R must
// be a multiple of 4 (aligned lane windows).  These are the measured best on
// MI355X (where the variants that lost are listed).
struct Variant {
  int R, NW, tm;
};

Variant variant_for(int D, bool demod, Src src) {
  switch (D) {
    case 10: return {2, 1, 1};
    case 5: return {4, 1, 1};
    // D = 1 (the band-pass filters): SGPR taps too -- 31.4 vs 37.8 us per
    // 1,024 x 5,120 block against LDS tap rows (scripts/d1bench.py)
    case 1: return {4, 1, 1};
    default: return {0, 0, 0};
  }
}

// Runtime twin of Geom: only tile 0 may read the carried state, i.e. tile
// 1's span must start at p >= 0.
bool geometry_ok(int D, int T, int ns, bool demod, Variant v) {
  if (v.R == 0 || ns < T - 1) return false;
  const int halo = (T - 1 + 3) / 4 * 4;
  const int E = demod ? v.R : 0;
  const long long adv = (long long)v.NW * (64 * v.R - E);
  return (long long)D * adv - halo >= 0;
}

template <int NCH, bool DEMOD, Src SRC>
hipError_t dispatch_tile(const FirLaunch& a, const float* h, hipStream_t st, bool* handled) {
  *handled = true;
  constexpr bool kPersistFused = SRC == Src::U8;
  if (a.ntaps == 101) {
    if constexpr (DEMOD) {
      // SDR_ARITH_FMA: instantiated for the fused kernels; any other shape
      // runs the exact arithmetic (inside the tolerance)
      switch (a.D) {
        // fir_tile_sc by default (SDR_FIR_SC=0 / SDR_FIR_SC_U8=0: fir_tile,
        // the u8 wire format on persistent groups) -- DESIGN.md 4.1, 5.2
        case 10:
          if (SRC == Src::F32 ? sc_enabled() : sc_u8_enabled())
            return a.fma ? run_tile_sc<10, 101, 2, SRC, true>(a, h, st) : run_tile_sc<10, 101, 2, SRC>(a, h, st);
          return a.fma ? run_tile<10, 101, 2, 1, NCH, DEMOD, SRC, 1, true>(a, h, st, kPersistFused, 64)
                       : run_tile<10, 101, 2, 1, NCH, DEMOD, SRC, 1>(a, h, st, kPersistFused, 64);
        case 5:
          return a.fma ? run_tile<5, 101, 4, 1, NCH, DEMOD, SRC, 1, true>(a, h, st, kPersistFused, 32)
                       : run_tile<5, 101, 4, 1, NCH, DEMOD, SRC, 1>(a, h, st, kPersistFused, 32);
        default: break;
      }
    } else if constexpr (NCH == 1) {
      switch (a.D) {
        case 10: return run_tile<10, 101, 2, 1, NCH, DEMOD, SRC, 1>(a, h, st, true, 32);
        case 5: return run_tile<5, 101, 4, 1, NCH, DEMOD, SRC, 1>(a, h, st, true, 32);
        case 1: return run_tile<1, 101, 4, 1, NCH, DEMOD, SRC, 1>(a, h, st, true, 32);
        default: break;
      }
    }
  }
  *handled = false;
  return hipSuccess;
}

}  // namespace

bool fir_has_fast_path(int D, int ntaps, int ns, int nch, bool demod, Src src) {
  if (ntaps != 101) return false;
  if (src == Src::U8 && (nch != 2 || !demod)) return false;
  if (demod != (nch == 2)) return false;  // instantiated: fused 2-channel, or 1-channel FIR
  if (D != 10 && D != 5 && !(D == 1 && !demod)) return false;
  return geometry_ok(D, ntaps, ns, demod, variant_for(D, demod, src));
}

hipError_t launch_demod(const float* I, const float* Q, long long n, int nstreams, long long stride, float* prev_i,
                        float* prev_q, float* out, long long out_stride, hipStream_t st) {
  const long long gx = (n + kWG - 1) / kWG;
  hipLaunchKernelGGL(demod_kernel, dim3((unsigned)gx, (unsigned)nstreams), dim3(kWG), 0, st, I, Q, n, stride, prev_i,
                     prev_q, out, out_stride);
  return hipGetLastError();
}

// a.y0/a.y1 receive FIR outputs (non-demod); scratch_y{0,1} ([nstreams][n/D])
// hold decimated I/Q when a demod launch takes the generic path.
hipError_t launch_fir(const FirLaunch& a, const float* h, bool demod, int nch, Src src, hipStream_t st,
                      float* scratch_y0, float* scratch_y1, bool allow_fast) {
  if (allow_fast && fir_has_fast_path(a.D, a.ntaps, a.ns, nch, demod, src)) {
    bool handled = false;
    hipError_t e = hipSuccess;
    if (src == Src::U8) {
      e = dispatch_tile<2, true, Src::U8>(a, h, st, &handled);
    } else if (demod) {
      e = dispatch_tile<2, true, Src::F32>(a, h, st, &handled);
    } else {
      e = dispatch_tile<1, false, Src::F32>(a, h, st, &handled);
    }
    if (handled) return e;
  }
  if (allow_fast && !demod && nch == 1 && src == Src::F32 && fir_long_ok(a.D, a.ntaps, a.ns, a.n))
    return launch_fir_long(a, h, st);
  // generic: FIR (+ separate state commit) (+ separate demod)
  const long long nout = a.n / a.D;
  float* y0 = demod ? scratch_y0 : a.y0;
  float* y1 = demod ? scratch_y1 : a.y1;
  const long long ys = demod ? nout : a.y_stride;
  const dim3 grid((unsigned)((nout + kWG - 1) / kWG), (unsigned)a.nstreams);
  if (src == Src::U8)
    hipLaunchKernelGGL(fir_generic<Src::U8>, grid, dim3(kWG), 0, st, a, h, nch, y0, y1, ys);
  else
    hipLaunchKernelGGL(fir_generic<Src::F32>, grid, dim3(kWG), 0, st, a, h, nch, y0, y1, ys);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const dim3 cgrid((unsigned)((a.ns + kWG - 1) / kWG), (unsigned)a.nstreams);
  if (a.ns > 0) {
    if (src == Src::U8)
      hipLaunchKernelGGL(commit_state<Src::U8>, cgrid, dim3(kWG), 0, st, a, nch);
    else
      hipLaunchKernelGGL(commit_state<Src::F32>, cgrid, dim3(kWG), 0, st, a, nch);
    e = hipGetLastError();
    if (e != hipSuccess) return e;
  }
  if (demod) return launch_demod(y0, y1, nout, a.nstreams, nout, a.prev0, a.prev1, a.out, a.out_stride, st);
  return hipSuccess;
}

}  // namespace sdr

#ifdef SDR_FIR_TRACE
extern "C" int sdr_debug_fir_trace(void* dst, size_t bytes, int reset) {
  if (reset) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_fir_trace)) != hipSuccess) return -2;
    return hipMemset(p, 0, sizeof g_fir_trace) == hipSuccess ? 0 : -2;
  }
  if (bytes > sizeof g_fir_trace) bytes = sizeof g_fir_trace;
  return hipMemcpyFromSymbol(dst, HIP_SYMBOL(g_fir_trace), bytes, 0, hipMemcpyDeviceToHost) == hipSuccess ? 0 : -2;
}
#endif
