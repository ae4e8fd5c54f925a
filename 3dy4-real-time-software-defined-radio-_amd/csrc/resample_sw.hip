// resample_sw.hip -- the polyphase resampler (src/filter.cpp:142-173) as a
// sliding window over each stream: lane = stream segment, taps as SGPR
// operands of packed instructions, every staged input read once per two
// outputs.  Opt-in (SDR_RESAMPLE_SW=1): measured slower than resample_lp on
// cfg3 (DESIGN.md section 4.4 records why).
//
// Phase algebra (resample.hip): output j has tap row p(j) = (j*M) mod L and
// newest input q(j) = floor(j*M/L); y[j] = sum_{i<C} h[p + i*L] * x[q - i],
// i ascending, separately rounded products and sums from 0.0f.
//
// Shape.  For the taps to be scalar operands all 64 lanes of a workgroup sit
// at the same output offset r of their own segment, and every segment starts
// on a column boundary (a multiple of L outputs), so p and q - q(segment
// start) depend on r only.  Lane l owns segment l of the workgroup's lane
// group (a stream, or a run of K columns of one); the workgroup walks the
// outputs r in [o0, o1) of its 64 segments in slabs of SL consecutive
// outputs, wave w taking outputs r0 + 2w and r0 + 2w + 1.  One ds_read_b128
// of four staged inputs feeds both outputs: v_pk_mul_f32 multiplies an
// input (broadcast to both halves by op_sel) by an SGPR pair (tap of a, tap
// of b) and v_pk_add_f32 advances both sums -- one full-rate instruction per
// multiply-add (unpacked ops with an SGPR or DPP operand issue at half rate,
// profiles/r02_ubench_valu.txt).  The inner loop is one self-contained asm
// statement (resample_sw_pair.inc, scripts/gen_sw_asm.py).
//
// Staging: each lane keeps a ring of kSwRingC 16-B chunks of its segment's
// inputs (LDS, odd chunk stride between lanes: the 16 lanes of a b128 lane
// group hit 16 different bank quads).  The chunks slab k+1 adds are loaded
// into registers during slab k-1 (coalesced: 16 lanes per column) and
// written to ring slots slab k does not read after slab k's compute (the
// launcher checks the ring holds slab k's window plus slab k+1's new chunks
// for every slab alignment); one barrier per slab publishes them.  Results
// go through an LDS tile [segment][slab output] and out as contiguous rows.
//
// Exactness: the pair table holds zero taps outside each output's window, so
// a sum over whole 4-chunk blocks adds exactly +0 beyond the reference's C
// terms (order unchanged) whenever the inputs there are finite; a lane whose
// result is not finite is recomputed term by term (sw_exact), so an Inf/NaN
// outside an output's window cannot reach it.
#include <cstdint>
#include <cstdlib>
#include <utility>

#include "sdr_common.hpp"

#pragma clang fp contract(off)

namespace sdr {
namespace {

constexpr int kSwWaves = 16;
constexpr int kSwThreads = 64 * kSwWaves;
constexpr int kSwRingC = 128;                // 16-B chunks per lane ring (power of 2)
constexpr int kSwStride = 4 * kSwRingC + 4;  // floats between lane rings (odd chunk count)
constexpr int kSwMaxL = 1024;                // phase table entries in LDS
constexpr int kSwOut = 36;
constexpr int kSwLd = 3;                     // staging loads per thread per slab (16 x 3 = 48 chunks per column)                   // floats per segment row of the output tile (16-B rows)

typedef float f4v __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const f4v lds_f4;
typedef __attribute__((address_space(4))) const f4v cst_f4;  // uniform address: scalar loads

struct SwArgs {
  const float* x;
  long long n, x_stride;
  const float* hs;  // [4][L][NCP*4] padded shifted rows (build_sw_taps)
  int up, down;
  float* state;
  int ns;
  float* y;
  long long y_stride, ny;
  int K;      // columns per lane segment
  int nseg;   // segments per stream
  int nlanes; // nstreams * nseg
  int nsub;   // units (workgroups) per lane group along the outputs
  int osub;   // outputs per unit, a multiple of SL
  int SL;     // outputs per slab (even, <= 2*kSwWaves)
  int ablate; // timing only: 1 = no staging, 2 = no arithmetic, 3 = no output stores
};

// Output offset r inside a segment as (r div L, r mod L), advanced without
// dividing (uniform scalar arithmetic).
struct RPos {
  int d, m;
};
__device__ __forceinline__ RPos radv(RPos p, int by, int up) {
  p.m += by;
  while (p.m >= up) {
    p.m -= up;
    ++p.d;
  }
  return p;
}

template <int CMAX>
struct SwGeo {
  static constexpr int base0 = -(((CMAX - 1) + 3) / 4 * 4);  // ring coordinate origin (multiple of 4)
  static constexpr int NC = (CMAX + 6) / 4;                  // chunks per shifted row
};

// Segment of ring column cl: stream, input offset of its first column.
struct Seg {
  int s;
  long long pos0;
  bool ok;
};
__device__ __forceinline__ Seg seg_of(const SwArgs& a, int gl) {
  Seg g;
  g.ok = gl < a.nlanes;
  const int gg = g.ok ? gl : 0;
  g.s = gg / a.nseg;
  g.pos0 = (long long)(gg - g.s * a.nseg) * a.K * a.down;
  return g;
}

template <int CMAX>
struct SwPipe {
  static constexpr int NC = SwGeo<CMAX>::NC;         // chunks a window touches, at most
  static constexpr int DMAX = 4;                      // newest-chunk distance of a pair (host-checked)
  static constexpr int NB = (3 + DMAX + NC - 1) / 4 + 1;  // blocks of 4 chunks per pair, at most
  static constexpr int ROW = 32 * (NB + 2);           // floats per pair-table row (+2 blocks of zeros:
                                                      // the loop prefetches one block past the last)
};

// Pair table: row phi serves the outputs r (phase phi) and r + 1 of any
// column: float pair k = (tap of a at index ia + k, tap of b at ib + k), 0
// where the index is outside [0, CMAX), ia / ib = the tap index of element 3
// of the pair's first block's first chunk (so element k of the block walk
// meets pair k).  Everything it depends on is a function of phi (column
// shifts are multiples of M = 0 mod 4).
template <int CMAX>
__device__ __forceinline__ void sw_pair_geom(int phi, int up, int down, int& ia, int& ib, int& pa, int& pb) {
  constexpr int base0 = SwGeo<CMAX>::base0;
  const long long qa = (long long)phi * down / up, qb = (long long)(phi + 1) * down / up;
  const int ea = (int)qa - base0, eb = (int)qb - base0;
  const int cb0 = (eb >> 2) | 3;
  ia = 4 * ((ea >> 2) - cb0) + (ea & 3) - 3;
  ib = 4 * ((eb >> 2) - cb0) + (eb & 3) - 3;
  pa = (int)((long long)phi * down % up);
  pb = (int)((long long)(phi + 1) * down % up);
}

template <int CMAX>
__global__ __launch_bounds__(kWG) void build_sw_pairs(const float* __restrict__ h, int up, int down,
                                                      float* __restrict__ table) {
  constexpr int ROW = SwPipe<CMAX>::ROW;
  const long long idx = (long long)blockIdx.x * kWG + threadIdx.x;  // (phi, k)
  if (idx >= (long long)up * (ROW / 2)) return;
  const int phi = (int)(idx / (ROW / 2)), k = (int)(idx % (ROW / 2));
  int ia, ib, pa, pb;
  sw_pair_geom<CMAX>(phi, up, down, ia, ib, pa, pb);
  const int i = ia + k, j = ib + k;
  table[2 * idx] = (i >= 0 && i < CMAX) ? h[pa + (long long)i * up] : 0.0f;
  table[2 * idx + 1] = (j >= 0 && j < CMAX) ? h[pb + (long long)j * up] : 0.0f;
}

// The exact sum of one output, term by term (only for a lane whose fast
// result is not finite: there a zero tap may have met an Inf/NaN input
// outside the output's window).  X = 0: output a, 1: output b.
template <int CMAX>
__device__ __forceinline__ float sw_exact(lds_f4* lr, const float* tab, int cb0, int nb, int i0, int X) {
  float acc = 0.0f;
  for (int k = 0; k < 16 * nb; ++k) {
    const int i = i0 + k;
    if (i < 0 || i >= CMAX) continue;
    const int n = k >> 4, j = (k >> 2) & 3, e = 3 - (k & 3);
    const f4v xv = lr[(cb0 - 4 * n - j) & (kSwRingC - 1)];
    const float x = e == 0 ? xv.x : e == 1 ? xv.y : e == 2 ? xv.z : xv.w;
    acc = acc + tab[2 * k + X] * x;
  }
  return acc;
}

template <int CMAX>
__global__ __launch_bounds__(kSwThreads, 1) void resample_sw(SwArgs a) {
  __shared__ __attribute__((aligned(16))) float ring[64 * kSwStride];
  __shared__ int qoff[kSwMaxL];  // floor(phi*M/L)
  // a slab's results [segment][output], written out coalesced after the next
  // barrier (two buffers: slab parity)
  __shared__ __attribute__((aligned(16))) float obuf[2][64 * kSwOut];
  constexpr int base0 = SwGeo<CMAX>::base0;
  constexpr int NC = SwGeo<CMAX>::NC;
  constexpr int ROW = SwPipe<CMAX>::ROW;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), ln = threadIdx.x & 63;
  const int lg = (int)blockIdx.x / a.nsub, sub = (int)blockIdx.x - lg * a.nsub;
  const int olen = a.K * a.up;  // outputs per segment
  const int o0 = sub * a.osub;
  const int o1 = min(o0 + a.osub, olen);
  const int L = a.up, M = a.down;
  for (int phi = threadIdx.x; phi < L; phi += kSwThreads)
    qoff[phi] = (int)(((unsigned)phi * (unsigned)M) / (unsigned)L);  // < 2^31 (sw_shape_ok)
  // ring chunks a block walk reads below a slab's window hold earlier inputs
  // of the lane (finite) or, before the first slab, these zeros -- never
  // stale LDS that could send a lane down the term-by-term path
  for (int i = threadIdx.x; i < 64 * kSwStride / 4; i += kSwThreads)
    reinterpret_cast<float4*>(ring)[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  // output tile writer: thread t stores outputs 2(t%16), +1 of segment t/16
  // of the tile (consecutive threads: consecutive 8 B of one segment's row)
  const int wl = threadIdx.x >> 4, we = 2 * (threadIdx.x & 15);
  const Seg wseg = seg_of(a, lg * 64 + wl);
  const long long wjb = wseg.ok ? (wseg.pos0 / M) * L : 0;
  const long long wlim = wseg.ok ? min((long long)olen, a.ny - wjb) : 0;  // r < wlim is a real output
  float* wys = a.y + (long long)wseg.s * a.y_stride + wjb;
  lds_f4* lr = (lds_f4*)(ring + ln * kSwStride);
  __syncthreads();
  auto qof = [&](RPos p) { return p.d * M + qoff[p.m]; };
  // slab k covers outputs r0 .. r0 + SL - 1; its window is ring chunks [lo, hi)
  RPos r0 = radv(RPos{0, 0}, o0, L);
  auto lo_of = [&](RPos p) { return (qof(p) - (CMAX - 1) - base0) >> 2; };
  auto hi_of = [&](RPos p) { return ((qof(radv(p, a.SL - 1, L)) - base0) >> 2) + 1; };
  // Staging by registers: thread t serves ring column sc = t / 16 and
  // chunks c0 + sj + 16 i (i < kSwLd) of each new range [c0, c1): one slab's
  // new chunks are loaded right after the barrier that starts the previous
  // slab's compute and written to the ring after that compute (16
  // consecutive chunks of one column per 16 lanes: coalesced 256-B runs).
  const int sc = threadIdx.x >> 4, sj = threadIdx.x & 15;
  const Seg sseg = seg_of(a, lg * 64 + sc);
  const long long sbase = sseg.pos0 + base0;  // input position of ring chunk 0 of column sc
  const float* sx = a.x + (long long)sseg.s * a.x_stride;
  const float* sst = a.state + (long long)sseg.s * a.ns;
  float* scol = ring + sc * kSwStride;
  const long long pos0_max = (long long)(a.nseg - 1) * a.K * M;
  // chunk c of column sc (positions outside [0, n): the carried state before
  // the block, zeros past it)
  auto chunk_at = [&](int c, bool interior) -> float4 {
    const long long gp = sbase + 4LL * c;
    if (interior) return *reinterpret_cast<const float4*>(sx + gp);
    float w4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long long q = gp + r;
      w4[r] = q >= 0 ? (q < a.n ? sx[q] : 0.0f) : (q >= -a.ns ? sst[a.ns + q] : 0.0f);
    }
    return make_float4(w4[0], w4[1], w4[2], w4[3]);
  };
  auto interior_of = [&](int c0, int c1) { return base0 + 4LL * c0 >= 0 && pos0_max + base0 + 4LL * c1 <= a.n; };
  float4 sv[kSwLd];
  // (interior and edge paths apart: sharing registers between them made the
  // compiler wait for each load before issuing the next)
  auto stage_load = [&](int c0, int c1) {
    if (interior_of(c0, c1)) {
#pragma unroll
      for (int i = 0; i < kSwLd; ++i) {
        const int c = c0 + sj + 16 * i;
        if (sseg.ok && c < c1) sv[i] = *reinterpret_cast<const float4*>(sx + sbase + 4LL * c);
      }
    } else {
#pragma unroll
      for (int i = 0; i < kSwLd; ++i) {
        const int c = c0 + sj + 16 * i;
        if (sseg.ok && c < c1) sv[i] = chunk_at(c, false);
      }
    }
  };
  auto stage_store = [&](int c0, int c1) {
#pragma unroll
    for (int i = 0; i < kSwLd; ++i) {
      const int c = c0 + sj + 16 * i;
      if (sseg.ok && c < c1) *reinterpret_cast<float4*>(scol + 4 * (c & (kSwRingC - 1))) = sv[i];
    }
  };
  int hi = hi_of(r0);
  if (a.ablate != 1) {
    // the first window, synchronously
    const int c0 = lo_of(r0);
    const bool in = interior_of(c0, hi);
    for (int c = c0 + sj; c < hi; c += 16)
      if (sseg.ok) *reinterpret_cast<float4*>(scol + 4 * (c & (kSwRingC - 1))) = chunk_at(c, in);
  }
  // slab 1's new chunks into the staging registers: from here on, the chunks
  // slab k+1 adds are written to the ring after slab k's compute, and the
  // chunks of slab k+2 loaded right after (registers carry them across slab
  // k+1's compute, which hides their latency)
  int hi1 = hi;
  if (o1 - o0 > a.SL) {
    hi1 = hi_of(radv(r0, a.SL, L));
    if (a.ablate != 1 && hi1 > hi) stage_load(hi, hi1);
  }
  __syncthreads();
  // the unit holding each stream's first outputs is the only reader of its
  // carried state, now staged: state <- last ns inputs (src/filter.cpp:169)
  if (o0 == 0) {
    for (int idx = threadIdx.x; idx < 64 * a.ns; idx += kSwThreads) {
      const int cl = idx / a.ns, i = idx - cl * a.ns;
      const Seg g = seg_of(a, lg * 64 + cl);
      if (g.ok && g.pos0 == 0)
        a.state[(long long)g.s * a.ns + i] = a.x[(long long)g.s * a.x_stride + a.n - a.ns + i];
    }
  }
  // slab k's results go out at the start of slab k+1, after the barrier
  // that makes the tile complete, so the next drain never waits on them
  auto flush = [&](int kk) {
    if (a.ablate == 3) return;
    const int r = o0 + kk * a.SL + we;  // outputs r, r + 1 of segment wl
    const float* t = obuf[kk & 1] + wl * kSwOut + we;
    if (we < a.SL && r < o1) {
      const bool two = r + 1 < o1 && r + 1 < wlim;
      float* dst = wys + r;
      if (two && (reinterpret_cast<uintptr_t>(dst) & 7) == 0) {
        *reinterpret_cast<float2*>(dst) = make_float2(t[0], t[1]);
      } else {
        if (r < wlim) dst[0] = t[0];
        if (two) dst[1] = t[1];
      }
    }
  };
  const int nslab = (o1 - o0 + a.SL - 1) / a.SL;
  const int ra_off = 2 * wv;
  typedef float f2v __attribute__((ext_vector_type(2)));
  for (int k = 0; k < nslab; ++k) {
    const bool more = k + 1 < nslab;
    const RPos rn = radv(r0, a.SL, L);
    const int nhi = hi1;  // slab k+1's window top, its chunks [hi, nhi) are in the staging registers
    if (k > 0) flush(k - 1);
    const int ra = o0 + k * a.SL + ra_off;
    if (ra_off < a.SL && ra < o1 && a.ablate != 2) {
      const RPos pa_ = radv(r0, ra_off, L), pb_ = radv(pa_, 1, L);
      const int ea = qof(pa_) - base0, eb = qof(pb_) - base0;
      const int cta = ea >> 2;
      const int top = (eb >> 2) | 3;                  // top chunk of the first block
      const int nb = ((top - (cta - (NC - 1))) >> 2) + 1;
      const float* tab = a.hs + (long long)pa_.m * ROW;
      const float* ntab = a.hs + (long long)radv(rn, ra_off, L).m * ROW;  // next slab's row (cache warm-up)
      const auto vb = lr;
      f2v acc = {0.0f, 0.0f};
#include "resample_sw_pair.inc"
      float pa = acc.x, pb = acc.y;
      if (!__builtin_isfinite(pa) && a.ablate != 1) pa = sw_exact<CMAX>(lr, tab, top, nb, 4 * (cta - top) + (ea & 3) - 3, 0);
      if (!__builtin_isfinite(pb) && a.ablate != 1) pb = sw_exact<CMAX>(lr, tab, top, nb, 4 * ((eb >> 2) - top) + (eb & 3) - 3, 1);
      *reinterpret_cast<float2*>(obuf[k & 1] + ln * kSwOut + ra_off) = make_float2(pa, pb);
    }
    if (more && a.ablate != 1 && nhi > hi) stage_store(hi, nhi);
    if (k + 2 < nslab) {
      hi1 = hi_of(radv(rn, a.SL, L));
      if (a.ablate != 1 && hi1 > nhi) stage_load(nhi, hi1);
    }
    hi = nhi;
    r0 = rn;
    __syncthreads();
  }
  if (nslab > 0) flush(nslab - 1);
}

// Opt-in (SDR_RESAMPLE_SW=1): measured 5-10 % slower than resample_lp on
// cfg3; read per launch so a test can switch it.
bool sw_enabled() {
  const char* e = std::getenv("SDR_RESAMPLE_SW");
  return e && std::atoi(e) != 0;
}

// The ring must hold slab k's window and slab k+1's new chunks at once, for
// every alignment of a slab start within the period L (q(r+L) = q(r) + M).
// and a slab's new chunks must fit the staging registers (kSwLd per thread,
// 16 threads per column)
template <int CMAX>
bool sw_ring_fits(int up, int down, int SL) {
  constexpr int base0 = SwGeo<CMAX>::base0;
  auto q = [&](long long r) { return (long long)(r / up) * down + (r % up) * (long long)down / up; };
  for (int r0 = 0; r0 < up; ++r0) {
    const long long lo = (q(r0) - (CMAX - 1) - base0) >> 2;
    const long long hi1 = ((q(r0 + SL - 1) - base0) >> 2) + 1;
    const long long hi2 = ((q(r0 + 2LL * SL - 1) - base0) >> 2) + 1;
    if (hi2 - lo > kSwRingC || hi2 - hi1 > 16 * kSwLd) return false;
  }
  return true;
}

template <int CMAX>
bool launch_sw_t(int up, int down, const float* x, long long n, int nstreams, long long x_stride,
                 const float* hs, float* state, int ns, float* y, long long y_stride, long long ny, hipStream_t st,
                 hipError_t* err) {
  int SL = 2 * kSwWaves;
  while (SL >= 2 && !sw_ring_fits<CMAX>(up, down, SL)) SL -= 2;
  if (SL < 2) return false;
  // the pair pipeline's block count assumes the two outputs' newest chunks
  // are at most DMAX apart
  {
    constexpr int base0 = SwGeo<CMAX>::base0;
    for (int phi = 0; phi < up; ++phi) {
      const long long qa = (long long)phi * down / up, qb = (long long)(phi + 1) * down / up;
      if (((qb - base0) >> 2) - ((qa - base0) >> 2) > SwPipe<CMAX>::DMAX) return false;
    }
  }
  const long long np = (ny + up - 1) / up;  // columns per stream
  // lane segments: whole streams when there are enough of them to fill the
  // lanes, else runs of K columns
  long long nseg = 1;
  if (nstreams < 64) {
    nseg = (64 + nstreams - 1) / nstreams;
    if (nseg > np) nseg = np;
  }
  long long K = (np + nseg - 1) / nseg;
  // a segment after a stream's first reaches back into the previous segment,
  // never into the carried state (only the first unit of a stream reads it)
  const long long kmin = (CMAX + 3 + down - 1) / down;
  if (K < kmin) K = kmin;
  nseg = (np + K - 1) / K;
  const long long nlanes = nseg * nstreams;
  const long long olen = K * up;
  if (nlanes > (1LL << 30) || (olen + 4LL * SL + up) * (long long)down >= (1LL << 30)) return false;
  const long long nlg = (nlanes + 63) / 64;
  // units along the outputs: about one workgroup per CU in all; every unit
  // but the first starts past the carried state's reach
  const int ncu = device_cu_count();
  long long nsub = (ncu + nlg - 1) / nlg;
  const long long min_o = 4LL * SL;  // at least four slabs per unit
  if (nsub > olen / min_o) nsub = olen / min_o;
  if (nsub < 1) nsub = 1;
  long long osub = (olen + nsub - 1) / nsub;
  osub = (osub + SL - 1) / SL * SL;
  auto q = [&](long long r) { return (r / up) * down + (r % up) * down / up; };
  while (osub < olen && q(osub) - (CMAX - 1) < 4) osub += SL;
  nsub = (olen + osub - 1) / osub;
  if (nlg * nsub > 0x7fffffffLL) return false;
  SwArgs a;
  a.x = x;
  a.n = n;
  a.x_stride = x_stride;
  a.hs = hs;
  a.up = up;
  a.down = down;
  a.state = state;
  a.ns = ns;
  a.y = y;
  a.y_stride = y_stride;
  a.ny = ny;
  a.K = (int)K;
  a.nseg = (int)nseg;
  a.nlanes = (int)nlanes;
  a.nsub = (int)nsub;
  a.osub = (int)osub;
  a.SL = SL;
  static const int ablate = env_int("SDR_ABLATE", 0);
  a.ablate = ablate;
  hipLaunchKernelGGL(resample_sw<CMAX>, dim3((unsigned)(nlg * nsub)), dim3(kSwThreads), 0, st, a);
  *err = hipGetLastError();
  return true;
}

}  // namespace

// Shapes: T = C*L with C in {101, 151}, M % 16 == 0 (a column moves the
// window by M/4 chunks, a multiple of the 4-chunk block: the pair table row,
// the alignment A and the block grid depend on the phase only), L <=
// kSwMaxL, L*M < 2^31.
bool sw_shape_ok(int up, int down, int ntaps) {
  const int cmax = (ntaps + up - 1) / up;
  if (!sw_enabled()) return false;
  return up >= 2 && up <= kSwMaxL && ntaps == cmax * up && (cmax == 151 || cmax == 101) && down % 16 == 0 &&
         (long long)up * down < (1LL << 31);
}

// ... and 16-B aligned rows.  false = not covered, nothing launched.
bool sw_covers(int up, int down, int ntaps, const float* x, int nstreams, long long x_stride) {
  if (!sw_shape_ok(up, down, ntaps)) return false;
  return !((reinterpret_cast<uintptr_t>(x) & 15) || (nstreams > 1 && x_stride % 4));
}

size_t sw_table_floats(int up, int ntaps) {
  const int cmax = (ntaps + up - 1) / up;
  return (size_t)up * (cmax == 151 ? SwPipe<151>::ROW : SwPipe<101>::ROW);
}

hipError_t build_sw_table(int up, int down, const float* h, int ntaps, float* table, hipStream_t st) {
  const int cmax = (ntaps + up - 1) / up;
  const long long tot = (long long)sw_table_floats(up, ntaps) / 2;
  const dim3 grid((unsigned)((tot + kWG - 1) / kWG));
  if (cmax == 151)
    hipLaunchKernelGGL(build_sw_pairs<151>, grid, dim3(kWG), 0, st, h, up, down, table);
  else
    hipLaunchKernelGGL(build_sw_pairs<101>, grid, dim3(kWG), 0, st, h, up, down, table);
  return hipGetLastError();
}

bool launch_resample_sw(int up, int down, const float* x, long long n, int nstreams, long long x_stride,
                        int ntaps, const float* table, float* state, int ns, float* y, long long y_stride,
                        long long ny, hipStream_t st, hipError_t* err) {
  const int cmax = (ntaps + up - 1) / up;
  if (cmax == 151)
    return launch_sw_t<151>(up, down, x, n, nstreams, x_stride, table, state, ns, y, y_stride, ny, st, err);
  return launch_sw_t<101>(up, down, x, n, nstreams, x_stride, table, state, ns, y, y_stride, ny, st, err);
}

}  // namespace sdr
