// fir_long.hip -- long FIRs without decimation: the reference's
// blockConvolveFIR (src/filter.cpp:66-83) for T a multiple of 32 (cfg5:
// T = 1024 on 1 M-sample I and Q blocks).
//
// Same arithmetic contract as fir_tile.hip: y[m] = sum over k = 0..T-1, in
// order, of separately rounded h[k]*x~[m-k] added to an accumulator that
// starts at 0.0f; x~ reads the carried state before the block.
//
// Structure.  A workgroup of NW waves takes 64*R*NW consecutive outputs of
// one stream; its input image (the outputs' span plus a T-1 halo) is
// staged in LDS once with 16-B loads.  Lane l of wave w owns R consecutive
// outputs and walks its window in passes of KP = 32 taps: the pass's taps
// are SGPR operands (one batch of scalar loads, one wait per pass) and its
// inputs are (32 + R)/4 + 1 16-B LDS reads (lane stride R floats:
// conflict-free).  Every pass has the same shape, shifted by 8 chunks, so
// the pass body is unrolled once and looped at run time.  At R = 4 a pass
// is 256 multiplies/adds per lane against 10 LDS reads: VALU-bound, the
// bound of this config (4,096 FLOP per IQ pair).
#include <algorithm>

#include "sdr_common.hpp"

#pragma clang fp contract(off)

namespace sdr {
namespace {

constexpr int kLongKP = 32;  // taps per pass
constexpr int kLongR = 4;    // outputs per lane
constexpr int kLongNW = 4;   // waves per workgroup

struct LongArgs {
  const float* x;
  long long n, x_stride;
  const float* h;
  int ntaps;  // multiple of kLongKP
  const float* state;
  int ns;
  float* y;
  long long y_stride;
  int tiles_per_stream;
  int halo;   // roundup4(ntaps - 1)
  int img;    // LDS floats per workgroup image
  float* commit;  // = state when only a stream's first workgroup reads the state (halo <= OUT_WG): it
                  // writes the new state itself; nullptr: long_commit runs after the kernel
};

// VTAP = 1: the taps are staged in LDS behind the image and each pass's 32
// are read into VGPRs by 8 wave-uniform (broadcast) ds_read_b128, so the
// multiplies take no SGPR operand; VTAP = 0: SGPR taps (SDR_LONG_VTAP=0).
template <int VTAP>
__global__ __launch_bounds__(64 * kLongNW) void fir_long(LongArgs a) {
  extern __shared__ __attribute__((aligned(16))) float img[];
  constexpr int R = kLongR, KP = kLongKP, NTH = 64 * kLongNW;
  constexpr int OUT_WG = 64 * R * kLongNW;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int s = blockIdx.x / a.tiles_per_stream;
  const int tile = blockIdx.x - s * a.tiles_per_stream;
  const long long m0 = (long long)tile * OUT_WG;      // first output of the workgroup
  const long long pb = m0 - a.halo;                   // stream position of image element 0
  const float* xs = a.x + (long long)s * a.x_stride;
  const float* st = a.state + (long long)s * a.ns;

  // ---- stage [pb, pb + img): 16-B loads, element-wise at the block edges
  const int n4 = a.img >> 2;
  for (int c = tid; c < n4; c += NTH) {
    const long long p = pb + 4LL * c;
    float4 v;
    if (p >= 0 && p + 4 <= a.n) {
      v = *reinterpret_cast<const float4*>(xs + p);
    } else {
      float w[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long long q = p + r;
        w[r] = q >= 0 ? (q < a.n ? xs[q] : 0.0f) : (q >= -a.ns ? st[a.ns + q] : 0.0f);
      }
      v = make_float4(w[0], w[1], w[2], w[3]);
    }
    *reinterpret_cast<float4*>(img + 4 * c) = v;
  }
  float* hl = img + a.img;  // the taps behind the image (a.img is a multiple of 4)
  if constexpr (VTAP) {
    for (int c = tid; c < (a.ntaps >> 2); c += NTH)
      *reinterpret_cast<float4*>(hl + 4 * c) = *reinterpret_cast<const float4*>(a.h + 4 * c);
  }
  __syncthreads();

  // ---- passes.  Lane window: output r of this lane sits at image index
  // lb + halo + r; tap k reads image index lb + halo + r - k.  Pass P covers
  // k in [32P, 32P+32): indices lb + halo - 32P - 32 + (32 + r - kk), kk = k - 32P.
  const int lb = (wave * 64 + lane) * R;
  using hconst = const __attribute__((address_space(4))) float*;
  const hconst hc = (hconst)a.h;
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0f;
  const int npass = a.ntaps / KP;
  constexpr int NC = (KP + R - 1) / 4 + 1;  // chunks per pass (relative indices 1 .. KP+R-1)
  for (int P = 0; P < npass; ++P) {
    float hs[KP];
    if constexpr (VTAP) {
#pragma unroll
      for (int i = 0; i < KP; i += 4) {
        const float4 t = *reinterpret_cast<const float4*>(hl + P * KP + i);
        hs[i] = t.x;
        hs[i + 1] = t.y;
        hs[i + 2] = t.z;
        hs[i + 3] = t.w;
      }
    } else {
#pragma unroll
      for (int i = 0; i < KP; ++i) hs[i] = hc[P * KP + i];
#pragma unroll
      for (int i = 0; i < KP; ++i) asm volatile("" : "+s"(hs[i]));
    }
    const float* base = img + lb + a.halo - KP * (P + 1);  // relative index 0, 16-B aligned
    float4 q = *reinterpret_cast<const float4*>(base + 4 * (NC - 1));
#pragma unroll
    for (int c = NC - 1; c >= 0; --c) {
      float4 nx = q;
      if (c > 0) nx = *reinterpret_cast<const float4*>(base + 4 * (c - 1));
      const float e[4] = {q.x, q.y, q.z, q.w};
#pragma unroll
      for (int j = 3; j >= 0; --j) {
        const int rel = 4 * c + j;  // = KP + r - kk
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int kk = KP + r - rel;
          if (kk >= 0 && kk < KP) acc[r] = acc[r] + hs[kk] * e[j];
        }
      }
      q = nx;
#pragma unroll
      for (int r = 0; r < R; ++r) asm volatile("" : "+v"(acc[r]));
      __builtin_amdgcn_sched_barrier(0);
    }
  }

  const long long m = m0 + lb;
  float* ys = a.y + (long long)s * a.y_stride;
  if (m + R <= a.n && ((reinterpret_cast<uintptr_t>(ys + m) & 15) == 0)) {
    *reinterpret_cast<float4*>(ys + m) = make_float4(acc[0], acc[1], acc[2], acc[3]);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (m + r < a.n) ys[m + r] = acc[r];
  }
  // state <- the last ns inputs (src/filter.cpp:82): this workgroup's image
  // holds every old-state value any workgroup reads (staged before the
  // barrier above), so the state is free to rewrite
  if (a.commit != nullptr && tile == 0) {
    float* nst = a.commit + (long long)s * a.ns;
    for (int i = tid; i < a.ns; i += NTH) nst[i] = xs[a.n - a.ns + i];
  }
}

// state <- last ns inputs, after every reader of the old state is done.
__global__ __launch_bounds__(kWG) void long_commit(const float* __restrict__ x, long long n, long long x_stride,
                                                   float* state, int ns) {
  const int s = blockIdx.y;
  const int i = blockIdx.x * kWG + threadIdx.x;
  if (i >= ns) return;
  state[(long long)s * ns + i] = x[(long long)s * x_stride + n - ns + i];
}

}  // namespace

bool fir_long_ok(int D, int ntaps, int ns, long long n) {
  return D == 1 && ntaps >= 2 * kLongKP && ntaps % kLongKP == 0 && ns >= ntaps - 1 && n >= ns &&
         ntaps <= 8192;
}

hipError_t launch_fir_long(const FirLaunch& f, const float* h, hipStream_t st) {
  LongArgs a;
  a.x = f.x0;
  a.n = f.n;
  a.x_stride = f.x_stride;
  a.h = h;
  a.ntaps = f.ntaps;
  a.state = f.state0;
  a.ns = f.ns;
  a.y = f.y0;
  a.y_stride = f.y_stride;
  constexpr int OUT_WG = 64 * kLongR * kLongNW;
  a.tiles_per_stream = (int)((f.n + OUT_WG - 1) / OUT_WG);
  a.halo = (f.ntaps - 1 + 3) / 4 * 4;
  a.img = a.halo + OUT_WG + 4;
  // tile 1 starts at OUT_WG - halo: with halo <= OUT_WG (T <= 1025) only tile 0
  // reads the state, and it commits the new one in the same launch
  const bool in_kernel = a.halo <= OUT_WG && sw(kSwLongCommit) != 0;
  a.commit = in_kernel && f.ns > 0 ? f.state0 : nullptr;
  const long long blocks = (long long)a.tiles_per_stream * f.nstreams;
  if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
  // LDS-staged taps (switch SDR_LONG_VTAP, measured at T = 1024) need 16-B
  // aligned taps (ntaps is a multiple of 32) and ntaps*4 more LDS per
  // workgroup; where that extra LDS would cut the workgroups a CU can hold
  // below both 8 (four waves per SIMD) and the SGPR kernel's count -- long
  // taps, e.g. T = 8192: 69.7 vs 36.9 KiB, 2 vs 4 per CU -- the SGPR-tap
  // kernel runs.  Same bits either way.
  const size_t lds_s = (size_t)a.img * sizeof(float), lds_v = lds_s + (size_t)f.ntaps * sizeof(float);
  const size_t lds_cu = (size_t)device_lds_bytes();
  if (lds_s > lds_cu) return hipErrorInvalidConfiguration;
  const bool vtap = sw(kSwLongVtap) != 0 && (reinterpret_cast<uintptr_t>(h) & 15) == 0 && lds_v <= lds_cu &&
                    lds_cu / lds_v >= std::min<size_t>(8, lds_cu / lds_s);
  if (vtap)
    hipLaunchKernelGGL(fir_long<1>, dim3((unsigned)blocks), dim3(64 * kLongNW), lds_v, st, a);
  else
    hipLaunchKernelGGL(fir_long<0>, dim3((unsigned)blocks), dim3(64 * kLongNW), lds_s, st, a);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess || f.ns <= 0 || a.commit != nullptr) return e;
  hipLaunchKernelGGL(long_commit, dim3((f.ns + kWG - 1) / kWG, (unsigned)f.nstreams), dim3(kWG), 0, st, f.x0, f.n,
                     f.x_stride, f.state0, f.ns);
  return hipGetLastError();
}


// ------------------------------------------------------------------ fp16 --
// BASELINE config 5's fp16 arm: the same long FIR on fp16 storage (inputs,
// state and taps rounded to fp16), fp32 accumulation with
// v_dot2_f32_f16 -- two taps per instruction, a quarter of the exact
// path's instruction count.  NOT bit-exact by construction (fp16 operands,
// fused dot): its error against the fp32 reference is what the tolerance
// sweep reports (tests/test_gpu_parity.py, bench.py --config cfg5h).
//
// Term h[k]*x[i-k] of the output at image index i, grouped by fp16 pair
// W = (x[2W], x[2W+1]): d = i - 2W, pair taps (h[d], h[d-1]) with h[-1] =
// h[T] = 0 -- the table hp2[d], d = 0..T, packed half2 (lo, hi).
namespace {

typedef _Float16 half2_t __attribute__((ext_vector_type(2)));
constexpr int kLongRH = 8;  // outputs per lane (keeps each lane's pair window 16-B aligned)

struct LongHArgs {
  const _Float16* x;
  long long n, x_stride;       // in halves
  const uint32_t* hp2;          // T+1 packed pairs, padded to a multiple of 32
  int ntaps;
  const _Float16* state;
  int ns;
  float* y;
  long long y_stride;
  int tiles_per_stream;
  int halo;   // roundup8(ntaps): image halves before the first output
  int img;    // image halves (multiple of 8)
};

// The tap pairs are SGPR operands of the dot2 (one scalar batch per pass).
// (VGPR pairs read from LDS by broadcast ds_read_b128 were slower: 0.0544 vs
// 0.0425 ms, profiles/r04a/ab_vtap.txt -- 8 reads per pass on top of the
// inputs' 10 saturate the LDS at 16 waves per CU.)
__global__ __launch_bounds__(64 * kLongNW) void fir_long_h(LongHArgs a) {
  extern __shared__ __attribute__((aligned(16))) uint32_t imgw[];  // image as packed pairs
  constexpr int R = kLongRH, NTH = 64 * kLongNW, KP = 32;  // KP tap pairs (d values) per pass
  constexpr int OUT_WG = 64 * R * kLongNW;
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int s = blockIdx.x / a.tiles_per_stream;
  const int tile = blockIdx.x - s * a.tiles_per_stream;
  const long long m0 = (long long)tile * OUT_WG;
  const long long pb = m0 - a.halo;  // multiple of 8
  const _Float16* xs = a.x + (long long)s * a.x_stride;
  const _Float16* st = a.state + (long long)s * a.ns;
  _Float16* imgh = reinterpret_cast<_Float16*>(imgw);
  const int n8 = a.img >> 3;  // 16-B chunks
  for (int c = tid; c < n8; c += NTH) {
    const long long p = pb + 8LL * c;
    if (p >= 0 && p + 8 <= a.n) {
      *reinterpret_cast<uint4*>(imgh + 8 * c) = *reinterpret_cast<const uint4*>(xs + p);
    } else {
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const long long q = p + r;
        imgh[8 * c + r] = q >= 0 ? (q < a.n ? xs[q] : (_Float16)0) : (q >= -a.ns ? st[a.ns + q] : (_Float16)0);
      }
    }
  }
  __syncthreads();

  // output r of this lane: image half index i_r = I0 + r, I0 = lb + halo
  const int lb = (wave * 64 + lane) * R;
  const int I0 = lb + a.halo;                      // multiple of 8: pair index I0/2 16-B aligned
  using hconst = const __attribute__((address_space(4))) uint32_t*;
  const hconst hc = (hconst)a.hp2;
  float acc[R];
#pragma unroll
  for (int r = 0; r < R; ++r) acc[r] = 0.0f;
  const int npass = (a.ntaps + 1 + KP - 1) / KP;  // d = 0..T
  for (int P = 0; P < npass; ++P) {
    uint32_t hs[KP];
#pragma unroll
    for (int i = 0; i < KP; ++i) hs[i] = hc[P * KP + i];
#pragma unroll
    for (int i = 0; i < KP; ++i) asm volatile("" : "+s"(hs[i]));
    // pair W for (r, d): 2W = I0 + r - d, d = KP*P + dd.  Word index
    // W = I0/2 - KP*P/2 + (r - dd)/2 ranges over base + [-(KP/2), 1].
    const int wbase = (I0 >> 1) - (KP / 2) * P - (KP / 2);  // word of relative index 0
    // relative word u = (r - dd)/2 + KP/2 in [0, KP/2 + 1]; read 4-word chunks
    constexpr int NU = KP / 2 + R / 2;  // u = (r - dd)/2 + KP/2 in [1, KP/2 + R/2 - 1]
    constexpr int NC = (NU + 3) / 4;
    // I0/2 and (KP/2)*(P+1) are multiples of 4: 16-B aligned chunks
    const uint32_t* base = imgw + wbase;
#pragma unroll
    for (int c = 0; c < NC; ++c) {
      const uint4 v = *reinterpret_cast<const uint4*>(base + 4 * c);
      const uint32_t wv[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
      for (int q = 0; q < 4; ++q) {
        const int u = 4 * c + q;
#pragma unroll
        for (int r = 0; r < R; ++r) {
          const int dd = r - 2 * (u - KP / 2);  // d - KP*P
          if (dd >= 0 && dd < KP) {
            half2_t xv = __builtin_bit_cast(half2_t, wv[q]);
            half2_t hv = __builtin_bit_cast(half2_t, hs[dd]);
            acc[r] = __builtin_amdgcn_fdot2(xv, hv, acc[r], false);
          }
        }
      }
    }
  }
  const long long m = m0 + lb;
  float* ys = a.y + (long long)s * a.y_stride;
  if (m + R <= a.n && ((reinterpret_cast<uintptr_t>(ys + m) & 15) == 0)) {
    *reinterpret_cast<float4*>(ys + m) = make_float4(acc[0], acc[1], acc[2], acc[3]);
    *reinterpret_cast<float4*>(ys + m + 4) = make_float4(acc[4], acc[5], acc[6], acc[7]);
  } else {
#pragma unroll
    for (int r = 0; r < R; ++r)
      if (m + r < a.n) ys[m + r] = acc[r];
  }
}

// ---- MFMA form (the default for T % 8 == 0): the FIR as a Toeplitz GEMM on
// v_mfma_f32_32x32x16_f16.  A 32x32 tile of outputs m = m0 + i + 32 j
// (i = row, j = column: 32 blocks of 32 consecutive outputs) is
//   D[i][j] = sum_t A[i][t] B[t][j],  A[i][t] = h[i + T - t]  (0 outside [0, T)),
//                                     B[t][j] = x~[m0 + 32 j + t - T],
// t = 0 .. KD-1, KD = roundup96(T + 31): 66 MFMAs per 1,024 outputs at T =
// 1024 (3 % of them on the band's zero corners).  B's fragment (lane: column
// j = l & 31, k-half h = l >> 5) is 8 consecutive inputs -- one 16-B LDS read
// from the staged input image (a 16-B pad per 64 B row keeps the 32 columns'
// reads, 64 B apart, on distinct banks); A's fragment is 8 consecutive
// reversed taps starting at 16 s + 8 h - i - 1, read 16-B aligned from one of
// eight copies of the reversed f16 taps, copy q shifted by q halves.
// Same operands as the dot2 kernel (fp16 x, state and taps), fp32
// accumulation inside the MFMA: the same tolerance contract.
// the default: cfg5h 0.0161-0.0163 vs 0.0427-0.0428 ms on the dot2 kernel
// (profiles/r04e/ab.txt); switch SDR_F16_MFMA=0 selects v_dot2
constexpr int kMfOut = 8192;                  // outputs per workgroup: 8 tiles of 1,024
// SDR_F16_TSTORE: the fp16 MFMA kernel's outputs transposed through LDS so
// each store instruction writes 1 KB contiguous instead of 32 B in each of 32
// rows: cfg5h 0.0076 vs 0.0078 ms, 3 of 3 pairs (profiles/r05d/ab_tstore.txt)
#ifndef SDR_F16_TSTORE
#define SDR_F16_TSTORE 1
#endif
constexpr int kMfOstRow = 36;  // floats per 32-output row of a transpose area (bank spread)
// (Round 5: the output stores non-temporal measured 0.0095 vs 0.0079 ms on
// cfg5h, profiles/r05c/ab_f16nt.txt; not kept.)

// SDR_F16_G: k-steps per fragment group of fir_long_mfma's MFMA loop (the
// next group's 2 G reads are issued before this group's MFMAs).  3 measured
// best: 2 / 4 / 6 gave cfg5h 0.0075-0.0077 vs 0.0071-0.0073 ms
// (profiles/r05i/ab_g.txt)
#ifndef SDR_F16_G
#define SDR_F16_G 3
#endif
constexpr int kMfG = SDR_F16_G;
constexpr int kMfMaxKd = (4096 + 31 + 32 * kMfG - 1) / (32 * kMfG) * (32 * kMfG);  // kd at T = 4096
static_assert((kMfMaxKd + 8 + 127) / 128 * 128 + 32 + 40 <= 4424, "reversed-tap staging covers the copies");

struct MfArgs {
  const _Float16* x;
  long long n, x_stride;  // halves
  const float* h;
  int ntaps, kd, lc;      // taps, K extent (multiple of 16), halves per tap copy
  _Float16* state;        // read by each stream's first workgroup, then rewritten by it
  int ns;
  float* y;
  long long y_stride;
  int wg_per_stream;
  int span;               // staged input halves per workgroup (kMfOut + kd - 32)
  int ablate;             // timing ablations only (SDR_ABLATE): 1 = one cached input chunk, 2 = no MFMA,
                          // 3 = no tap staging, 4 = no output stores, 7 = the head as interior, 14 = reversed grid
  int head_pre;           // the first workgroup's state loads in the first load batch (SDR_F16_HEAD, A/B)
  const _Float16* hplan;  // PLAN: the 8 tap copies (8 * lc halves) prebuilt by sdr_fir_f16_plan_create
  int ost;                // SDR_F16_TSTORE: LDS half offset of the per-wave output transpose areas
  unsigned long long* trace;  // timing builds (SDR_F16_TRACE): per-wave phase stamps, else null
};

// Timing builds only: wall-clock stamps (100 MHz) of each wave's phases,
// kMfTraceW per workgroup -- [k * 8 + wave], k = 0 entry, 1 after the staging
// barrier, 2 after the MFMA loop, 3 stores issued, 4 stores complete.
#ifdef SDR_TIMING_BUILD
constexpr int kMfTraceW = 40;
// stamps held in registers and stored together at the end (a store per
// stamp would be a vector-memory operation every later s_waitcnt vmcnt(0)
// of the kernel waits for)
#define MF_STAMP(k)                         \
  do {                                      \
    if (a.trace) mf_stamp[k] = wall_clock64(); \
  } while (0)
#define MF_STAMP_FLUSH()                                                                        \
  do {                                                                                          \
    if (a.trace && lane == 0)                                                                   \
      for (int k_ = 0; k_ < 5; ++k_) a.trace[(long long)blockIdx.x * kMfTraceW + 8 * k_ + wave] = mf_stamp[k_]; \
  } while (0)
#else
#define MF_STAMP(k) \
  do {              \
  } while (0)
#endif

__host__ __device__ __forceinline__ int mf_pad(int p) { return p + 8 * (p >> 5); }  // padded LDS half index
// Output row of the MFMA's row v (a permutation of 0..31 that keeps blocks of
// four rows, so each accumulator float4 is still 4 consecutive outputs): block
// b = v >> 2 goes to 2 (b & 3) + (b >> 2).  Row v's taps come from copy
// (-row-1) mod 8 at row >> 3 slots back; this order gives every lane group of
// a ds_read_b128 (both the guide's {0-3,12-15,20-27}-style groups and 16
// consecutive lanes) 16 distinct (row & 3, row >> 3) pairs = distinct banks.
__host__ __device__ __forceinline__ int mf_row(int v) { return 4 * (2 * ((v >> 2) & 3) + (v >> 4)) + (v & 3); }

// kMfWaves waves (4: one per SIMD, two tiles each; 8: two per SIMD, one tile each).
// PLAN: the tap copies come prebuilt (a tap plan, sdr_fir_f16_plan_*), brought
// into LDS by LDS-DMA beside the image loads -- no f32 tap loads, no reversed
// row, no copy pass and one barrier fewer; else they are built here.
template <int kMfWaves, bool PLAN = false>
__global__ __launch_bounds__(64 * kMfWaves) void fir_long_mfma(MfArgs a) {
  constexpr int kMfNT = 8 / kMfWaves;           // 1,024-output tiles per wave
  typedef _Float16 half8 __attribute__((ext_vector_type(8)));
  typedef float f16x __attribute__((ext_vector_type(16)));
  extern __shared__ __attribute__((aligned(16))) _Float16 mf_lds[];
  _Float16* img = mf_lds;                              // padded input image
  _Float16* hcp = mf_lds + mf_pad(a.span) + 8;         // 8 tap copies, a.lc halves each
  const int tid = threadIdx.x;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6), lane = tid & 63;
  const int s = blockIdx.x / a.wg_per_stream;
  // (timing ablation 14: each stream's workgroups in reverse order -- is a
  // slow head workgroup its position in the grid or its work?)
  const int wb = SDR_ABL(a.ablate) == 14 ? a.wg_per_stream - 1 - (int)(blockIdx.x - s * a.wg_per_stream)
                                         : (int)(blockIdx.x - s * a.wg_per_stream);
  const long long m0 = (long long)wb * kMfOut;
  const long long pb = m0 - a.ntaps;                   // stream position of image element 0 (multiple of 8)
  const _Float16* xs = a.x + (long long)s * a.x_stride;
  const _Float16* st = a.state + (long long)s * a.ns;
#ifdef SDR_TIMING_BUILD
  unsigned long long mf_stamp[5] = {0, 0, 0, 0, 0};
#endif
  MF_STAMP(0);
  // ---- issue every load first (image chunks, taps), then write LDS: a
  // load-then-store loop waits out one memory latency per iteration.
  // kMfChunks covers the image at T <= 4096 (span = kMfOut + kd - 32 halves)
  // and kMfTaps the reversed taps (a.lc + 40 <= 4,424 halves).
  constexpr int kNT = 64 * kMfWaves, kMfChunks = (kMfOut + kMfMaxKd - 32 + 8 * kNT - 1) / (8 * kNT),
                kMfTaps = (4424 + kNT - 1) / kNT;
  const int nchunk = a.span >> 3;
  // every register defined (clamped, in-bounds addresses: n >= 8 on this
  // path), so the array stays in VGPRs; the edge chunks are rewritten below
  typedef unsigned u32x4 __attribute__((ext_vector_type(4)));  // (HIP's uint4 struct defeats SROA here)
  u32x4 iv[kMfChunks];
#pragma unroll
  for (int k = 0; k < kMfChunks; ++k) {
    long long p = pb + 8LL * (tid + k * kNT);
    p = p < 0 ? 0 : (p > a.n - 8 ? a.n - 8 : p);
    if (SDR_ABL(a.ablate) == 1) p = 0;  // (ablation 1: one cached chunk instead of the stream)
    iv[k] = *reinterpret_cast<const u32x4*>(xs + (p & ~7LL));
  }
  // the stream's first workgroup (pb = -T, T <= 4096 = kMfSt * kNT): the
  // carried state for image positions q in [-T, 0) and the new state (the
  // block's last ns inputs, src/filter.cpp:82) join the same load batch, so
  // this workgroup waits out one memory latency like the others, not three.
  // The halves are held zero-extended in 32-bit registers (packed two to a
  // register, each load would be waited for where it is packed), and each
  // loop runs only the rows k that hold some lane's element -- a uniform
  // bound: a load issued with EXEC = 0 still costs the CU's address path,
  // and 12 of the 16 loads per thread at T = 1024 were such (0.8 us of this
  // workgroup's 2.3 us of staging, phase trace profiles/r05z/)
  constexpr int kMfSt = 4096 / kNT;
  const bool head = a.head_pre && pb < 0 && SDR_ABL(a.ablate) != 7;  // (timing 7: head as interior)
  const int kst = (int)((-pb + kNT - 1) / kNT);                      // rows of positions [-T, 0)
  const int knv = (a.ns + kNT - 1) / kNT < kMfSt ? (a.ns + kNT - 1) / kNT : kMfSt;  // rows of the new state
  unsigned short sv[kMfSt], nv[kMfSt];  // raw fp16 bits
  if (head) {
#pragma unroll
    for (int k = 0; k < kMfSt; ++k) {
      if (k >= kst) break;
      const int q = (int)pb + tid + k * kNT;
      sv[k] = (q < 0 && q >= -a.ns) ? reinterpret_cast<const unsigned short*>(st)[a.ns + q] : (unsigned short)0;
    }
#pragma unroll
    for (int k = 0; k < kMfSt; ++k) {
      if (k >= knv) break;
      const int i = tid + k * kNT;
      nv[k] = i < a.ns ? reinterpret_cast<const unsigned short*>(xs)[a.n - a.ns + i] : (unsigned short)0;
    }
  }
  // the reversed f16 taps once, hb[j] = hr[j - 32], hr[v] = h[T-1-v]
  // (coalesced f32 loads); the tap copies are built from them in LDS below
  _Float16* hb = hcp + 8 * a.lc;
  const int nhb = a.lc + 40;
  float hv[PLAN ? 1 : kMfTaps];
  if constexpr (PLAN) {
    // the plan's copies: lc 16-B chunks, LDS-DMA (lane l of an instruction
    // lands at the wave-uniform base + 16 l), waited for before the barrier
    for (int c0 = wave * 64; c0 < a.lc; c0 += kNT)
      if (c0 + lane < a.lc) __builtin_amdgcn_global_load_lds(a.hplan + 8 * (c0 + lane), hcp + 8 * c0, 16, 0, 0);
  } else {
    const int ntl = SDR_ABL(a.ablate) == 3 ? 0 : a.ntaps;  // (ablation 3: no tap loads, no copies)
#pragma unroll
    for (int k = 0; k < kMfTaps; ++k) {
      const int v = tid + k * kNT - 32;
      hv[k] = (v >= 0 && v < ntl) ? a.h[a.ntaps - 1 - v] : 0.0f;
    }
  }
#pragma unroll
  for (int k = 0; k < kMfChunks; ++k) {
    const int c = tid + k * kNT;
    if (c < nchunk && !(head && pb + 8LL * c < 0)) *reinterpret_cast<u32x4*>(img + mf_pad(8 * c)) = iv[k];
  }
  if (head) {
#pragma unroll
    for (int k = 0; k < kMfSt; ++k) {
      if (k >= kst) break;
      const int q = (int)pb + tid + k * kNT;
      if (q < 0) reinterpret_cast<unsigned short*>(img)[mf_pad(q - (int)pb)] = sv[k];
    }
  }
  // block edges (the stream's first and last workgroups), element-wise over
  // the clamped chunks: the carried state before 0, zeros past n
  if ((pb < 0 && !head && SDR_ABL(a.ablate) != 7) || pb + a.span > a.n) {
    for (int c = tid; c < nchunk; c += kNT) {
      const long long p = pb + 8LL * c;
      if ((p >= 0 || head) && p + 8 <= a.n) continue;
      _Float16* d = img + mf_pad(8 * c);
#pragma unroll
      for (int r = 0; r < 8; ++r) {
        const long long q = p + r;
        d[r] = q >= 0 ? (q < a.n ? xs[q] : (_Float16)0) : (q >= -a.ns ? st[a.ns + q] : (_Float16)0);
      }
    }
  }
  if constexpr (PLAN) {
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the copies' DMAs (the barrier does not wait for them)
  } else {
#pragma unroll
    for (int k = 0; k < kMfTaps; ++k)
      if (tid + k * kNT < nhb) hb[tid + k * kNT] = (_Float16)hv[k];
  }
  __syncthreads();
  // the stream's first workgroup is the only reader of the old state (staged
  // above): it writes the new one, the block's last ns inputs
  // (src/filter.cpp:82), after that barrier
  if (head) {
#pragma unroll
    for (int k = 0; k < kMfSt; ++k) {
      if (k >= knv) break;
      if (tid + k * kNT < a.ns) reinterpret_cast<unsigned short*>(a.state)[(long long)s * a.ns + tid + k * kNT] = nv[k];
    }
    for (int i = tid + kMfSt * kNT; i < a.ns; i += kNT) a.state[(long long)s * a.ns + i] = xs[a.n - a.ns + i];
  } else if (m0 == 0 && SDR_ABL(a.ablate) != 7) {
    for (int i = tid; i < a.ns; i += kNT) a.state[(long long)s * a.ns + i] = xs[a.n - a.ns + i];
  }
  if constexpr (!PLAN) {
    const int cpr = a.lc >> 3;  // 16-B chunks per copy
    for (int c = tid; c < (SDR_ABL(a.ablate) == 3 ? 0 : 8 * cpr); c += 64 * kMfWaves) {
      const int q = c / cpr, w0 = 8 * (c - q * cpr);
      half8 v;
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = hb[w0 + q + k];
      *reinterpret_cast<half8*>(hcp + q * a.lc + w0) = v;
    }
    __syncthreads();
  }
  MF_STAMP(1);
  // Lane (i, hh) supplies A's row i with the taps of output row rho = mf_row(i)
  // (so the MFMA's row i is output row rho): with copies lc = 32 mod 128
  // halves apart, the 16 lanes of every ds_read_b128 lane group then read 16
  // distinct 16-B bank slots -- conflict-free (the identity mapping at
  // lc = 1,192 cost 8 LDS cycles per A read, SQ_LDS_BANK_CONFLICT = a third
  // of the loop's LDS cycles, profiles/r05g/)
  const int i = lane & 31, hh = lane >> 5;
  const int rho = mf_row(i);
  const int q = 7 - (rho & 7);                          // (-rho-1) mod 8
  const _Float16* arow = hcp + q * a.lc + (8 * hh - rho - 1 + 32 - q);  // + 16 s: A fragment of step s
  const int tb0 = wave * kMfNT * 1024;                  // this wave's first tile, relative to m0
  f16x acc[kMfNT];
#pragma unroll
  for (int t = 0; t < kMfNT; ++t)
#pragma unroll
    for (int r = 0; r < 16; ++r) acc[t][r] = 0.0f;
  // G steps per group; the next group's 3 G fragments are read while this
  // group's 2 G MFMAs run (kd is a multiple of 32 G: an even group count)
  constexpr int G = kMfG;
  const int ngrp = SDR_ABL(a.ablate) == 2 ? 0 : a.kd / (16 * G);  // (ablation 2: no MFMA)
  half8 av[G], bv[G][kMfNT];
  // B's fragment of step s, tile t sits at padded index mf_pad(b + 16 s +
  // 1024 t), b = tb0 + 32 i + 8 hh; since 8 hh < 32 that is mf_pad(b) + 16 s
  // + 8 (s >> 1) + 1280 t.  The loop walks both operands from pointers that
  // advance once per pair of groups (2 G steps: A 32 G halves, B 40 G), so
  // every read in the body is one ds_read_b128 at an immediate offset -- no
  // per-read address arithmetic (mf_pad of a run-time step index cost ~4
  // VALU per B read)
  const _Float16* brow = img + mf_pad(tb0 + 32 * i + 8 * hh);
  auto fetch = [&](const _Float16* ap, const _Float16* bp, int par, half8 (&aa)[G], half8 (&bb)[G][kMfNT])
      __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < G; ++u) {
      const int st = par * G + u;  // step within the pair of groups (a constant once inlined)
      aa[u] = *reinterpret_cast<const half8*>(ap + 16 * st);
#pragma unroll
      for (int t = 0; t < kMfNT; ++t)
        bb[u][t] = *reinterpret_cast<const half8*>(bp + 1280 * t + 16 * st + 8 * (st >> 1));
    }
  };
  auto mfmas = [&](const half8 (&aa)[G], const half8 (&bb)[G][kMfNT]) __attribute__((always_inline)) {
#pragma unroll
    for (int u = 0; u < G; ++u)
#pragma unroll
      for (int t = 0; t < kMfNT; ++t) acc[t] = __builtin_amdgcn_mfma_f32_32x32x16_f16(aa[u], bb[u][t], acc[t], 0, 0, 0);
  };
  // two register sets in ping-pong (ngrp is even): no copies between groups
  half8 an[G], bn[G][kMfNT];
  const _Float16* ap = arow;
  const _Float16* bp = brow;
  fetch(ap, bp, 0, av, bv);
  for (int g = 0; g < ngrp; g += 2) {
    fetch(ap, bp, 1, an, bn);
    mfmas(av, bv);
    ap += 32 * G;
    bp += 40 * G;
    if (g + 2 < ngrp) fetch(ap, bp, 0, av, bv);
    mfmas(an, bn);
  }
#ifdef SDR_TIMING_BUILD
  if (a.trace) {  // the accumulators ready (the stamp would otherwise pass the MFMAs in flight)
#pragma unroll
    for (int t = 0; t < kMfNT; ++t) asm volatile("" ::"v"(acc[t][0]), "v"(acc[t][15]));
  }
#endif
  MF_STAMP(2);
  // ---- outputs: lane (column j = i, half hh) holds rows (r & 3) + 8 (r >> 2) + 4 hh
  float* ys = a.y + (long long)s * a.y_stride;
#if SDR_F16_TSTORE
  float* ost = reinterpret_cast<float*>(mf_lds + a.ost) + wave * 32 * kMfOstRow;
  const bool ys_al = (reinterpret_cast<uintptr_t>(ys) & 15) == 0;
#endif
#pragma unroll
  for (int t = 0; t < kMfNT; ++t) {
#if SDR_F16_TSTORE
    // a whole tile inside the block: through this wave's LDS area, then 4
    // stores of 1 KB contiguous each (instead of 32 rows x 32 B per store)
    const long long mt = m0 + tb0 + t * 1024;
    if (ys_al && mt + 1024 <= a.n) {
#pragma unroll
      for (int g = 0; g < 4; ++g)
        *reinterpret_cast<float4*>(ost + kMfOstRow * i + mf_row(8 * g + 4 * hh)) =
            make_float4(acc[t][4 * g], acc[t][4 * g + 1], acc[t][4 * g + 2], acc[t][4 * g + 3]);
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      __builtin_amdgcn_wave_barrier();
#pragma unroll
      for (int k = 0; k < 4; ++k) {
        const int q = 4 * (lane + 64 * k);
        const float4 v = *reinterpret_cast<const float4*>(ost + kMfOstRow * (q >> 5) + (q & 31));
        *reinterpret_cast<float4*>(ys + mt + q) = v;
      }
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // the area is reused by the next tile
      __builtin_amdgcn_wave_barrier();
      continue;
    }
#endif
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const long long m = m0 + tb0 + t * 1024 + 32 * i + mf_row(8 * g + 4 * hh);
      const float4 v = make_float4(acc[t][4 * g], acc[t][4 * g + 1], acc[t][4 * g + 2], acc[t][4 * g + 3]);
      if (SDR_ABL(a.ablate) == 4 && v.x != -0x1.234p100f) continue;  // (ablation 4: no stores)
      if (m + 4 <= a.n && ((reinterpret_cast<uintptr_t>(ys + m) & 15) == 0)) {
        *reinterpret_cast<float4*>(ys + m) = v;
      } else {
        const float w[4] = {v.x, v.y, v.z, v.w};
#pragma unroll
        for (int r = 0; r < 4; ++r)
          if (m + r < a.n) ys[m + r] = w[r];
      }
    }
  }
#ifdef SDR_TIMING_BUILD
  MF_STAMP(3);
  if (a.trace) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  MF_STAMP(4);
  MF_STAMP_FLUSH();
#endif
}

// hp2[d] = (half(h[d]), half(h[d-1])) for d = 0..T, zero past both ends and
// up to the padded length.
__global__ __launch_bounds__(kWG) void build_pairs_h(const float* __restrict__ h, int ntaps, int len, uint32_t* hp2) {
  const int d = blockIdx.x * kWG + threadIdx.x;
  if (d >= len) return;
  const _Float16 lo = d < ntaps ? (_Float16)h[d] : (_Float16)0;
  const _Float16 hi = (d >= 1 && d - 1 < ntaps) ? (_Float16)h[d - 1] : (_Float16)0;
  half2_t v = {lo, hi};
  hp2[d] = __builtin_bit_cast(uint32_t, v);
}

// The tap plan of fir_long_mfma<.., true>: copy q of the reversed f16 taps,
// shifted by q halves -- plan[q*lc + w] = hr[w + q - 32], hr[v] = h[T-1-v]
// (0 outside [0, T)) -- exactly what the kernel otherwise builds in LDS.
__global__ __launch_bounds__(kWG) void build_mf_plan(const float* __restrict__ h, int ntaps, int lc, _Float16* plan) {
  const int idx = blockIdx.x * kWG + threadIdx.x;
  if (idx >= 8 * lc) return;
  const int q = idx / lc, w = idx - q * lc;
  const int v = w + q - 32;
  plan[idx] = (v >= 0 && v < ntaps) ? (_Float16)h[ntaps - 1 - v] : (_Float16)0;
}

__global__ __launch_bounds__(kWG) void long_commit_h(const _Float16* __restrict__ x, long long n,
                                                     long long x_stride, _Float16* state, int ns) {
  const int s = blockIdx.y;
  const int i = blockIdx.x * kWG + threadIdx.x;
  if (i >= ns) return;
  state[(long long)s * ns + i] = x[(long long)s * x_stride + n - ns + i];
}

__global__ __launch_bounds__(kWG) void f32_to_f16(const float* __restrict__ x, long long count, _Float16* y) {
  const long long i = (long long)blockIdx.x * kWG + threadIdx.x;
  if (i < count) y[i] = (_Float16)x[i];
}

}  // namespace

// T <= 4096: the image, tap copies, reversed taps and one output transpose
// area per wave fit the LDS (at 4096: 123 KiB with 4 waves, 141 KiB with 8;
// at 1024: 61 / 79 KiB; launch_fir_long_h checks the CU's LDS), and no
// workgroup but a stream's first reaches into the state (T < kMfOut), which
// lets that one commit the new state in-kernel
bool fir_f16_uses_mfma(int ntaps) {
  return ntaps % 8 == 0 && ntaps <= 4096 && sw(kSwF16Mfma) != 0;
}

size_t fir_long_h_pairs(int ntaps) { return (size_t)((ntaps + 1 + 31) / 32 * 32); }

namespace {
int mf_kd(int ntaps) { return (ntaps + 31 + 32 * kMfG - 1) / (32 * kMfG) * (32 * kMfG); }  // even group count
// halves per tap copy: >= kd + 40, and 32 mod 128 (copy q's 16-B slots then
// sit 4q mod 16 slots apart, which with mf_row makes the A reads conflict-free)
int mf_lc(int ntaps) { return (mf_kd(ntaps) + 40 - 32 + 127) / 128 * 128 + 32; }
}  // namespace

#ifdef SDR_TIMING_BUILD
namespace {
unsigned long long* g_mf_trace = nullptr;
size_t g_mf_trace_n = 0, g_mf_trace_used = 0;
unsigned long long* mf_trace_buffer(size_t n) {  // (not for graph capture: a timing-build probe)
  if (n > g_mf_trace_n) {
    if (g_mf_trace) (void)hipFree(g_mf_trace);
    if (hipMalloc(&g_mf_trace, n * sizeof(unsigned long long)) != hipSuccess) return g_mf_trace = nullptr;
    g_mf_trace_n = n;
  }
  g_mf_trace_used = n;
  return g_mf_trace;
}
}  // namespace
}  // namespace sdr
// Timing builds only: copy the last traced fir_long_mfma launch's stamps
// (kMfTraceW per workgroup) to host; returns the count available.
extern "C" long long sdr_timing_f16_trace(unsigned long long* host, long long max) {
  if (!sdr::g_mf_trace) return 0;
  if (hipDeviceSynchronize() != hipSuccess) return -1;
  const long long n = (long long)sdr::g_mf_trace_used < max ? (long long)sdr::g_mf_trace_used : max;
  if (host && n > 0 && hipMemcpy(host, sdr::g_mf_trace, n * sizeof(unsigned long long), hipMemcpyDeviceToHost) != hipSuccess)
    return -1;
  return (long long)sdr::g_mf_trace_used;
}
namespace sdr {
#endif

size_t fir_f16_plan_halves(int ntaps) {
  return (ntaps % 8 == 0 && ntaps >= 8 && ntaps <= 4096) ? (size_t)8 * mf_lc(ntaps) : 0;
}

hipError_t build_fir_f16_plan(const float* h, int ntaps, void* plan, hipStream_t st) {
  const int lc = mf_lc(ntaps);
  hipLaunchKernelGGL(build_mf_plan, dim3((8 * lc + kWG - 1) / kWG), dim3(kWG), 0, st, h, ntaps, lc,
                     static_cast<_Float16*>(plan));
  return hipGetLastError();
}

hipError_t launch_fir_long_h(const void* x, long long n, int nstreams, long long x_stride, const float* h, int ntaps,
                             void* state, int ns, float* y, long long y_stride, uint32_t* scratch_pairs,
                             hipStream_t st, const void* plan) {
  // the MFMA form: T % 8 == 0 keeps the staged image's 16-B chunks aligned
  // (x rows are 16-B aligned, checked by the caller); SDR_F16_MFMA=0 selects
  // the dot2 kernel below (A/B, tests)
  if (fir_f16_uses_mfma(ntaps) && n >= 8) {  // (n >= 8: the clamped staging loads stay in the row)
    MfArgs a;
    a.x = static_cast<const _Float16*>(x);
    a.n = n;
    a.x_stride = x_stride;
    a.h = h;
    a.ntaps = ntaps;
    a.kd = mf_kd(ntaps);  // zero taps past the band
    a.lc = mf_lc(ntaps);
    a.state = static_cast<_Float16*>(state);
    a.ns = ns;
    a.y = y;
    a.y_stride = y_stride;
    a.wg_per_stream = (int)((n + kMfOut - 1) / kMfOut);
    a.span = kMfOut + a.kd - 32;
    static const int ablate = SDR_TIMING_ENV("SDR_ABLATE", 0);
    a.ablate = ablate;
    const int head_pre = sw(kSwF16Head);  // (switch: the tests run both orders)
    a.head_pre = head_pre;
    a.hplan = static_cast<const _Float16*>(plan);
    a.trace = nullptr;
#ifdef SDR_TIMING_BUILD
    static const int tr = SDR_TIMING_ENV("SDR_F16_TRACE", 0);
    if (tr) a.trace = mf_trace_buffer((size_t)a.wg_per_stream * nstreams * kMfTraceW);
#endif
    // one launch: each stream's first workgroup commits the state itself
    // two waves per SIMD, one tile each: 8.8 vs 10.9 us per kernel on cfg5h
    // (profiles/r04y/); SDR_F16_W8=0 restores four waves of two tiles
    const int w8 = sw(kSwF16W8);
    // image, 8 tap copies, (no plan) the reversed taps (a.lc + 40 halves),
    // (SDR_F16_TSTORE) one output transpose area per wave of the variant
    const size_t taps_end = (size_t)mf_pad(a.span) + 8 + (plan ? 8 : 9) * (size_t)a.lc + (plan ? 0 : 40);
    a.ost = (int)((taps_end + 7) / 8 * 8);
    const size_t waves = w8 ? 8 : 4;
    const size_t lds = (SDR_F16_TSTORE ? (size_t)a.ost * sizeof(_Float16) + waves * 32 * kMfOstRow * sizeof(float)
                                       : taps_end * sizeof(_Float16));
    const long long blocks = (long long)a.wg_per_stream * nstreams;
    if (blocks > 0x7fffffffLL || lds > (size_t)device_lds_bytes()) return hipErrorInvalidValue;
    if (w8 && plan)
      hipLaunchKernelGGL((fir_long_mfma<8, true>), dim3((unsigned)blocks), dim3(512), lds, st, a);
    else if (w8)
      hipLaunchKernelGGL((fir_long_mfma<8, false>), dim3((unsigned)blocks), dim3(512), lds, st, a);
    else if (plan)
      hipLaunchKernelGGL((fir_long_mfma<4, true>), dim3((unsigned)blocks), dim3(256), lds, st, a);
    else
      hipLaunchKernelGGL((fir_long_mfma<4, false>), dim3((unsigned)blocks), dim3(256), lds, st, a);
    return hipGetLastError();
  }
  const int len = (int)fir_long_h_pairs(ntaps);
  hipLaunchKernelGGL(build_pairs_h, dim3((len + kWG - 1) / kWG), dim3(kWG), 0, st, h, ntaps, len, scratch_pairs);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  LongHArgs a;
  a.x = static_cast<const _Float16*>(x);
  a.n = n;
  a.x_stride = x_stride;
  a.hp2 = scratch_pairs;
  a.ntaps = ntaps;
  a.state = static_cast<const _Float16*>(state);
  a.ns = ns;
  a.y = y;
  a.y_stride = y_stride;
  constexpr int OUT_WG = 64 * kLongRH * kLongNW;
  a.tiles_per_stream = (int)((n + OUT_WG - 1) / OUT_WG);
  a.halo = (ntaps + 7) / 8 * 8 + 32;  // covers d up to the padded pass end
  a.img = a.halo + OUT_WG + 8;
  const long long blocks = (long long)a.tiles_per_stream * nstreams;
  if (blocks > 0x7fffffffLL) return hipErrorInvalidValue;
  hipLaunchKernelGGL(fir_long_h, dim3((unsigned)blocks), dim3(64 * kLongNW), (size_t)a.img * 2, st, a);
  e = hipGetLastError();
  if (e != hipSuccess || ns <= 0) return e;
  hipLaunchKernelGGL(long_commit_h, dim3((ns + kWG - 1) / kWG, (unsigned)nstreams), dim3(kWG), 0, st,
                     static_cast<const _Float16*>(x), n, x_stride, static_cast<_Float16*>(state), ns);
  return hipGetLastError();
}

hipError_t launch_f32_to_f16(const float* x, long long count, void* y, hipStream_t st) {
  hipLaunchKernelGGL(f32_to_f16, dim3((unsigned)((count + kWG - 1) / kWG)), dim3(kWG), 0, st, x, count,
                     static_cast<_Float16*>(y));
  return hipGetLastError();
}

}  // namespace sdr
