// resample_sg.hip -- the polyphase resampler (src/filter.cpp:142-173) with
// lane = column, taps as SGPR operands, and two adjacent phases per wave
// sharing every LDS read.
//
// Phase algebra (resample.hip): output j = L*t + phi has phase
// p = (phi*M) mod L and newest input q(phi) = t*M + floor(phi*M/L); a
// *column* is one period t of one stream.  A workgroup's *unit* is 64
// columns (lane = column) x one phase group of 2*NCW consecutive phases;
// compute wave w takes the phase pair (phiA, phiB) = (2(NCW g + w),
// 2(NCW g + w) + 1), whose windows [q - (C-1), q] are 5-6 inputs apart at
// 147/800: both outputs are accumulated from ONE stream of 16-B chunk reads
// of the lane's column window (resample_lp reads one chunk per 4
// multiply-adds of one output; this kernel one per 8).
//
// Taps: per pair, two rows pre-shifted onto the chunk grid of the group's
// window (sg tables, built once per plan): element jj of chunk cc meets
// rowB[4cc + 3 - jj] and rowA[...] -- the tap i of output B / A whose input
// that element is, or 0 where the element is outside that output's window.
// Every output therefore still sums exactly its C products in ascending k
// (i = 0..C-1), separately rounded, from +0.0f; the padding terms are
// 0 * x = +-0 and leave the sum unchanged (it is never -0) as long as x is
// finite; and a non-finite x in a padding position makes the output NaN.
// So an output that comes out finite is the reference's, and a wave with a
// non-finite output rescans its pair with every padding element masked to 0:
// bit-exact for every input.
//
// Waves: NCW compute waves + one loader wave.  The loader stages unit u+1
// (LDS-DMA; edge chunks from the carried state or zeros via registers) into
// the other of two LDS images while the compute waves scan unit u; one
// barrier per unit.  The first unit of a block also commits the new state of
// every stream whose first column the block holds (only that unit reads the
// old state; host-checked).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "sdr_common.hpp"

#pragma clang fp contract(off)

namespace sdr {
namespace {

constexpr int kSgMaxDelta = 10;   // ceil(M/L) this kernel takes
constexpr int kSgVPC = 5;         // VGPR taps: chunks of both rows per pass (2 x 2 x 5 x 4 VGPRs in flight)
constexpr int kSgPC = 6;          // SGPR taps: chunks of both rows per pass (2 x 24 SGPRs; 8 spills)
constexpr int kSgPF = 2;          // LDS chunk reads in flight ahead of the one in use
constexpr int kSgLds = 163840 - 256;

struct SgGeom {
  int ncw = 0;    // compute waves (phase pairs per group)
  int ngrp = 0;   // phase groups
  int npairs = 0;
  int nc = 0;     // chunks per pair scan
  int slack = 0;  // chunks of window below the group's lowest needed input
  int segc = 0;   // chunks staged per column per unit (64..128)
  int stride = 0; // LDS floats per column segment (stride / 4 odd)
};

__host__ __device__ inline long long sg_q(long long phi, int up, int down) { return phi * down / up; }
__host__ __device__ inline long long sg_floor4(long long v) { return v & ~3LL; }

// Window base (relative to t*M) of group g.
__host__ __device__ inline long long sg_wbase(int g, int ncw, int cmax, int slack, int up, int down) {
  return sg_floor4(sg_q(2LL * ncw * g, up, down) - (cmax - 1)) - 4LL * slack;
}

bool sg_geometry(int up, int down, int cmax, SgGeom* G) {
  if (up < 2 || down % 4 != 0 || (down + up - 1) / up > kSgMaxDelta) return false;
  const int dmax = (down + up - 1) / up;
  const int nc = (cmax + 3 + dmax + 3) / 4;
  for (int ncw = 15; ncw >= 4; --ncw) {
    SgGeom g;
    g.ncw = ncw;
    g.ngrp = (up + 2 * ncw - 1) / (2 * ncw);
    g.npairs = (up + 1) / 2;
    g.nc = nc;
    // slack: every pair's lowest chunk, ctop - (nc - 1), must stay in the segment
    int slack = 0;
    for (int pi = 0; pi < g.npairs; ++pi) {
      const int grp = pi / ncw;
      const long long phiB = 2LL * pi + 1 < up ? 2LL * pi + 1 : 2LL * pi;
      const long long eB = sg_q(phiB, up, down) - sg_wbase(grp, ncw, cmax, 0, up, down);
      const long long low = (eB >> 2) - (nc - 1);
      if (-low > slack) slack = (int)(-low);
    }
    g.slack = slack;
    int segc = 0;
    for (int grp = 0; grp < g.ngrp; ++grp) {
      const long long last = std::min<long long>(2LL * ncw * (grp + 1), up) - 1;
      const long long top = sg_q(last, up, down) - sg_wbase(grp, ncw, cmax, slack, up, down);
      segc = std::max<int>(segc, (int)(top >> 2) + 1);
    }
    // odd chunk stride: the 16-lane groups of a ds_read_b128 (same chunk of
    // 16 columns) then meet 16 different bank quads
    g.segc = segc;
    g.stride = 4 * (segc | 1);
    // groups >= 1 must not read the carried state (only a block's first unit
    // reads it, before committing the new one)
    if (g.ngrp > 1 && sg_wbase(1, ncw, cmax, slack, up, down) < 0) return false;
    // the loader moves a column in two DMA instructions
    if (g.segc < 64 || g.segc > 128) return false;
    if (2LL * 64 * g.stride * 4 <= kSgLds) {
      *G = g;
      return true;
    }
  }
  return false;
}

// tables: [npairs][2][4*nc] shifted rows (B then A), then int4 meta per pair
__global__ __launch_bounds__(kWG) void build_sg_tables(const float* __restrict__ h, int up, int down, int cmax,
                                                       int ncw, int npairs, int nc, int slack, float* tab) {
  const int NU = 4 * nc;
  const long long idx = (long long)blockIdx.x * kWG + threadIdx.x;
  if (idx >= (long long)npairs * 2 * NU) return;
  const int pi = (int)(idx / (2 * NU));
  const int which = (int)(idx / NU) & 1;  // 0 = B, 1 = A
  const int u = (int)(idx % NU);
  const int grp = pi / ncw;
  const long long phiA = 2LL * pi;
  const long long phiB = phiA + 1 < up ? phiA + 1 : phiA;
  const long long wb = sg_wbase(grp, ncw, cmax, slack, up, down);
  const long long eB = sg_q(phiB, up, down) - wb;
  const int A1 = (int)(eB & 3);
  const int delta = (int)(sg_q(phiB, up, down) - sg_q(phiA, up, down));
  const long long phi = which ? phiA : phiB;
  const int p = (int)(phi * down % up);
  const int i = u - (3 - A1) - (which ? delta : 0);
  tab[idx] = (i >= 0 && i < cmax) ? h[p + (long long)i * up] : 0.0f;
  if (which == 0 && u == 0) {
    int* meta = reinterpret_cast<int*>(tab + (size_t)npairs * 2 * NU) + 4 * pi;
    meta[0] = (int)(eB >> 2);  // ctop: the chunk holding output B's newest input
    meta[1] = A1;
    meta[2] = delta;
    meta[3] = (int)phiA | ((int)phiB << 16);
  }
}

struct SgArgs {
  const float* x;
  long long n, x_stride;
  const float* tab;  // build_sg_tables
  float* state;
  int ns;
  float* y;
  long long y_stride, ny;
  int up, down, cmax;
  int np;       // columns per stream
  int ncols;    // nstreams * np
  int nunits;   // blocks * ngrp
  int ngrp, ncw, npairs, slack, segc, stride;
  int gmajor;  // unit order: 0 block-major (a block's groups in a row), 1 group-major
  int ablate;  // timing experiments only (SDR_ABLATE): 1 = no staging, 2 = no scan
};

// Stage unit u (64 columns x segc chunks, column c's segment at c * stride
// floats) into buf.  Loader wave only, so its instruction count is its time:
// lane c holds column c's window row (one vector division per unit), and per
// column the loop reads that row with v_readlane and issues two LDS-DMA
// instructions (chunks 0..63, then 64..segc-1; 64 <= segc <= 128), lane k
// landing at base + 16k.  A column whose window reaches into the carried
// state or past the block takes the per-lane path (registers).  Fire and
// forget: the DMAs are drained once, before the barrier that publishes the
// image.
__device__ __forceinline__ void sg_unit(const SgArgs& a, int u, int& b, int& g) {
  if (a.gmajor) {
    const int nblk = a.nunits / a.ngrp;
    g = u / nblk;
    b = u - g * nblk;
  } else {
    b = u / a.ngrp;
    g = u - b * a.ngrp;
  }
}

// Columns c0, c0 + dc, ... of unit u.  No drain: the caller waits vmcnt(0)
// before the barrier that publishes the image.
__device__ __forceinline__ void sg_stage(const SgArgs& a, float* buf, int u, int ln, int c0, int dc) {
  int b, g;
  sg_unit(a, u, b, g);
  const long long wb = sg_wbase(g, a.ncw, a.cmax, a.slack, a.up, a.down);
  const int segc = a.segc;
  const int colL = b * 64 + ln;  // lane ln: column b*64 + ln
  const int sL = colL / a.np, tL = colL - sL * a.np;
  const long long pL = (long long)tL * a.down + wb;
  const unsigned long long rowL = reinterpret_cast<unsigned long long>(a.x + (long long)sL * a.x_stride + pL);
  const unsigned long long inner =
      __builtin_amdgcn_ballot_w64(colL < a.ncols && pL >= 0 && pL + 4LL * segc <= a.n);
  const int ncol = min(64, a.ncols - b * 64);
  const bool tail = ln < segc - 64;
  for (int c = c0; c < ncol; c += dc) {
    float* lds = buf + c * a.stride;
    if ((inner >> c) & 1) {
      const unsigned lo = __builtin_amdgcn_readlane((unsigned)rowL, c);
      const unsigned hi = __builtin_amdgcn_readlane((unsigned)(rowL >> 32), c);
      const float* r = reinterpret_cast<const float*>(((unsigned long long)hi << 32) | lo) + 4 * ln;
      __builtin_amdgcn_global_load_lds(r, lds, 16, 0, 0);
      if (tail) __builtin_amdgcn_global_load_lds(r + 256, lds + 256, 16, 0, 0);
    } else {
      const int col = b * 64 + c;
      const int s = col / a.np, t = col - s * a.np;
      const float* xs = a.x + (long long)s * a.x_stride;
      for (int j = ln; j < segc; j += 64) {
        const long long P = (long long)t * a.down + wb + 4LL * j;
        float w4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long long p = P + r;
          w4[r] = p >= 0 ? (p < a.n ? xs[p] : 0.0f) : (p >= -a.ns ? a.state[(long long)s * a.ns + a.ns + p] : 0.0f);
        }
        *reinterpret_cast<float4*>(lds + 4 * j) = make_float4(w4[0], w4[1], w4[2], w4[3]);
      }
      // a stream's first column in its first group holds the only reads of
      // its old state (consumed just above, by this wave): state <- last ns
      // inputs of the block (src/filter.cpp:169)
      if (g == 0 && t == 0)
        for (int i = ln; i < a.ns; i += 64)
          a.state[(long long)s * a.ns + i] = xs[(a.n - a.ns) + i];
    }
  }
}

template <int B, int E, class F>
__device__ __forceinline__ void sg_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    sg_for<B + 1, E>(f);
  }
}

// One pair over NC chunks.  lo = the lane's chunk (ctop - NC + 1); chunk cc
// (u = 4cc + 3 - jj) sits at lo + 4*(NC - 1 - cc).  MASK: padding elements
// (u outside [loB, loB + CMAX) for B, [loA, loA + CMAX) for A) enter as 0.
typedef __attribute__((address_space(3))) float lds_f;
typedef float sg_f4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) const sg_f4 lds_f4;

// One pair over NC chunks.  lo = the lane's chunk (ctop - NC + 1); chunk cc
// (u = 4cc + 3 - jj) sits at lo[NC - 1 - cc].  The taps stream through
// VGPRs: vector loads of the (wave-uniform) rows, kSgVPC chunks of both rows
// per pass, the next pass's in flight during this one -- vmcnt counts them
// in order, where scalar loads share the out-of-order lgkmcnt with the LDS
// reads and could not be waited for one pass at a time; and a VGPR operand
// issues at full rate, an SGPR one at half (profiles/r02_ubench_valu.txt).
// MASK: padding elements (u outside [loB, loB + CMAX) for B, [loA, loA +
// CMAX) for A) enter as 0.
template <int CMAX, int NC, bool MASK>
__device__ __forceinline__ void sg_scan_v(lds_f4* lo, const float* rows, float& accA, float& accB, int loB,
                                          int loA) {
  constexpr int PC = kSgVPC, NP = (NC + PC - 1) / PC;
  int z = 0;
  asm volatile("" : "+v"(z));  // a per-lane address: vector loads, not scalar ones
  const sg_f4* rb = reinterpret_cast<const sg_f4*>(rows) + z;  // row B chunks 0..NC-1, row A NC..2NC-1
  sg_f4 tb[2][PC], ta[2][PC];
  auto load = [&](auto pi, auto bi) __attribute__((always_inline)) {
    constexpr int c0 = decltype(pi)::value * PC;
    constexpr int c1 = c0 + PC < NC ? c0 + PC : NC;
    constexpr int q = decltype(bi)::value;
#pragma unroll
    for (int i = 0; i < c1 - c0; ++i) {
      tb[q][i] = rb[c0 + i];
      ta[q][i] = rb[NC + c0 + i];
    }
  };
  load(std::integral_constant<int, 0>{}, std::integral_constant<int, 0>{});
  sg_f4 pf[kSgPF + 1];
  sg_for<0, kSgPF>([&](auto ui) {
    constexpr int cc = decltype(ui)::value;
    if constexpr (cc < NC) pf[cc] = lo[NC - 1 - cc];
  });
  sg_for<0, NP>([&](auto pi) {
    constexpr int p = decltype(pi)::value;
    constexpr int c0 = p * PC;
    constexpr int c1 = c0 + PC < NC ? c0 + PC : NC;
    constexpr int q = p & 1;
    if constexpr (p + 1 < NP) load(std::integral_constant<int, p + 1>{}, std::integral_constant<int, q ^ 1>{});
    sg_for<c0, c1>([&](auto ci) {
      constexpr int cc = decltype(ci)::value;
      if constexpr (cc + kSgPF < NC) pf[kSgPF] = lo[NC - 1 - cc - kSgPF];
      const sg_f4 hbv = tb[q][cc - c0], hav = ta[q][cc - c0];
      sg_for<0, 4>([&](auto ji) {
        constexpr int jj = 3 - decltype(ji)::value;
        constexpr int u = 4 * cc + 3 - jj;
        float xb = pf[0][jj], xa = pf[0][jj];
        if constexpr (MASK) {
          xb = (u >= loB && u < loB + CMAX) ? xb : 0.0f;
          xa = (u >= loA && u < loA + CMAX) ? xa : 0.0f;
        }
        accB = accB + hbv[3 - jj] * xb;
        accA = accA + hav[3 - jj] * xa;
      });
#pragma unroll
      for (int k = 0; k < kSgPF; ++k) pf[k] = pf[k + 1];
      asm volatile("" : "+v"(accA), "+v"(accB));
      __builtin_amdgcn_sched_barrier(0);
    });
  });
}

// The same scan with the taps as SGPR operands (scalar loads, kSgPC chunks
// of both rows per pass, one lgkmcnt(0) wait each).
template <int CMAX, int NC, bool MASK>
__device__ __forceinline__ void sg_scan_s(lds_f4* lo, const float* rows, float& accA, float& accB, int loB,
                                          int loA) {
  constexpr int NU = 4 * NC, NP = (NC + kSgPC - 1) / kSgPC;
  using hconst = const __attribute__((address_space(4))) float*;
  const hconst hr = (hconst)rows;
  sg_f4 pf[kSgPF + 1];
  sg_for<0, kSgPF>([&](auto ui) {
    constexpr int cc = decltype(ui)::value;
    if constexpr (cc < NC) pf[cc] = lo[NC - 1 - cc];
  });
  sg_for<0, NP>([&](auto pi) {
    constexpr int c0 = decltype(pi)::value * kSgPC;
    constexpr int c1 = c0 + kSgPC < NC ? c0 + kSgPC : NC;
    float hb[4 * kSgPC], ha[4 * kSgPC];
#pragma unroll
    for (int i = 0; i < 4 * (c1 - c0); ++i) {
      hb[i] = hr[4 * c0 + i];
      ha[i] = hr[NU + 4 * c0 + i];
    }
#pragma unroll
    for (int i = 0; i < 4 * (c1 - c0); ++i) asm volatile("" : "+s"(hb[i]), "+s"(ha[i]));
    sg_for<c0, c1>([&](auto ci) {
      constexpr int cc = decltype(ci)::value;
      if constexpr (cc + kSgPF < NC) pf[kSgPF] = lo[NC - 1 - cc - kSgPF];
      sg_for<0, 4>([&](auto ji) {
        constexpr int jj = 3 - decltype(ji)::value;
        constexpr int u = 4 * cc + 3 - jj;
        float xb = pf[0][jj], xa = pf[0][jj];
        if constexpr (MASK) {
          xb = (u >= loB && u < loB + CMAX) ? xb : 0.0f;
          xa = (u >= loA && u < loA + CMAX) ? xa : 0.0f;
        }
        accB = accB + hb[u - 4 * c0] * xb;
        accA = accA + ha[u - 4 * c0] * xa;
      });
#pragma unroll
      for (int k = 0; k < kSgPF; ++k) pf[k] = pf[k + 1];
      asm volatile("" : "+v"(accA), "+v"(accB));
      __builtin_amdgcn_sched_barrier(0);
    });
  });
}

// SDR_SG_TAPS (build switch): 0 taps as SGPR operands, 1 streamed through VGPRs
#ifndef SDR_SG_TAPS
#define SDR_SG_TAPS 0
#endif
template <int CMAX, int NC, bool MASK>
__device__ __forceinline__ void sg_scan(lds_f4* lo, const float* rows, float& accA, float& accB, int loB,
                                        int loA) {
  if constexpr (SDR_SG_TAPS)
    sg_scan_v<CMAX, NC, MASK>(lo, rows, accA, accB, loB, loA);
  else
    sg_scan_s<CMAX, NC, MASK>(lo, rows, accA, accB, loB, loA);
}

template <int CMAX, int NC>
__global__ __launch_bounds__(1024, 1) void resample_sg(SgArgs a) {
  extern __shared__ __attribute__((aligned(16))) float sgbuf[];
  const int nw = blockDim.x >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), ln = threadIdx.x & 63;
  // staging: by the loader waves past the a.ncw compute waves, or (no
  // loader) by every wave, each a stride of the 64 columns
  const bool loader = wv >= a.ncw;
  const bool stager = a.ncw == nw || loader;
  const int sw = a.ncw == nw ? wv : wv - a.ncw, nsw = a.ncw == nw ? nw : nw - a.ncw;
  const int per = a.nunits / (int)gridDim.x, extra = a.nunits % (int)gridDim.x;
  const int u0 = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int u1 = u0 + per + ((int)blockIdx.x < extra ? 1 : 0);
  if (u0 >= u1) return;
  const int* meta = reinterpret_cast<const int*>(a.tab + (size_t)a.npairs * 2 * 4 * NC);
  if (stager && a.ablate != 1) sg_stage(a, sgbuf, u0, ln, sw, nsw);
  for (int u = u0, k = 0; u < u1; ++u, ++k) {
    // every wave drained its own DMAs (and stores): unit u is staged, and
    // the image unit u-1 used is free.  A raw barrier: __syncthreads() would
    // wait vmcnt(0) itself -- here it is explicit.
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    if (stager && u + 1 < u1 && a.ablate != 1)
      sg_stage(a, sgbuf + ((k + 1) & 1) * 64 * a.stride, u + 1, ln, sw, nsw);
    if (loader) continue;
    int b, g;
    sg_unit(a, u, b, g);
    const int pi = __builtin_amdgcn_readfirstlane(g * a.ncw + wv);  // uniform (the loop's divergent staging hides it)
    if (pi >= a.npairs || a.ablate >= 2) continue;
    const int ctop = meta[4 * pi], A1 = meta[4 * pi + 1], delta = meta[4 * pi + 2], ph = meta[4 * pi + 3];
    const int phiA = ph & 0xffff, phiB = ph >> 16;
    // the lane's lowest chunk of this pair, as an LDS (address space 3) pointer
    int off = (k & 1) * 64 * a.stride + ln * a.stride + 4 * (ctop - (NC - 1));
    asm volatile("" : "+v"(off));  // one VGPR base; chunk offsets stay immediates
    lds_f4* lo = (lds_f4*)((__attribute__((address_space(3))) char*)((lds_f*)sgbuf) + 4 * off);
    const float* rows = a.tab + (size_t)pi * 2 * 4 * NC;
    float accA = 0.0f, accB = 0.0f;
    const int loB = 3 - A1, loA = 3 - A1 + delta;
    sg_scan<CMAX, NC, false>(lo, rows, accA, accB, loB, loA);
    // A padding term is 0 * x: +-0 for finite x, NaN for an infinite or NaN
    // x, which then makes the output non-finite.  So a finite output is the
    // reference's; a wave with a non-finite one rescans with the padding
    // elements masked to 0 (each output then has exactly its own terms).
    if (__builtin_amdgcn_ballot_w64(!__builtin_isfinite(accA) || !__builtin_isfinite(accB))) {
      accA = accB = 0.0f;
      // opaque: the rescan reloads its taps (reusing the first scan's loads
      // would keep all 2 * 4 * NC taps live across it)
      const float* rows2 = rows;
      asm volatile("" : "+s"(rows2));
      sg_scan<CMAX, NC, true>(lo, rows2, accA, accB, loB, loA);
    }
    const int col = b * 64 + ln;
    if (col < a.ncols) {
      const int s = col / a.np, t = col - s * a.np;
      float* ys = a.y + (long long)s * a.y_stride;
      const long long jA = (long long)a.up * t + phiA, jB = (long long)a.up * t + phiB;
      if (jA < a.ny) ys[jA] = accA;
      if (phiB != phiA && jB < a.ny) ys[jB] = accB;
    }
  }
}

// read per launch (a getenv scan), so a test can switch kernels in-process
bool sg_enabled() {
  const char* e = std::getenv("SDR_RESAMPLE_SG");
  return e && std::atoi(e) != 0;  // off: slower than resample_lp on cfg3
}

template <int CMAX>
hipError_t launch_sg_nc(const SgGeom& G, const SgArgs& a, dim3 grid, dim3 blk, size_t lds, hipStream_t st) {
  switch (G.nc - (CMAX + 3 + 3) / 4) {  // nc = (CMAX + 3 + dmax + 3) / 4, dmax <= kSgMaxDelta
    case 0: hipLaunchKernelGGL((resample_sg<CMAX, (CMAX + 6) / 4>), grid, blk, lds, st, a); break;
    case 1: hipLaunchKernelGGL((resample_sg<CMAX, (CMAX + 6) / 4 + 1>), grid, blk, lds, st, a); break;
    case 2: hipLaunchKernelGGL((resample_sg<CMAX, (CMAX + 6) / 4 + 2>), grid, blk, lds, st, a); break;
    case 3: hipLaunchKernelGGL((resample_sg<CMAX, (CMAX + 6) / 4 + 3>), grid, blk, lds, st, a); break;
    default: return hipErrorInvalidValue;
  }
  return hipGetLastError();
}

}  // namespace

size_t resample_sg_table_floats(int up, int ntaps) {
  // upper bound over down (dmax <= kSgMaxDelta): nc <= (cmax + 3 + 10 + 3) / 4
  const int cmax = (ntaps + up - 1) / up;
  const size_t nc = (size_t)(cmax + 3 + kSgMaxDelta + 3) / 4;
  return (size_t)((up + 1) / 2) * 2 * 4 * nc + 4 * (size_t)((up + 1) / 2);
}

bool resample_sg_covers(int up, int down, int ntaps, int ns) {
  const int cmax = (ntaps + up - 1) / up;
  SgGeom G;
  return sg_enabled() && up >= 2 && ntaps == cmax * up && (cmax == 151 || cmax == 101) && ns >= cmax - 1 &&
         sg_geometry(up, down, cmax, &G);
}

bool resample_sg_tables(int up, int down, const float* h, int ntaps, float* tables, hipStream_t st,
                        hipError_t* err) {
  const int cmax = (ntaps + up - 1) / up;
  SgGeom G;
  if (up < 2 || ntaps != cmax * up || (cmax != 151 && cmax != 101) || !sg_geometry(up, down, cmax, &G)) return false;
  const long long n = (long long)G.npairs * 2 * 4 * G.nc;
  hipLaunchKernelGGL(build_sg_tables, dim3((unsigned)((n + kWG - 1) / kWG)), dim3(kWG), 0, st, h, up, down, cmax,
                     G.ncw, G.npairs, G.nc, G.slack, tables);
  *err = hipGetLastError();
  return true;
}

bool launch_resample_sg(int up, int down, const float* x, long long n, int nstreams, long long x_stride,
                        const float* h, int ntaps, float* state, int ns, float* y, long long y_stride, long long ny,
                        float* scratch, const float* tables, hipStream_t st, hipError_t* err) {
  if (!resample_sg_covers(up, down, ntaps, ns)) return false;
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (nstreams > 1 && x_stride % 4)) return false;
  const int cmax = ntaps / up;
  SgGeom G;
  sg_geometry(up, down, cmax, &G);
  const long long np = (ny + up - 1) / up;
  if (np * nstreams > 0x7fffffffLL - 64 || (long long)up * down > 0x7fffffffLL || n < ns) return false;
  if (!tables) {
    if (!resample_sg_tables(up, down, h, ntaps, scratch, st, err)) return false;
    if (*err != hipSuccess) return true;
    tables = scratch;
  }
  SgArgs a;
  a.x = x;
  a.n = n;
  a.x_stride = x_stride;
  a.tab = tables;
  a.state = state;
  a.ns = ns;
  a.y = y;
  a.y_stride = y_stride;
  a.ny = ny;
  a.up = up;
  a.down = down;
  a.cmax = cmax;
  a.np = (int)np;
  a.ncols = (int)(np * nstreams);
  const int nblk = (a.ncols + 63) / 64;
  a.ngrp = G.ngrp;
  a.ncw = G.ncw;
  a.npairs = G.npairs;
  a.slack = G.slack;
  a.segc = G.segc;
  a.stride = G.stride;
  a.nunits = nblk * G.ngrp;
  static const int ablate = env_int("SDR_ABLATE", 0);
  a.ablate = ablate;
  static const int gmajor = env_int("SDR_SG_GMAJOR", 0);
  static const int loaders = env_int("SDR_SG_LOADERS", 1);  // 0: every wave stages
  a.gmajor = gmajor;
  const int ncu = device_cu_count();
  const int grid = a.nunits < ncu ? a.nunits : ncu;
  const size_t lds = (size_t)2 * 64 * G.stride * sizeof(float);
  const dim3 blk(64 * (G.ncw + (loaders > 0 ? 1 : 0)));
  *err = cmax == 151 ? launch_sg_nc<151>(G, a, dim3((unsigned)grid), blk, lds, st)
                     : launch_sg_nc<101>(G, a, dim3((unsigned)grid), blk, lds, st);
  return true;
}

}  // namespace sdr
