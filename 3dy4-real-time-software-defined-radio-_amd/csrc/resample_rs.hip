// resample_rs.hip -- the polyphase resampler (src/filter.cpp:142-173) as a
// sliding-window kernel: every input sample is staged in LDS about once.
//
// Decomposition (see resample.hip for the phase algebra): output
// j = L*t + phi has phase p = (phi*M) mod L and newest input
// q = t*M + floor(phi*M/L).  A *column* is one period t of one stream; a
// workgroup owns 64 columns (lane = column) and walks ALL L phases of them
// in groups of 32 (wave w takes phases 32g + w and 32g + 16 + w: two
// independent accumulation chains per lane).  Consecutive phase groups need
// windows that slide right by ~32*M/L inputs, so each column keeps a ring of
// RING floats in LDS and only the new inputs of the next group are fetched
// (LDS-DMA, one wave-instruction per column) while the current group is
// computed.  Per-wave taps are SGPR operands read from a table pre-shifted
// by the wave's window alignment A, so the chunk -> tap mapping is the same
// for every A; the few out-of-range elements at the window ends are skipped
// by uniform branches (the reference's sum has exactly CMAX terms).
//
// Arithmetic contract as everywhere: per output, k ascending (i = 0..CMAX-1),
// separately rounded products and sums from 0.0f.
#include <cstdlib>
#include <type_traits>

#include "sdr_common.hpp"

#pragma clang fp contract(off)

namespace sdr {
namespace {

constexpr int kRsLanes = 64;
constexpr int kRsWaves = 16;
constexpr int kRsPG = 2 * kRsWaves;  // phases per group
constexpr int kRsRing = 512;         // floats per column ring (power of 2)
constexpr int kRsRingC = kRsRing / 4;
// column stride in LDS: one 16-B chunk of padding, so the 64 lanes' rings
// (same ring offset, different columns) start on different banks
constexpr int kRsColStride = kRsRing + 4;

// LDS-DMA writes are counted by vmcnt, which the workgroup fence of
// __syncthreads() does not wait for: every wave drains its own DMAs before a
// barrier that publishes them to the other waves.
__device__ __forceinline__ void dma_drain() { asm volatile("s_waitcnt vmcnt(0)" ::: "memory"); }

struct RsArgs {
  const float* x;
  long long n, x_stride;
  const float* hs;  // [4][L][U] taps pre-shifted by A: hs[A][p][u] = tap u + A - 3
  int U;            // row length (multiple of 4)
  int up, down;
  const float* state;
  int ns;
  float* y;
  long long y_stride, ny;
  int np;           // periods per stream
  int ncols;        // nstreams * np
  int ngrp;         // phase groups = ceil(up / kRsPG)
  int ablate;
};

// Ring-relative coordinates: rel = (input position) - t*M - base0 with
// base0 = -(CMAX-1) rounded down to a multiple of 4, so rel >= 0 for every
// input any phase of the column reads; chunk c = rel/4 lives in ring slot
// c mod (RING/4).

// One DMA wave-instruction per (column, chunk range): chunks [c0, c1) of ring
// coordinates (c = rel/4) of column cl.  Lanes past the range, and chunks that
// reach outside [0, n), are skipped here and written in rs_edge().
template <int CMAX>
__device__ __forceinline__ void rs_dma(const RsArgs& a, float* ring, int cb, int wv, int ln, int base0,
                                       int c0, int c1) {
  for (int cl = wv; cl < kRsLanes; cl += kRsWaves) {
    const int col = cb * kRsLanes + cl;
    if (col >= a.ncols) break;
    const int s = col / a.np, t = col - s * a.np;
    const float* xs = a.x + (long long)s * a.x_stride;
    float* col_ring = ring + cl * kRsColStride;
    // pieces of <= 64 chunks that do not cross the ring's end: the LDS
    // destination of lane k is always the (wave-uniform) base + 16*k
    for (int p0 = c0; p0 < c1;) {
      const int slot = p0 & (kRsRingC - 1);
      int len = c1 - p0;
      if (len > 64) len = 64;
      if (len > kRsRingC - slot) len = kRsRingC - slot;
      const long long g = (long long)t * a.down + base0 + 4 * (p0 + ln);  // input position of the chunk (multiple of 4)
      if (ln < len && g >= 0 && g + 4 <= a.n)
        __builtin_amdgcn_global_load_lds(xs + g, col_ring + 4 * slot, 16, 0, 0);
      p0 += len;
    }
  }
}

template <int CMAX>
__device__ __forceinline__ void rs_edge(const RsArgs& a, float* ring, int cb, int wv, int ln, int base0,
                                        int c0, int c1) {
  for (int cl = wv; cl < kRsLanes; cl += kRsWaves) {
    const int col = cb * kRsLanes + cl;
    if (col >= a.ncols) break;
    const int s = col / a.np, t = col - s * a.np;
    for (int c = c0 + ln; c < c1; c += 64) {
      const long long g = (long long)t * a.down + base0 + 4LL * c;
      if (!(g >= 0 && g + 4 <= a.n)) {
        const float* xs = a.x + (long long)s * a.x_stride;
        const float* st = a.state + (long long)s * a.ns;
        float w4[4];
#pragma unroll
        for (int r = 0; r < 4; ++r) {
          const long long gg = g + r;
          w4[r] = gg >= 0 ? (gg < a.n ? xs[gg] : 0.0f) : (gg >= -a.ns ? st[a.ns + gg] : 0.0f);
        }
        *reinterpret_cast<float4*>(ring + cl * kRsColStride + 4 * (c & (kRsRingC - 1))) =
            make_float4(w4[0], w4[1], w4[2], w4[3]);
      }
    }
  }
}

// Two phases of one wave over all shifted-tap chunks: element jj of chunk cc
// is tap i = 4*cc + A - jj of its phase (uniform A per phase), at ring chunk
// (ctop - cc) of the lane's ring; the four taps of chunk cc are one
// broadcast ds_read_b128 of the phase's LDS tap row (hs row u = 4cc..4cc+3).
template <int CMAX>
__device__ __forceinline__ void rs_scan(float& acc0, float& acc1, const float* lr, int ctop0, int ctop1, int A0,
                                        int A1, const float* t0row, const float* t1row) {
  constexpr int NC = (CMAX + 3 + 3) / 4;  // shifted-tap chunks (u < CMAX + 3)
  auto xchunk = [&](int ctop, int cc) {
    return *reinterpret_cast<const float4*>(lr + 4 * ((ctop - cc) & (kRsRingC - 1)));
  };
  float4 x0 = xchunk(ctop0, 0), x1 = xchunk(ctop1, 0);
  float4 h0 = *reinterpret_cast<const float4*>(t0row), h1 = *reinterpret_cast<const float4*>(t1row);
#pragma unroll
  for (int cc = 0; cc < NC; ++cc) {
    float4 nx0 = x0, nx1 = x1, nh0 = h0, nh1 = h1;
    if (cc + 1 < NC) {  // next chunk in flight while this one is multiplied
      nx0 = xchunk(ctop0, cc + 1);
      nx1 = xchunk(ctop1, cc + 1);
      nh0 = *reinterpret_cast<const float4*>(t0row + 4 * (cc + 1));
      nh1 = *reinterpret_cast<const float4*>(t1row + 4 * (cc + 1));
    }
    const float e0[4] = {x0.x, x0.y, x0.z, x0.w}, e1[4] = {x1.x, x1.y, x1.z, x1.w};
    // shifted row: u = 4cc + 3 - jj, so element jj pairs with component 3 - jj
    const float g0[4] = {h0.w, h0.z, h0.y, h0.x}, g1[4] = {h1.w, h1.z, h1.y, h1.x};
#pragma unroll
    for (int jj = 3; jj >= 0; --jj) {
      // i = 4*cc + A - jj must lie in [0, CMAX): only the end chunks can miss.
      // There the shifted tap is 0 and the ring element is replaced by 0, so
      // the term is +0 and acc + 0 == acc exactly (acc starts at +0 and can
      // never become -0): the sum keeps exactly the reference's CMAX terms,
      // without branches.
      float a0 = e0[jj], a1 = e1[jj];
      if ((cc == 0) || (4 * cc + 3 - jj >= CMAX)) {
        a0 = (4 * cc + A0 - jj >= 0 && 4 * cc + A0 - jj < CMAX) ? a0 : 0.0f;
        a1 = (4 * cc + A1 - jj >= 0 && 4 * cc + A1 - jj < CMAX) ? a1 : 0.0f;
      }
      acc0 = acc0 + g0[jj] * a0;
      acc1 = acc1 + g1[jj] * a1;
    }
    x0 = nx0;
    x1 = nx1;
    h0 = nh0;
    h1 = nh1;
    asm volatile("" : "+v"(acc0), "+v"(acc1));
    __builtin_amdgcn_sched_barrier(0);
  }
}

template <int CMAX>
__global__ __launch_bounds__(64 * kRsWaves, 1) void resample_rs(RsArgs a) {
  __shared__ __attribute__((aligned(16))) float ring[kRsLanes * kRsColStride];
  constexpr int U = (CMAX + 3 + 3) / 4 * 4;                 // shifted row length
  constexpr int TPT = (kRsPG * U + 64 * kRsWaves - 1) / (64 * kRsWaves);  // tap floats per thread
  __shared__ __attribute__((aligned(16))) float trow[kRsPG * U];  // this group's rows, pre-shifted
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), ln = threadIdx.x & 63;
  const int ncb = (a.ncols + kRsLanes - 1) / kRsLanes;
  const int per = (ncb + (int)gridDim.x - 1) / (int)gridDim.x;
  const int cbA = (int)blockIdx.x * per;
  const int cbB = cbA + per < ncb ? cbA + per : ncb;
  if (cbA >= cbB) return;
  // ring coordinates: rel = pos - t*M - base0, base0 = -(CMAX-1) rounded down to a multiple of 4
  constexpr int base0 = -(((CMAX - 1) + 3) / 4 * 4);
  // chunk range [lo, hi) of rel/4 that phase group g needs: its lowest phase's
  // oldest input .. its highest phase's newest input (phi*M < 2^31 on every path)
  auto need = [&](int g, int& lo, int& hi) {
    const int p0 = g * kRsPG;
    const int p1 = min(p0 + kRsPG, a.up) - 1;
    const int q0 = p0 * a.down / a.up, q1 = p1 * a.down / a.up;
    lo = (q0 - (CMAX - 1) - base0) >> 2;
    hi = ((q1 - base0) >> 2) + 1;
  };
  const int lane_ring = ln * kRsColStride;
  // group g's tap rows: trow[k*U + u] = hs[A(phi)][p(phi)][u], phi = 32g + k
  auto fetch_taps = [&](int g, float (&tv)[TPT]) {
#pragma unroll
    for (int r = 0; r < TPT; ++r) {
      const int idx = threadIdx.x + r * 64 * kRsWaves;
      tv[r] = 0.0f;
      if (idx < kRsPG * U) {
        const int k = idx / U, u = idx - k * U;
        const int phi = g * kRsPG + k;
        if (phi < a.up) {
          const int q = phi * a.down / a.up;
          const int A = (q - base0) & 3;
          const int p = phi * a.down % a.up;
          tv[r] = a.hs[(A * a.up + p) * a.U + u];
        }
      }
    }
  };
  auto store_taps = [&](const float (&tv)[TPT]) {
#pragma unroll
    for (int r = 0; r < TPT; ++r) {
      const int idx = threadIdx.x + r * 64 * kRsWaves;
      if (idx < kRsPG * U) trow[idx] = tv[r];
    }
  };
  float tv[TPT];

  for (int cb = cbA; cb < cbB; ++cb) {
    // a new column block: the first group's whole window
    int lo, hi;
    need(0, lo, hi);
    if (SDR_ABL(a.ablate) != 1) {
      rs_dma<CMAX>(a, ring, cb, wv, ln, base0, lo, hi);
      rs_edge<CMAX>(a, ring, cb, wv, ln, base0, lo, hi);
    }
    fetch_taps(0, tv);
    store_taps(tv);
    dma_drain();
    __syncthreads();
    int have = hi;  // chunks [.., have) of this block are in the rings
    for (int g = 0; g < a.ngrp; ++g) {
      // the next group's new chunks are fetched while this group computes
      int nlo = 0, nhi = 0;
      const bool more = g + 1 < a.ngrp;
      if (more) {
        need(g + 1, nlo, nhi);
        nlo = have;
        if (SDR_ABL(a.ablate) != 1 && nhi > nlo) rs_dma<CMAX>(a, ring, cb, wv, ln, base0, nlo, nhi);
        fetch_taps(g + 1, tv);  // registers; written to LDS after this group is done
      }
      // this wave's two phases
      const int pa = g * kRsPG + wv, pb = pa + kRsWaves;
      if (pa < a.up && SDR_ABL(a.ablate) != 2) {
        const bool on1 = pb < a.up;
        const int pbb = on1 ? pb : pa;
        const int qa = pa * a.down / a.up, qb = pbb * a.down / a.up;
        const int e1a = qa - base0, e1b = qb - base0;  // ring rel of the newest input
        const int Aa = e1a & 3, Ab = e1b & 3;
        // the shifted row puts tap i at u = i + 3 - A, input rel e1 - i = 4*(e1 >> 2) + 3 - u:
        // chunk cc (u = 4cc..4cc+3) is ring chunk (e1 >> 2) - cc
        const int ctopa = e1a >> 2, ctopb = e1b >> 2;
        float acc0 = 0.0f, acc1 = 0.0f;
        rs_scan<CMAX>(acc0, acc1, ring + lane_ring, ctopa, ctopb, Aa, Ab, trow + wv * U,
                      trow + (on1 ? wv + kRsWaves : wv) * U);
        const int col = cb * kRsLanes + ln;
        if (col < a.ncols) {
          const int s = col / a.np, t = col - s * a.np;
          const long long ja = (long long)a.up * t + pa, jb = (long long)a.up * t + pb;
          float* ys = a.y + (long long)s * a.y_stride;
          if (ja < a.ny) ys[ja] = acc0;
          if (on1 && jb < a.ny) ys[jb] = acc1;
        }
      }
      if (more && SDR_ABL(a.ablate) != 1 && nhi > nlo) rs_edge<CMAX>(a, ring, cb, wv, ln, base0, nlo, nhi);
      if (more) have = nhi > have ? nhi : have;
      dma_drain();
      __syncthreads();  // the next group's chunks have landed; this group's reads are done
      if (more) {
        store_taps(tv);
        __syncthreads();
      }
    }
  }
}

// hs[A][p][u] = h[p + (u + A - 3) * L] for 0 <= u + A - 3 < CMAX, else 0.
__global__ __launch_bounds__(kWG) void build_shifted(const float* __restrict__ h, int ntaps, int up, int cmax,
                                                     int U, float* hs) {
  const long long idx = (long long)blockIdx.x * kWG + threadIdx.x;
  const long long tot = 4LL * up * U;
  if (idx >= tot) return;
  const int u = (int)(idx % U);
  const int p = (int)((idx / U) % up);
  const int A = (int)(idx / ((long long)U * up));
  const int i = u + A - 3;
  const long long k = (long long)p + (long long)i * up;
  hs[idx] = (i >= 0 && i < cmax && k < ntaps) ? h[k] : 0.0f;
}

// ---------------------------------------------------------------------------
// resample_lp: lane = (phase, column subset), taps in VGPRs.
//
// Workgroup = 7 waves = 448 lanes; lane slots hold (phi, sub) items, phi < L,
// sub < S = floor(448 / L) (S = 3 at L = 147).  A lane keeps its phase's
// shifted tap row (U floats) in VGPRs for the whole launch and computes the
// outputs of that phase for columns c = sub + S*k, k < K (K accumulation
// chains), reading its inputs from an LDS image of the item's span with
// 16-B ds_read_b128 (aligned because the row is pre-shifted by the lane's
// A).  Per multiply-add only 4 B of LDS are read (no tap traffic), which is
// half of what the column-lane kernels above read.  Work item = (stream,
// batch of up to S*K consecutive columns); the next item's span is brought
// in by LDS-DMA into the other buffer while the current one is computed.
//
// Lane placement: ds_read_b128 serves a wave in four groups of 16 lanes, and
// two lanes of one group conflict when their chunk indices differ by a
// multiple of 16 (64 banks).  A lane's chunk index mod 16 is fixed for the
// launch ((sub*M/4 + ctop(phi)) mod 16, the column stride adds the same
// amount to every lane), so build_lanes() sorts the items by that class and
// deals them round-robin over the 28 groups: a group gets two items of one
// class only when the class has more than 28 items.
// SDR_LP_EARLY: the loader wave issues the next item's DMAs before the edge
// loads and the state copy (0.1207-0.1211 vs 0.1206-0.1236 ms on cfg3, same
// box, profiles/r04f/ab_resample_loader.txt).  The ordered scan (the K
// products, then the K sums, inline asm) made the scan alone 5 % faster
// (0.1018 vs 0.1072 ms without staging) and the kernel 3 % slower
// (profiles/r04f/ab_resample_ord.txt); not kept.
#ifndef SDR_LP_EARLY
#define SDR_LP_EARLY 1
#endif
// SDR_LP_NT: the items' LDS-DMA with the non-temporal policy (each input is
// read once; MI355X_MICROARCH.md's nt-weights row: issued -> landed -18 %):
// cfg3 0.1171-0.1192 vs 0.1170-0.1202 ms, neutral (profiles/r04f/), off
#ifndef SDR_LP_NT
#define SDR_LP_NT 0
#endif
// Round 5 (code at 821f6db): the scan software-pipelined by
// one tap (each add 2K-1 instructions after its multiply) measured 0.1203-
// 0.1226 vs 0.1172-0.1189 ms, and the next item's DMAs split between the
// loader and the compute wave on its SIMD 0.143-0.145 ms: neither kept.
constexpr int kLpWaves = 7;
constexpr int kLpSlots = 64 * kLpWaves;
constexpr int kLpGroups = kLpSlots / 16;
constexpr int kLpBuf = 19456;  // floats per staging buffer (76 KiB); two buffers

struct LpArgs {
  const float* x;
  long long n, x_stride;
  const float* hs;   // [4][L][U] taps pre-shifted by A (build_lp_tables)
  const int* lanes;  // [kLpSlots]: phi | sub << 16, or -1 (build_lp_tables)
  int up, down;
  float* state;      // read by each stream's first item, then rewritten by it
  int ns;
  float* y;
  long long y_stride, ny;
  int np;      // columns (periods) per stream
  int C;       // columns per item
  int nbat;    // items per stream
  int nitems;  // nstreams * nbat
  int S;       // column subsets
  int ablate;
};

// lanes of each ds_read_b128 lane group (MI355X_MICROARCH.md, LDS table)
__constant__ unsigned char kB128Groups[4][16] = {
    {0, 1, 2, 3, 12, 13, 14, 15, 20, 21, 22, 23, 24, 25, 26, 27},
    {4, 5, 6, 7, 8, 9, 10, 11, 16, 17, 18, 19, 28, 29, 30, 31},
    {32, 33, 34, 35, 44, 45, 46, 47, 52, 53, 54, 55, 56, 57, 58, 59},
    {36, 37, 38, 39, 40, 41, 42, 43, 48, 49, 50, 51, 60, 61, 62, 63}};

// Every workgroup builds the lane table itself (448 items, LDS atomics):
// counting sort of the L*S items by bank class, then deal round-robin over
// the 28 lane groups.  Which lane gets which item does not change any
// output bit (each output is computed by exactly one lane, in the same
// order), so the atomics' nondeterminism is harmless.
__device__ __forceinline__ int lp_lane_code(int up, int down, int S, int base0, int* cnt, int* start, int* fill,
                                            int* order, int* codes) {
  const int t = threadIdx.x;
  const int nit = up * S;
  if (t < 16) {
    cnt[t] = 0;
    fill[t] = 0;
  }
  codes[t] = -1;
  __syncthreads();
  int cls = -1;
  if (t < nit) {
    const int phi = t % up, sub = t / up;
    const int q = (int)((long long)phi * down / up);
    cls = ((sub * (down / 4)) + ((q - base0) >> 2)) & 15;
    atomicAdd(&cnt[cls], 1);
  }
  __syncthreads();
  if (t == 0) {
    int acc = 0;
    for (int c = 0; c < 16; ++c) {
      start[c] = acc;
      acc += cnt[c];
    }
  }
  __syncthreads();
  if (t < nit) order[start[cls] + atomicAdd(&fill[cls], 1)] = t;
  __syncthreads();
  if (t < nit) {
    // position r in class order -> group r mod 28, member r / 28
    const int g = t % kLpGroups, m = t / kLpGroups;
    const int item = order[t];
    codes[(g >> 2) * 64 + kB128Groups[g & 3][m]] = (item % up) | ((item / up) << 16);
  }
  __syncthreads();
  // A slot left empty still issues the scan's reads: as (0, 0) it would add a
  // second address of one bank class to its lane group -- one extra LDS
  // cycle on every ds_read_b128 of that group (the 448 - 441 empty slots at
  // L = 147 sit in 7 of the 28 groups: ~23 % SQ_LDS_BANK_CONFLICT).  It
  // shadows its group's first member instead (same address = a broadcast)
  // and is flagged 0x8000 so it stores nothing.
  int code = codes[t];
  if (code < 0) {
    const int l = t & 63, w = t >> 6;
    for (int g4 = 0; g4 < 4; ++g4)
      for (int m = 0; m < 16; ++m)
        if (kB128Groups[g4][m] == l) {
          const int twin = codes[w * 64 + kB128Groups[g4][0]];
          if (twin >= 0) code = twin | 0x8000;
        }
  }
  return code;
}

// One launch for both tables of resample_lp: blocks 0..G-2 write the shifted
// rows hs[A][p][u] = h[p + (u + A - 3) * L] (0 where u + A - 3 is outside
// [0, CMAX)), the last block builds the lane table.
__global__ __launch_bounds__(kLpSlots) void build_lp_tables(const float* __restrict__ h, int up, int down, int cmax,
                                                            int U, int S, int base0, float* __restrict__ hs,
                                                            int* __restrict__ lanes) {
  if (blockIdx.x == gridDim.x - 1) {
    __shared__ int cnt[16], start[16], fill[16], order[kLpSlots], codes[kLpSlots];
    lanes[threadIdx.x] = lp_lane_code(up, down, S, base0, cnt, start, fill, order, codes);
    return;
  }
  const long long idx = (long long)blockIdx.x * kLpSlots + threadIdx.x;
  if (idx >= 4LL * up * U) return;
  const int u = (int)(idx % U);
  const int p = (int)((idx / U) % up);
  const int A = (int)(idx / ((long long)U * up));
  const int i = u + A - 3;
  hs[idx] = (i >= 0 && i < cmax) ? h[p + (long long)i * up] : 0.0f;
}

// Stage item `it` (its whole input span) into buf: LDS-DMA for the chunks
// inside [0, n), registers for the chunks that reach into the carried state
// or past the end.
// The staging threads: tid of nth, in waves wv of nwv (all of the compute
// waves, or the one loader wave).
template <int CMAX, bool DMA_FIRST = false>
__device__ __forceinline__ void lp_stage(const LpArgs& a, float* buf, int it, int tid, int nth, int wv, int nwv,
                                         int ln) {
  constexpr int base0 = -(((CMAX - 1) + 3) / 4 * 4);
  const int st = it / a.nbat, b = it - st * a.nbat;
  const int t0 = b * a.C;
  const int ce = min(a.C, a.np - t0);
  const long long P0 = (long long)t0 * a.down + base0;
  const int qmax = (int)((long long)(a.up - 1) * a.down / a.up);
  const int W = (ce - 1) * a.down + qmax + 1 - base0;
  const int nch = (W + 3) >> 2;
  const float* xs = a.x + (long long)st * a.x_stride;
  // DMA: chunk j covers positions P0 + 4j .. +3; lanes of one instruction are consecutive chunks
  const long long jlo = P0 < 0 ? (-P0 + 3) >> 2 : 0;          // first chunk with g >= 0
  long long jhi = (a.n - P0) >> 2;                             // chunks j < jhi end inside [0, n)
  if (jhi > nch) jhi = nch;
  // edges first (chunks below jlo and from jhi up): their register loads then
  // do not wait behind this item's DMAs
  auto edge = [&](int j) {
    const long long g = P0 + 4LL * j;
    float w4[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
      const long long gg = g + r;
      w4[r] = gg >= 0 ? (gg < a.n ? xs[gg] : 0.0f) : (gg >= -a.ns ? a.state[(long long)st * a.ns + a.ns + gg] : 0.0f);
    }
    *reinterpret_cast<float4*>(buf + 4 * j) = make_float4(w4[0], w4[1], w4[2], w4[3]);
  };
  auto dma = [&]() __attribute__((always_inline)) {
    // lanes of one instruction are consecutive chunks
    for (int j0 = (int)(jlo & ~63LL) + wv * 64; j0 < jhi; j0 += 64 * nwv) {
      const int j = j0 + ln;
      if (j >= jlo && j < jhi) __builtin_amdgcn_global_load_lds(xs + P0 + 4LL * j, buf + 4 * j0, 16, 0, SDR_LP_NT ? 2 : 0);
    }
  };
  // DMA_FIRST (the loader wave, which waits for nothing else): the span's
  // DMAs go out before the edge loads, whose waits then cover the DMAs too
  // but no longer hold back their issue by a memory latency on every
  // stream's first item
  if constexpr (DMA_FIRST) dma();
  for (int j = tid; j < (int)jlo && j < nch; j += nth) edge(j);
  for (int j = (int)(jhi > jlo ? jhi : jlo) + tid; j < nch; j += nth) edge(j);
  if constexpr (!DMA_FIRST) dma();
}

template <int CMAX, int K, int LW, int NOLDS = 0>
__device__ __forceinline__ void lp_compute(const LpArgs& a, const float* buf, int it, const float (&tp)[(CMAX + 6) / 4 * 4],
                                           int phi, int sub, int A, int ctop0, bool valid) {
  constexpr int NC = (CMAX + 6) / 4;
  const int st = it / a.nbat, b = it - st * a.nbat;
  const int t0 = b * a.C;
  const int ce = min(a.C, a.np - t0);
  typedef float f4v __attribute__((ext_vector_type(4)));
  typedef __attribute__((address_space(3))) const f4v lds4;
  lds4* ptr[K];  // chunk (ctop - (NC-1)) of each chain; chunk ctop - cc sits at ptr + (NC-1-cc)
  bool act[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const int c = sub + a.S * k;
    act[k] = valid && c < ce;
    // an idle chain (ragged last item) reads a column of the same parity: the
    // chunk's bank class is 8*column + const (mod 16, down/4 = 200 at cfg3),
    // so its lane keeps its class and adds no conflict
    const int cc = c < ce ? c : ((c & 1) < ce ? (c & 1) : 0);
    ptr[k] = (lds4*)(buf + 4 * (cc * (a.down >> 2) + ctop0 - (NC - 1)));
    asm volatile("" : "+v"(ptr[k]));  // keep the base in a VGPR: per-chunk offsets stay immediates
  }
  float acc[K];
  f4v cur[K], nxt[K];
#pragma unroll
  for (int k = 0; k < K; ++k) {
    acc[k] = 0.0f;
    cur[k] = ptr[k][NC - 1];
  }
#pragma unroll
  for (int cc = 0; cc < NC; ++cc) {
    // the next chunk's reads go out first; this chunk's were issued one chunk ago
    if (cc + 1 < NC) {
#pragma unroll
      for (int k = 0; k < K; ++k) {
        if constexpr (NOLDS) {
          // timing ablation (SDR_ABLATE=4): the scan without its LDS reads
          nxt[k] = cur[k];
          asm volatile("" : "+v"(nxt[k]));
        } else {
          nxt[k] = ptr[k][NC - 2 - cc];
        }
      }
    }
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int jj = 3; jj >= 0; --jj) {
      const int u = 4 * cc + 3 - jj;
      // i = u + A - 3 must lie in [0, CMAX) -- only at the two ends; there the
      // shifted tap is 0 and the input is replaced by 0 (term +0: acc unchanged)
      const bool edge = (cc == 0) || (u >= CMAX);
      const bool ok = !edge || (u + A - 3 >= 0 && u + A - 3 < CMAX);
#pragma unroll
      for (int k = 0; k < K; ++k) {
        float v = cur[k][jj];
        if (edge) v = ok ? v : 0.0f;
        acc[k] = acc[k] + tp[u] * v;
      }
    }
#pragma unroll
    for (int k = 0; k < K; ++k) {
      cur[k] = nxt[k];
      asm volatile("" : "+v"(acc[k]));
    }
    __builtin_amdgcn_sched_barrier(0);
  }
  // The next item's DMAs (issued before this scan) are waited for here,
  // before the output stores: vmcnt also counts stores, so a drain after them
  // would wait out their write latency too.  (LW: the loader wave stages.)
  if (!LW) dma_drain();
  float* ys = a.y + (long long)st * a.y_stride;
#pragma unroll
  for (int k = 0; k < K; ++k) {
    const long long j = (long long)a.up * (t0 + sub + a.S * k) + phi;
    if (act[k] && j < a.ny) ys[j] = acc[k];
  }
}

// LW = 1: an eighth wave stages every item (and commits the state) while
// the seven compute waves only scan: the DMA issue -- 3-4 k cycles of each
// compute wave's item time -- leaves their instruction
// streams; its registers come free with the 2-waves-per-SIMD allocation.
template <int CMAX, int K, int LW, int NOLDS = 0>
__global__ __launch_bounds__(kLpSlots + 64 * LW, 1) void resample_lp(LpArgs a) {
  __shared__ __attribute__((aligned(16))) float bufA[kLpBuf];
  __shared__ __attribute__((aligned(16))) float bufB[kLpBuf];
  __shared__ float cbuf[kLpSlots];  // the new state, in flight during the compute
  constexpr int U = (CMAX + 6) / 4 * 4;
  constexpr int base0 = -(((CMAX - 1) + 3) / 4 * 4);
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), ln = threadIdx.x & 63;
  const bool loader = LW && wv == kLpWaves;  // wave-uniform
  // items: contiguous range per workgroup
  const int per = a.nitems / (int)gridDim.x, extra = a.nitems % (int)gridDim.x;
  const int i0 = (int)blockIdx.x * per + min((int)blockIdx.x, extra);
  const int i1 = i0 + per + ((int)blockIdx.x < extra ? 1 : 0);
  if (i0 >= i1) return;
  auto stage = [&](float* buf, int it) __attribute__((always_inline)) {
    if (SDR_ABL(a.ablate) == 1) return;
    if (!LW)
      lp_stage<CMAX>(a, buf, it, threadIdx.x, kLpSlots, wv, kLpWaves, ln);
    else if (loader)
      lp_stage<CMAX, SDR_LP_EARLY != 0>(a, buf, it, ln, 64, 0, 1, ln);
  };
  // the first item's DMA runs while this lane's item and taps are loaded
  stage(bufA, i0);
  const int code = loader ? -1 : a.lanes[threadIdx.x];
  const bool valid = code >= 0 && !(code & 0x8000);  // 0x8000: an empty slot shadowing a twin
  const int phi = code >= 0 ? (code & 0x7fff) : 0, sub = code >= 0 ? (code >> 16) : 0;
  const int q = (int)((long long)phi * a.down / a.up);
  const int A = (q - base0) & 3, ctop0 = (q - base0) >> 2;
  const int p = (int)((long long)phi * a.down % a.up);
  float tp[U];
  const float* row = a.hs + ((long long)A * a.up + p) * U;
  if (!loader) {
#pragma unroll
    for (int u = 0; u < U; u += 4) {
      const float4 v = *reinterpret_cast<const float4*>(row + u);
      tp[u] = v.x;
      tp[u + 1] = v.y;
      tp[u + 2] = v.z;
      tp[u + 3] = v.w;
    }
  }
  for (int it = i0; it < i1; ++it) {
    // (the previous item drained its DMAs before its output stores; the
    // loader drains its own here)
    if (it == i0 || SDR_ABL(a.ablate) == 2 || loader) dma_drain();
    __syncthreads();  // item it's span has landed; the other buffer is free
    // the stream's first item is the only reader of its old state and its span
    // is staged now: state <- last ns inputs of the block (src/filter.cpp:169)
    // (ns <= kLpSlots on this path).  LW: the loader copies it directly
    // (its own edge loads read the old state, before this); else it is
    // brought into LDS by DMA during the compute and stored after it.
    const bool commit = it % a.nbat == 0;
    const bool odd = ((it - i0) & 1) != 0;
    // SDR_LP_EARLY (loader wave): the next item's DMAs before this item's
    // state copy, whose load-to-store wait would otherwise hold them back
    if (SDR_LP_EARLY && LW && it + 1 < i1) stage(odd ? bufA : bufB, it + 1);
    if (LW) {
      if (loader && commit) {
        const long long s = it / a.nbat;
        for (int j = ln; j < a.ns; j += 64) a.state[s * a.ns + j] = a.x[s * a.x_stride + (a.n - a.ns) + j];
      }
    } else if (commit && (int)threadIdx.x < a.ns) {
      __builtin_amdgcn_global_load_lds(a.x + (long long)(it / a.nbat) * a.x_stride + (a.n - a.ns) + threadIdx.x,
                                       cbuf + wv * 64, 4, 0, 0);
    }
    if (!(SDR_LP_EARLY && LW) && it + 1 < i1) stage(odd ? bufA : bufB, it + 1);
    if (SDR_ABL(a.ablate) != 2 && !loader) {
      if (odd)
        lp_compute<CMAX, K, LW, NOLDS>(a, bufB, it, tp, phi, sub, A, ctop0, valid);
      else
        lp_compute<CMAX, K, LW, NOLDS>(a, bufA, it, tp, phi, sub, A, ctop0, valid);
    }
    if (!LW && commit && (int)threadIdx.x < a.ns) {
      dma_drain();
      a.state[(long long)(it / a.nbat) * a.ns + threadIdx.x] = cbuf[threadIdx.x];
    }
  }
}

// switches SDR_RESAMPLE_LP / _LOADER / _RS (the tests run every resampler kernel)
bool lp_enabled() { return sw(kSwResampleLp) != 0; }
bool lp_loader() { return sw(kSwResampleLoader) != 0; }
bool rs_enabled() { return sw(kSwResampleRs) != 0; }

}  // namespace

size_t resample_rs_scratch_floats(int up, int ntaps) {
  const int cmax = (ntaps + up - 1) / up;
  const int U = (cmax + 3 + 3) / 4 * 4;
  return (size_t)4 * up * U + kLpSlots;  // shifted rows (+ resample_lp's lane table)
}

// Returns false (nothing launched) when the shape is not one this kernel
// covers; the caller then takes the phase-major kernel of resample.hip.
bool resample_lp_tables(int up, int down, const float* h, int ntaps, int ns, float* tables, hipStream_t st,
                        hipError_t* err) {
  const int cmax = (ntaps + up - 1) / up;
  if (up < 2 || ntaps != cmax * up || (cmax != 151 && cmax != 101) || down % 4 != 0) return false;
  const int base0 = -(((cmax - 1) + 3) / 4 * 4);
  const int qmax = (int)((long long)(up - 1) * down / up);
  if (!(up <= kLpSlots && (long long)up * down < (1LL << 31) && qmax + 1 - base0 + 4 <= kLpBuf && ns <= kLpSlots))
    return false;
  const int S = kLpSlots / up;
  const int U = (cmax + 6) / 4 * 4;
  const long long tab = 4LL * up * U;
  int* lanes = reinterpret_cast<int*>(tables + tab);
  hipLaunchKernelGGL(build_lp_tables, dim3((unsigned)((tab + kLpSlots - 1) / kLpSlots + 1)), dim3(kLpSlots), 0, st, h,
                     up, down, cmax, U, S, base0, tables, lanes);
  *err = hipGetLastError();
  return true;
}

bool launch_resample_rs(int up, int down, const float* x, long long n, int nstreams, long long x_stride,
                        const float* h, int ntaps, float* state, int ns, float* y, long long y_stride, long long ny,
                        float* scratch, hipStream_t st, hipError_t* err, bool* state_done, const float* lp_tables) {
  *state_done = false;
  const int cmax = (ntaps + up - 1) / up;
  if (up < 2 || ntaps != cmax * up || (cmax != 151 && cmax != 101) || down % 4 != 0) return false;
  // 16-B chunks straight from the rows
  if ((reinterpret_cast<uintptr_t>(x) & 15) || (nstreams > 1 && x_stride % 4)) return false;
  // resample_lp: the staging buffer must hold at least one column's span
  const int base0 = -(((cmax - 1) + 3) / 4 * 4);
  const int qmax = (int)((long long)(up - 1) * down / up);
  bool use_lp = lp_enabled() && up <= kLpSlots && (long long)up * down < (1LL << 31) &&
                qmax + 1 - base0 + 4 <= kLpBuf && ns <= kLpSlots;
  const int np = (int)((ny + up - 1) / up);
  // resample_lp's columns per item: S*K chains, bounded by the staging buffer
  const int lpS = kLpSlots / up;
  const int lpK = (np <= 4 * lpS) ? 4 : 7;
  int lpC = lpS * lpK;
  {
    const long long fit = (kLpBuf - (qmax + 1 - base0) - 4) / down + 1;
    if (lpC > fit) lpC = (int)fit;
    if (lpC > np) lpC = np;
    if (lpC < 1) lpC = 1;
  }
  // resample_lp commits a stream's new state in its first item, at the top of
  // that item's iteration; that is only safe when the first item is the ONLY
  // reader of the old state, i.e. the second item's span starts at p >= 0
  // (up = 128, down = 4 gives C = 21, P0 = 21*4 - 152 < 0).
  if (use_lp && np > lpC && (long long)lpC * down + base0 < 0) use_lp = false;

  // resample_rs: the ring must hold a group's whole window plus the next group's new inputs
  const long long span = ((long long)(kRsPG - 1) * down + up - 1) / up + cmax + 8;
  const long long step = ((long long)kRsPG * down + up - 1) / up + 8;
  if (!use_lp && (!rs_enabled() || span + step > kRsRing)) return false;
  static const int ablate = SDR_TIMING_ENV("SDR_ABLATE", 0);
  const int ncu = device_cu_count();
  if (use_lp) {
    const int S = lpS, K = lpK, C = lpC;
    {
      LpArgs b;
      b.x = x;
      b.n = n;
      b.x_stride = x_stride;
      // tables built once by a plan (resample_lp_tables), or here for this call
      const float* tables = lp_tables ? lp_tables : scratch;
      b.hs = tables;
      b.lanes = reinterpret_cast<const int*>(tables + 4LL * up * ((cmax + 6) / 4 * 4));
      b.up = up;
      b.down = down;
      b.state = state;
      b.ns = ns;
      b.y = y;
      b.y_stride = y_stride;
      b.ny = ny;
      b.np = np;
      b.C = C;
      b.nbat = (np + C - 1) / C;
      b.nitems = b.nbat * nstreams;
      b.S = S;
      b.ablate = ablate;
      const int U = (cmax + 6) / 4 * 4;
      const long long tab = 4LL * up * U;
      if (!lp_tables) {
        hipLaunchKernelGGL(build_lp_tables, dim3((unsigned)((tab + kLpSlots - 1) / kLpSlots + 1)), dim3(kLpSlots), 0,
                           st, h, up, down, cmax, U, S, base0, scratch, reinterpret_cast<int*>(scratch + tab));
        if ((*err = hipGetLastError()) != hipSuccess) return true;
      }
      const int grid = b.nitems < ncu ? b.nitems : ncu;
      const dim3 g((unsigned)grid);
#ifdef SDR_TIMING_BUILD
      if (ablate == 4 && cmax == 151 && K == 7) {
        // timing ablation: no staging and no LDS reads in the scan
        b.ablate = 1;
        hipLaunchKernelGGL((resample_lp<151, 7, 1, 1>), g, dim3(kLpSlots + 64), 0, st, b);
      } else
#endif
      if (lp_loader()) {
        const dim3 blk(kLpSlots + 64);
        if (cmax == 151) {
          if (K == 4)
            hipLaunchKernelGGL((resample_lp<151, 4, 1>), g, blk, 0, st, b);
          else
            hipLaunchKernelGGL((resample_lp<151, 7, 1>), g, blk, 0, st, b);
        } else {
          if (K == 4)
            hipLaunchKernelGGL((resample_lp<101, 4, 1>), g, blk, 0, st, b);
          else
            hipLaunchKernelGGL((resample_lp<101, 7, 1>), g, blk, 0, st, b);
        }
      } else {
        const dim3 blk(kLpSlots);
        if (cmax == 151) {
          if (K == 4)
            hipLaunchKernelGGL((resample_lp<151, 4, 0>), g, blk, 0, st, b);
          else
            hipLaunchKernelGGL((resample_lp<151, 7, 0>), g, blk, 0, st, b);
        } else {
          if (K == 4)
            hipLaunchKernelGGL((resample_lp<101, 4, 0>), g, blk, 0, st, b);
          else
            hipLaunchKernelGGL((resample_lp<101, 7, 0>), g, blk, 0, st, b);
        }
      }
      *err = hipGetLastError();
      *state_done = true;  // resample_lp commits the state itself
      return true;
    }
  }
  const int U = (cmax + 3 + 3) / 4 * 4;
  const long long tab = 4LL * up * U;
  hipLaunchKernelGGL(build_shifted, dim3((unsigned)((tab + kWG - 1) / kWG)), dim3(kWG), 0, st, h, ntaps, up, cmax, U,
                     scratch);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) {
    *err = e;
    return true;
  }
  RsArgs a;
  a.x = x;
  a.n = n;
  a.x_stride = x_stride;
  a.hs = scratch;
  a.U = U;
  a.up = up;
  a.down = down;
  a.state = state;
  a.ns = ns;
  a.y = y;
  a.y_stride = y_stride;
  a.ny = ny;
  a.np = np;
  if ((long long)a.np * nstreams > 0x7fffffffLL - kRsLanes || (long long)up * down > 0x7fffffffLL) return false;
  a.ncols = a.np * nstreams;
  a.ngrp = (up + kRsPG - 1) / kRsPG;
  a.ablate = ablate;
  const int ncb = (a.ncols + kRsLanes - 1) / kRsLanes;
  const int grid = ncb < ncu ? ncb : ncu;
  if (cmax == 151)
    hipLaunchKernelGGL(resample_rs<151>, dim3((unsigned)grid), dim3(64 * kRsWaves), 0, st, a);
  else
    hipLaunchKernelGGL(resample_rs<101>, dim3((unsigned)grid), dim3(64 * kRsWaves), 0, st, a);
  *err = hipGetLastError();
  return true;
}

}  // namespace sdr
