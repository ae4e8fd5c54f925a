// resample.hip -- polyphase rational resampler, the reference's
// resampleBlockConvolveFIR (src/filter.cpp:142-173), for up > 1.
// (up == 1 is FIR+decimate by `down` and takes the tiled FIR path.)
//
// Reference loop, restated per output j (n = j*down):
//   p = n mod up,  q = n div up
//   y[j] = sum_{i: k = p + i*up < T} h[k] * x~[q - i]     (ascending k)
// with x~[i] = x[i] for i >= 0 and state[ns + i] before the block (the
// reference's state[state.size() - (k-n)/up]).  Same fp32 op order as the
// reference: separately rounded products and sums from 0.0f.
//
// Layout: a 256-thread workgroup takes 256 consecutive outputs of one
// stream.  Their input windows [q_j - (cnt-1), q_j] overlap heavily
// (consecutive q differ by down/up ~ 5.4 samples at 147/800), so the
// workgroup stages the union of them once in LDS with coalesced loads; each
// lane then walks its own window from LDS.  The taps are re-laid out as a
// polyphase table hp[p][i] = h[p + i*up] (built once per call into device
// scratch) so each lane streams its branch contiguously (16-B loads, L1/L2
// resident: the whole table is T floats).
#include <algorithm>
#include <cstdlib>
#include <type_traits>

#include "sdr_common.hpp"

#pragma clang fp contract(off)

namespace sdr {
namespace {

constexpr int kMaxSpan = 8192;  // LDS floats per workgroup for the staged window

// hp[p*cmax + i] = h[p + i*up] for p + i*up < T, else 0 (never read).
__global__ __launch_bounds__(kWG) void build_polyphase(const float* __restrict__ h, int ntaps, int up, int cmax,
                                                       float* hp) {
  const int idx = blockIdx.x * kWG + threadIdx.x;
  if (idx >= up * cmax) return;
  const int p = idx / cmax, i = idx - p * cmax;
  const int k = p + i * up;
  hp[idx] = k < ntaps ? h[k] : 0.0f;
}

__global__ __launch_bounds__(kWG) void resample_tile(const float* __restrict__ x, long long n, long long x_stride,
                                                     const float* __restrict__ hp, int ntaps, int up, int down,
                                                     int cmax, const float* __restrict__ state, int ns,
                                                     float* __restrict__ y, long long y_stride, long long ny) {
  extern __shared__ __attribute__((aligned(16))) float win[];
  const int s = blockIdx.y;
  const long long j0 = (long long)blockIdx.x * kWG;
  const long long jl = j0 + kWG - 1 < ny - 1 ? j0 + kWG - 1 : ny - 1;  // last output of this workgroup
  const long long lo = (j0 * down) / up - (cmax - 1);                  // lowest input index touched
  const long long hi = (jl * down) / up;                               // highest
  const int span = (int)(hi - lo + 1);
  const float* xs = x + (long long)s * x_stride;
  const float* st = state + (long long)s * ns;
  for (int i = threadIdx.x; i < span; i += kWG) {
    const long long g = lo + i;
    win[i] = g >= 0 ? (g < n ? xs[g] : 0.0f) : (g >= -ns ? st[ns + g] : 0.0f);
  }
  __syncthreads();
  const long long j = j0 + threadIdx.x;
  if (j >= ny) return;
  const long long nn = j * down;
  const int p = (int)(nn % up);
  const long long q = nn / up;
  const int cnt = (ntaps - p + up - 1) / up;
  const float* hr = hp + (long long)p * cmax;
  const float* wq = win + (q - lo);
  float acc = 0.0f;
  int i = 0;
  for (; i + 4 <= cnt; i += 4) {
    const float4 hv = *reinterpret_cast<const float4*>(hr + i);
    acc = acc + hv.x * wq[-i];
    acc = acc + hv.y * wq[-i - 1];
    acc = acc + hv.z * wq[-i - 2];
    acc = acc + hv.w * wq[-i - 3];
  }
  for (; i < cnt; ++i) acc = acc + hr[i] * wq[-i];
  y[(long long)s * y_stride + j] = acc;
}

// ------------------------------------------------ phase-major tiled kernel --
// For T == CMAX*up (every phase has exactly CMAX taps: the reference's
// num_taps*up convention, src/project.cpp:210) and up >= 2.
//
// Output j = up*t + phi has phase p = (phi*down) mod up and newest input
// q = t*down + (phi*down) div up: the phase depends on phi only.  A
// "column" is one period t of one stream (up consecutive outputs); a
// workgroup takes 64 columns (one per lane) x NW consecutive phi (one per
// wave).  Within a wave the taps are therefore uniform -- SGPR operands,
// loaded per pass of KP taps like fir_tile -- and each lane slides down its
// own window with 16-B LDS reads.  Each lane's window lives in its own LDS
// segment: inputs [t*down + q(phi0) - (CMAX-1) - sa, t*down + q(phi_last)],
// the union of its NW outputs' windows, 16-B aligned (sa) when down % 4 == 0;
// segment stride SEGPAD floats with SEGPAD/4 odd, so the 16-lane groups of
// ds_read_b128 never share a bank.
constexpr int kPPLanes = 64;

// Taps come from this wave's LDS tap row, pre-shifted by the wave's
// alignment A so that chunk cc's four taps are one aligned float4:
// trow[4*cc + 3 - jj] = tap i = 4*cc + A - jj.  All lanes read the same
// address (a broadcast); the window chunk is this lane's own.
template <int CMAX, int A>
__device__ __forceinline__ float pp_scan(const float* wl, int ctop, const float* trow) {
  constexpr int CHI = (CMAX - 1 + 3 - A) / 4;  // last chunk holding a tap
  constexpr int PD = 4;                        // chunks in flight ahead of the one consumed
  const float* lo = wl + 4 * (ctop - CHI);     // window chunk cc at lo + 4*(CHI - cc)
  float acc = 0.0f;
  float4 q[CHI + 1], t[CHI + 1];               // compile-time indexed: a register ring
#pragma unroll
  for (int cc = 0; cc < PD && cc <= CHI; ++cc) {
    q[cc] = *reinterpret_cast<const float4*>(lo + 4 * (CHI - cc));
    t[cc] = *reinterpret_cast<const float4*>(trow + 4 * cc);
  }
#pragma unroll
  for (int cc = 0; cc <= CHI; ++cc) {
    if (cc + PD <= CHI) {
      q[cc + PD] = *reinterpret_cast<const float4*>(lo + 4 * (CHI - cc - PD));
      t[cc + PD] = *reinterpret_cast<const float4*>(trow + 4 * (cc + PD));
    }
    const float e[4] = {q[cc].x, q[cc].y, q[cc].z, q[cc].w};
    const float hv[4] = {t[cc].w, t[cc].z, t[cc].y, t[cc].x};  // hv[jj] = tap 4*cc + A - jj
#pragma unroll
    for (int jj = 3; jj >= 0; --jj) {
      const int i = 4 * cc + A - jj;
      if (i >= 0 && i < CMAX) acc = acc + hv[jj] * e[jj];
    }
    asm volatile("" : "+v"(acc));
    __builtin_amdgcn_sched_barrier(0);
  }
  return acc;
}

struct PPArgs {
  const float* x;
  long long n, x_stride;
  const float* hp;  // polyphase table, row stride cpad
  int cpad, up, down;
  const float* state;
  int ns;
  float* y;
  long long y_stride, ny;
  int np;          // periods per stream
  long long ncols; // nstreams * np
  int nphg;        // phase groups (ceil(up / NW))
  int segpad;      // LDS floats per lane segment
  int vec;         // 16-B staging (down % 4 == 0 and aligned rows)
  int ablate;      // timing experiments only (SDR_ABLATE): 1 = no staging, 2 = no taps walk
};

constexpr int kPPSeg = 260;  // max LDS floats per column segment (host-checked)

// LDS image of one tile: kPPLanes column segments of a.segpad floats.
// Interior 16-B chunks arrive by LDS-DMA (lane k of a wave-instruction
// lands at segment base + 16*k, one instruction per column); the chunks
// that reach before the block (state) or past its end go through registers
// in pp_edge(), issued after the tile in flight has been computed.
template <int CMAX>
__device__ __forceinline__ void pp_dma(const PPArgs& a, long long cb, float* buf, int wv, int ln, int nw,
                                       long long q0, int sa, int per_col) {
  for (int cl = wv; cl < kPPLanes; cl += nw) {
    const long long col = cb * kPPLanes + cl;
    if (col >= a.ncols) break;
    const long long sidx = col / a.np, t = col - sidx * a.np;
    const long long g = t * a.down + q0 - (CMAX - 1) - sa + 4 * ln;  // multiple of 4
    if (ln < per_col && g >= 0 && g + 4 <= a.n)
      __builtin_amdgcn_global_load_lds(a.x + sidx * a.x_stride + g, buf + cl * a.segpad, 16, 0, 0);
  }
}

template <int CMAX>
__device__ __forceinline__ void pp_edge(const PPArgs& a, long long cb, float* buf, int wv, int ln, int nw,
                                        long long q0, int sa, int per_col) {
  for (int cl = wv; cl < kPPLanes; cl += nw) {
    const long long col = cb * kPPLanes + cl;
    if (col >= a.ncols) break;
    const long long sidx = col / a.np, t = col - sidx * a.np;
    const long long g = t * a.down + q0 - (CMAX - 1) - sa + 4 * ln;
    if (ln < per_col && !(g >= 0 && g + 4 <= a.n)) {
      const float* xs = a.x + sidx * a.x_stride;
      const float* st = a.state + sidx * a.ns;
      float w4[4];
#pragma unroll
      for (int r = 0; r < 4; ++r) {
        const long long gg = g + r;
        w4[r] = gg >= 0 ? (gg < a.n ? xs[gg] : 0.0f) : (gg >= -a.ns ? st[a.ns + gg] : 0.0f);
      }
      *reinterpret_cast<float4*>(buf + cl * a.segpad + 4 * ln) = make_float4(w4[0], w4[1], w4[2], w4[3]);
    }
  }
}

// Persistent: workgroup b keeps one phase group (its waves' phases, hence
// their SGPR tap rows, stay fixed and scalar-cache hot) and walks a run of
// column blocks with two LDS images: the DMA of block i+1 is in flight
// while block i is computed.  The two images are distinct __shared__
// objects, so the compiler's wait for the DMA does not hold the ds_reads of
// the other image.
template <int CMAX>
__global__ __launch_bounds__(1024, 1) void resample_pp(PPArgs a) {
  __shared__ __attribute__((aligned(16))) float imgA[kPPLanes * kPPSeg];
  __shared__ __attribute__((aligned(16))) float imgB[kPPLanes * kPPSeg];
  constexpr int TROW = ((CMAX + 3 + 3) / 4) * 4;  // floats per wave tap row
  __shared__ __attribute__((aligned(16))) float taps[16 * TROW];
  const int nw = blockDim.x >> 6;
  const int wv = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6), ln = threadIdx.x & 63;
  const int grp = blockIdx.x % a.nphg;
  const int slot = blockIdx.x / a.nphg, nslots = gridDim.x / a.nphg;
  const long long ncb = (a.ncols + kPPLanes - 1) / kPPLanes;
  const long long per = (ncb + nslots - 1) / nslots;
  const long long cb0 = (long long)slot * per;
  const long long cb1 = cb0 + per < ncb ? cb0 + per : ncb;
  if (cb0 >= cb1) return;
  const int phi0 = grp * nw;
  const int phi_last = min(phi0 + nw, a.up) - 1;
  const long long q0 = ((long long)phi0 * a.down) / a.up;
  const long long qlast = ((long long)phi_last * a.down) / a.up;
  const int sa = (int)(((q0 - (CMAX - 1)) % 4 + 4) % 4);  // 16-B align the segment start
  const int seglen = (int)(qlast - q0) + CMAX + sa;
  const int per_col = (seglen + 3) >> 2;
  // this wave's phase (idle waves past the last phase still stage and sync)
  const int phi = phi0 + wv;
  const bool wave_on = phi <= phi_last;
  const int p = (int)(((long long)phi * a.down) % a.up);
  const int off = (int)(((long long)phi * a.down) / a.up - q0);
  const int e1 = off + CMAX - 1 + sa;  // segment element of tap i = 0 (newest input)
  const int A = e1 & 3, ctop = e1 >> 2;
  // this wave's tap row, shifted by A (fixed for the workgroup's lifetime)
  float* trow = taps + wv * TROW;
  {
    const float* hrow = a.hp + (long long)(wave_on ? p : 0) * a.cpad;
    for (int u = ln; u < TROW; u += 64) {
      const int i = u + A - 3;
      trow[u] = (i >= 0 && i < CMAX) ? hrow[i] : 0.0f;
    }
  }

  auto compute = [&](long long cb, const float* img) __attribute__((always_inline)) {
    if (!wave_on || SDR_ABL(a.ablate) == 2) return;
    const long long col = cb * kPPLanes + ln;
    const long long sidx = col / a.np, t = col - sidx * a.np;
    const long long j = (long long)a.up * t + phi;
    // opaque per tile: keeps the chunk addresses from being hoisted out of
    // the tile loop into one VGPR each
    int woff = ln * a.segpad + 4 * ctop;
    asm volatile("" : "+v"(woff));
    const float* wl = img + woff;
    float acc;
    switch (A) {  // wave-uniform
      case 0: acc = pp_scan<CMAX, 0>(wl, 0, trow); break;
      case 1: acc = pp_scan<CMAX, 1>(wl, 0, trow); break;
      case 2: acc = pp_scan<CMAX, 2>(wl, 0, trow); break;
      default: acc = pp_scan<CMAX, 3>(wl, 0, trow); break;
    }
    if (col < a.ncols && j < a.ny) a.y[sidx * a.y_stride + j] = acc;
  };
  auto stage = [&](long long cb, float* img, bool edge) __attribute__((always_inline)) {
    if (SDR_ABL(a.ablate) == 1) return;
    if (edge)
      pp_edge<CMAX>(a, cb, img, wv, ln, nw, q0, sa, per_col);
    else
      pp_dma<CMAX>(a, cb, img, wv, ln, nw, q0, sa, per_col);
  };

  stage(cb0, imgA, false);
  stage(cb0, imgA, true);
  __syncthreads();
  for (long long cb = cb0; cb < cb1; cb += 2) {
    const bool nxt = cb + 1 < cb1;
    if (nxt) stage(cb + 1, imgB, false);
    compute(cb, imgA);
    if (nxt) stage(cb + 1, imgB, true);
    __syncthreads();  // image B landed; every wave is done reading A
    if (!nxt) break;
    const bool nxt2 = cb + 2 < cb1;
    if (nxt2) stage(cb + 2, imgA, false);
    compute(cb + 1, imgB);
    if (nxt2) stage(cb + 2, imgA, true);
    __syncthreads();
  }
}

// Fallback when the staged window would not fit LDS (huge down/up ratios):
// the same sum straight from global memory.
__global__ __launch_bounds__(kWG) void resample_direct(const float* __restrict__ x, long long n, long long x_stride,
                                                       const float* __restrict__ hp, int ntaps, int up, int down,
                                                       int cmax, const float* __restrict__ state, int ns,
                                                       float* __restrict__ y, long long y_stride, long long ny) {
  const int s = blockIdx.y;
  const long long j = (long long)blockIdx.x * kWG + threadIdx.x;
  if (j >= ny) return;
  const float* xs = x + (long long)s * x_stride;
  const float* st = state + (long long)s * ns;
  const long long nn = j * down;
  const int p = (int)(nn % up);
  const long long q = nn / up;
  const int cnt = (ntaps - p + up - 1) / up;
  const float* hr = hp + (long long)p * cmax;
  float acc = 0.0f;
  for (int i = 0; i < cnt; ++i) {
    const long long g = q - i;
    const float v = g >= 0 ? xs[g] : st[ns + g];
    acc = acc + hr[i] * v;
  }
  y[(long long)s * y_stride + j] = acc;
}

// state <- last ns inputs (src/filter.cpp:169), after every reader is done.
__global__ __launch_bounds__(kWG) void resample_commit(const float* __restrict__ x, long long n, long long x_stride,
                                                       float* state, int ns) {
  const int s = blockIdx.y;
  const int i = blockIdx.x * kWG + threadIdx.x;
  if (i >= ns) return;
  state[(long long)s * ns + i] = x[(long long)s * x_stride + n - ns + i];
}

// switch SDR_RESAMPLE_PP (the tests run every resampler kernel)
bool pp_enabled() { return sw(kSwResamplePp) != 0; }

}  // namespace

size_t resample_scratch_floats(int up, int ntaps) {
  const int cmax = (ntaps + up - 1) / up;
  const size_t pp = (size_t)up * (size_t)((cmax + 3) / 4 * 4);
  const size_t rs = resample_rs_scratch_floats(up, ntaps);
  return std::max(pp, rs);
}

hipError_t launch_resample(int up, int down, const float* x, long long n, int nstreams, long long x_stride,
                           const float* h, int ntaps, float* state, int ns, float* y, long long y_stride,
                           long long ny, float* scratch_taps, hipStream_t st, const float* lp_tables) {
  {
    // resample_rs.hip's kernels first (lane-phase, then sliding-window), for the shapes they cover
    hipError_t e = hipSuccess;
    bool state_done = false;
    if (launch_resample_rs(up, down, x, n, nstreams, x_stride, h, ntaps, state, ns, y, y_stride, ny, scratch_taps,
                           st, &e, &state_done, lp_tables)) {
      if (e != hipSuccess || ns <= 0 || state_done) return e;
      hipLaunchKernelGGL(resample_commit, dim3((ns + kWG - 1) / kWG, (unsigned)nstreams), dim3(kWG), 0, st, x, n,
                         x_stride, state, ns);
      return hipGetLastError();
    }
  }
  const int cmax = ((ntaps + up - 1) / up + 3) / 4 * 4;  // padded row length (16-B rows)
  const int tab = up * cmax;
  hipLaunchKernelGGL(build_polyphase, dim3((tab + kWG - 1) / kWG), dim3(kWG), 0, st, h, ntaps, up, cmax,
                     scratch_taps);
  hipError_t e = hipGetLastError();
  if (e != hipSuccess) return e;
  const int cnt_max = (ntaps + up - 1) / up;
  // phase-major tiled kernel: every phase has exactly cnt_max taps
  if (up >= 2 && ntaps == cnt_max * up && (cnt_max == 151 || cnt_max == 101) && pp_enabled()) {
    PPArgs a;
    a.x = x;
    a.n = n;
    a.x_stride = x_stride;
    a.hp = scratch_taps;
    a.cpad = cmax;
    a.up = up;
    a.down = down;
    a.state = state;
    a.ns = ns;
    a.y = y;
    a.y_stride = y_stride;
    a.ny = ny;
    a.np = (int)((ny + up - 1) / up);
    a.ncols = (long long)a.np * nstreams;
    const int nw = up < 16 ? up : 16;
    a.nphg = (up + nw - 1) / nw;
    const long long qspan = ((long long)(nw - 1) * down + up - 1) / up + 1;  // >= q(phi_last) - q(phi0)
    int segpad = (int)((qspan + cnt_max + 3 + 3) / 4 * 4);
    if ((segpad / 4) % 2 == 0) segpad += 4;
    a.segpad = segpad;
    a.vec = (down % 4 == 0) && x_stride % 4 == 0 && (reinterpret_cast<uintptr_t>(x) & 15) == 0;
    static const int ablate = SDR_TIMING_ENV("SDR_ABLATE", 0);
    a.ablate = ablate;
    const long long seglen_max = qspan + cnt_max + 3;  // one DMA wave-instruction per column
    if (segpad <= kPPSeg && seglen_max <= 256 && a.vec) {
      const int ncu = device_cu_count();
      const long long ncb = (a.ncols + kPPLanes - 1) / kPPLanes;
      long long slots = ncu / a.nphg;  // ~one workgroup per CU
      if (slots < 1) slots = 1;
      if (slots > ncb) slots = ncb;
      const long long grid = slots * a.nphg;
      if (cnt_max == 151)
        hipLaunchKernelGGL(resample_pp<151>, dim3((unsigned)grid), dim3(64 * nw), 0, st, a);
      else
        hipLaunchKernelGGL(resample_pp<101>, dim3((unsigned)grid), dim3(64 * nw), 0, st, a);
      e = hipGetLastError();
      if (e != hipSuccess) return e;
      if (ns > 0) {
        hipLaunchKernelGGL(resample_commit, dim3((ns + kWG - 1) / kWG, (unsigned)nstreams), dim3(kWG), 0, st, x, n,
                           x_stride, state, ns);
        e = hipGetLastError();
      }
      return e;
    }
  }
  const dim3 grid((unsigned)((ny + kWG - 1) / kWG), (unsigned)nstreams);
  // widest staged window: 256 outputs span (255*down)/up + 1 inputs + taps
  const long long span = (255LL * down) / up + 2 + cmax;
  if (span <= kMaxSpan && cnt_max <= cmax) {
    hipLaunchKernelGGL(resample_tile, grid, dim3(kWG), (size_t)span * sizeof(float), st, x, n, x_stride,
                       scratch_taps, ntaps, up, down, cmax, state, ns, y, y_stride, ny);
  } else {
    hipLaunchKernelGGL(resample_direct, grid, dim3(kWG), 0, st, x, n, x_stride, scratch_taps, ntaps, up, down, cmax,
                       state, ns, y, y_stride, ny);
  }
  e = hipGetLastError();
  if (e != hipSuccess) return e;
  if (ns > 0) {
    hipLaunchKernelGGL(resample_commit, dim3((ns + kWG - 1) / kWG, (unsigned)nstreams), dim3(kWG), 0, st, x, n,
                       x_stride, state, ns);
    e = hipGetLastError();
  }
  return e;
}

}  // namespace sdr
