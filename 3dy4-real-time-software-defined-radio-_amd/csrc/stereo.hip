// stereo.hip -- the device-resident stereo back end around the front end
// (stereo half): the pilot PLL
// (src/filter.cpp:174-228) fused with the stereo mixer (pointwiseMultiply,
// :253-266), and the output stage that forms L = mono + stereo,
// R = mono - stereo (:267-288), interleaves them (:289-301) and quantises to
// s16 (src/project.cpp:307-314).  The band-pass filters and both resamplers
// are the FIR / resampler kernels of fir_tile.hip / resample*.hip.
//
// fmPLL is a sequential recurrence (each sample's phase detector reads the
// previous sample's feedback oscillator), so it runs one lane per stream:
// streams are the parallel axis, samples are a loop; the NCO output, which
// does not feed back, is evaluated afterwards in parallel over samples.
// Arithmetic follows the reference's promotions exactly: the loop filter in
// fp32, atan2 / cos / sin of the fp32
// arguments as glibc's double routines give them (the reference calls the
// double C functions), every result rounded back to float where the reference
// stores a float: libm_exact.hpp, proved over every fp32 argument of sin / cos
// against glibc (tests/test_libm_exact.py).
#include <type_traits>

#include "sdr_common.hpp"
#include "libm_exact.hpp"
#include "pll_fast.hpp"

#pragma clang fp contract(off)

namespace sdr {
namespace {

constexpr double kPiD = 3.14159265358979323846;  // include/dy4.h:14

constexpr int kPllChunk = 8;
struct PllState {
  float fbI, fbQ, integrator, phaseEst, trigOffset, arg;
};
struct PllChunk {
  float v[kPllChunk];
};
// One step of the recurrence (src/filter.cpp:188-219) with libm_exact.hpp's
// routines: glibc's floats for every argument.
__device__ __forceinline__ void pll_exact_step(PllState& p, float v, float Kp, float Ki, double step) {
  const float eI = (v == 0.0f ? 1.0f : v) * p.fbI;
  const float eQ = v * (-1.0f * p.fbQ);
  const float eD = libmx::atan2_f(eQ, eI);
  p.integrator = p.integrator + Ki * eD;
  p.phaseEst = p.phaseEst + (Kp * eD + p.integrator);
  p.trigOffset = p.trigOffset + 1.0f;
  p.arg = (float)(step * (double)p.trigOffset + (double)p.phaseEst);
  const libmx::SinCos sc = libmx::sincos_f(p.arg);  // glibc's sincos (the reference's -O3 build fuses cos + sin)
  p.fbI = sc.c;
  p.fbQ = sc.s;
}
// An uncertified chunk's exact re-run (steps k0 .. k0+m-1, arguments to
// ar[k0+1 ..]), out of line: it is rare, and inlined it shares the hot loop's
// register allocation (pll_kernel 1,055 vs 946 us per stereo0 block,
// profiles/r06d/, r06e/).
__device__ __attribute__((noinline)) PllState pll_exact_chunk(PllState p, PllChunk c, int m, float Kp, float Ki,
                                                              double step, float* ar, long long k0, long long n) {
#pragma unroll
  for (int j = 0; j < kPllChunk; ++j) {
    if (j < m) {
      pll_exact_step(p, c.v[j], Kp, Ki, step);
      if (k0 + j + 1 < n) ar[k0 + j + 1] = p.arg;
    }
  }
  return p;
}


// pll[6] per stream: feedbackI, feedbackQ, integrator, phaseEst, trigOffset, nco_state
// (src/project.cpp:48-55).  Only the recurrence runs here: the phase detector
// (atan2) and the feedback oscillator (sin/cos) of every sample depend on the
// previous sample.  The NCO output cos(trigArg*ncoScale + phaseAdjust) does
// not feed back, so this kernel only records trigArg (args[k+1] for sample k,
// args[0] = the incoming nco_state) and nco_kernel evaluates all of them in
// parallel.  The last sample's NCO becomes the new nco_state here.
//
// FAST: each step first runs the short-chain atan2 / sincos of pll_fast.hpp,
// which certify that their float results are the reference's; a chunk of 8
// steps in which any lane of the wave could not certify a result is run again
// from its saved state with libm_exact.hpp's routines (a wave-uniform branch,
// off the recurrence's chain), which give glibc's floats.  The stored
// arguments of the first pass are rewritten by the second, so every output is
// the exact path's or a certified equal.
//
// GUARD: where a chunk's input check (pllfast::input_ok on its 8 samples)
// comes from -- 0: evaluated in the kernel, 1: guard[s * nchunk + c], written
// by pll_guard_kernel over every stream and chunk in parallel beforehand.  The
// check is off the recurrence's dependency chain, but the one wave per SIMD
// issues every instruction itself: in the kernel it cost 7.6 % of stereo0
// (profiles/r03_ab/pll_guard.txt).
template <int FAST, int GUARD>
__global__ __launch_bounds__(64) void pll_kernel(const float* __restrict__ in, long long n, int nstreams,
                                                 long long in_stride, float freq, float Fs, float nco_scale,
                                                 float phase_adjust, float norm_bw, float* __restrict__ pll,
                                                 float* __restrict__ args, long long args_stride,
                                                 const uint8_t* __restrict__ guard, long long nchunk) {
  const int s = blockIdx.x * 64 + threadIdx.x;
  if (s >= nstreams) return;
  const float* x = in + (long long)s * in_stride;
  float* ar = args + (long long)s * args_stride;
  float* st = pll + 6LL * s;
  float fbI = st[0], fbQ = st[1], integrator = st[2], phaseEst = st[3], trigOffset = st[4];
  ar[0] = st[5];  // ncoOut[0] = nco_state (src/filter.cpp:186)
  // src/filter.cpp:175-179: float Cp = 2.666, Ci = 3.555; Kp, Ki in float
  const float Kp = norm_bw * 2.666f;
  const float Ki = norm_bw * norm_bw * 3.555f;
  const double step = 2.0 * kPiD * (double)(freq / Fs);  // 2*PI*(freq/Fs), double (PI is a double literal)
  float arg = 0.0f;
  // m exact steps of the recurrence from the current state (out of line)
  auto exact_steps = [&](const float* buf, int m, long long k0) __attribute__((always_inline)) {
    PllChunk c;
#pragma unroll
    for (int j = 0; j < kPllChunk; ++j) c.v[j] = j < m ? buf[j] : 0.0f;
    const PllState p = pll_exact_chunk(PllState{fbI, fbQ, integrator, phaseEst, trigOffset, arg}, c, m, Kp, Ki, step,
                                       ar, k0, n);
    fbI = p.fbI;
    fbQ = p.fbQ;
    integrator = p.integrator;
    phaseEst = p.phaseEst;
    trigOffset = p.trigOffset;
    arg = p.arg;
  };
  // the same step through pll_fast.hpp; score / score_sc keep the chunk's
  // certificates (atan2 / sine and cosine: separate windows, pll_fast.hpp)
  struct DevOps {
    static __device__ double fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
    static __device__ double rcp(double u) { return __builtin_amdgcn_rcp(u); }
  };
  unsigned score = 0u, score_sc = 0u;
  // the oscillator the previous step left: every step but the kernel's first
  // rotates back from it (pllfast::atan2_rot) instead of evaluating atan2
  pllfast::Osc osc{0.0, 0.0, 1.0, 0};
  auto fast_step = [&](float v, auto rot) __attribute__((always_inline)) {
    const float eI = (v == 0.0f ? 1.0f : v) * fbI;
    const float eQ = v * (-1.0f * fbQ);
    float eD;
    if constexpr (decltype(rot)::value)
      eD = pllfast::atan2_rot<DevOps>(eQ, eI, v, osc, score);
    else
      eD = pllfast::atan2_fast<DevOps>(eQ, eI, score);
    integrator = integrator + Ki * eD;
    phaseEst = phaseEst + (Kp * eD + integrator);
    trigOffset = trigOffset + 1.0f;
    arg = (float)(step * (double)trigOffset + (double)phaseEst);
    pllfast::sincos_fast<DevOps>(arg, fbQ, fbI, score_sc, osc);
  };
  using rot_t = std::true_type;
  using poly_t = std::false_type;
  const bool gains_ok = __builtin_fabsf(Kp) <= 1.0f && __builtin_fabsf(Ki) <= 1.0f;  // chunk_ok's premise
  const float stepf = pllfast::step_bound(step);
  // chunk_ok of the state a chunk starts from (the previous chunk's closing check)
  bool start_ok = gains_ok && pllfast::chunk_ok(fbI, fbQ, integrator, phaseEst, trigOffset, stepf);
  // The chain is latency-bound (one lane per stream).  Inputs are loaded one
  // chunk ahead into registers, so no step waits on memory: a per-sample
  // load put a full load latency -- and the previous step's store, which
  // shares the vmcnt counter -- into every step.
  constexpr int CH = kPllChunk;
  const long long nc = n / CH * CH;
  float xa[CH], xb[CH];
  int ga = 1, gb = 1;  // GUARD 1: the chunks' input checks
  const uint8_t* gs = GUARD ? guard + (long long)s * nchunk : nullptr;
  auto load = [&](float (&buf)[CH], int& g, long long k) __attribute__((always_inline)) {
#pragma unroll
    for (int j = 0; j < CH; ++j) buf[j] = x[k + j];
    if constexpr (GUARD) g = gs[k / CH];
    // keep the loads here: left to the scheduler they sink to their use
    __builtin_amdgcn_sched_barrier(0);
  };
  // first: the kernel's first chunk, whose step 1 has no oscillator to rotate
  // from (the carried state holds only its floats) and runs the polynomial
  auto run = [&](const float (&buf)[CH], int g, long long k0, auto first) __attribute__((always_inline)) {
    if constexpr (FAST) {
      const float s0 = fbI, s1 = fbQ, s2 = integrator, s3 = phaseEst, s4 = trigOffset;
      // the chunk's inputs (already in registers, off the recurrence's chain)
      int in_ok = g;
      if constexpr (!GUARD) {
#pragma unroll
        for (int j = 0; j < CH; ++j) in_ok &= (int)pllfast::input_ok(buf[j]);
      }
      score = score_sc = (start_ok && in_ok) ? ~0u : 0u;
      // unconditional: args rows hold n + 1 floats (launch_pll_recurrence), so
      // ar[n] is the row's spare slot -- no per-step bounds compare and branch
      if constexpr (decltype(first)::value)
        fast_step(buf[0], poly_t{});
      else
        fast_step(buf[0], rot_t{});
      ar[k0 + 1] = arg;
#pragma unroll
      for (int j = 1; j < CH; ++j) {
        fast_step(buf[j], rot_t{});
        ar[k0 + j + 1] = arg;
      }
      start_ok = pllfast::chunk_end_ok(integrator, phaseEst, trigOffset, stepf);
      // 2: timing experiment only (no re-run)
      if (FAST == 2 || !__any(score < pllfast::kCertified || score_sc < pllfast::kCertifiedSc || !start_ok)) return;
      fbI = s0;
      fbQ = s1;
      integrator = s2;
      phaseEst = s3;
      trigOffset = s4;
    }
    exact_steps(buf, CH, k0);
    if constexpr (FAST) {
      start_ok = gains_ok && pllfast::chunk_ok(fbI, fbQ, integrator, phaseEst, trigOffset, stepf);
      // the next chunk's first step rotates from the oscillator of this
      // chunk's last argument (the library's floats are within an ulp of it)
      float tq, ti;
      unsigned unused = 0u;
      pllfast::sincos_fast<DevOps>(arg, tq, ti, unused, osc);
    }
  };
  // ping-pong register chunks (no copies, so no wait at the chunk boundary
  // beyond the chunk being consumed); a chunk past nc re-loads an in-bounds one
  if (nc > 0) {
    load(xa, ga, 0);
    load(xb, gb, CH < nc ? CH : 0);
    run(xa, ga, 0, std::true_type{});
  }
  for (long long k0 = CH; k0 < nc; k0 += 2 * CH) {
    load(xa, ga, k0 + CH < nc ? k0 + CH : k0);
    run(xb, gb, k0, std::false_type{});
    if (k0 + CH < nc) {
      load(xb, gb, k0 + 2 * CH < nc ? k0 + 2 * CH : k0);
      run(xa, ga, k0 + CH, std::false_type{});
    }
  }
  if (nc < n) {  // ragged tail
    float tail[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) tail[j] = nc + j < n ? x[nc + j] : 0.0f;
    exact_steps(tail, (int)(n - nc), nc);
  }
  st[0] = fbI;
  st[1] = fbQ;
  st[2] = integrator;
  st[3] = phaseEst;
  st[4] = trigOffset;
  st[5] = libmx::cos_f(arg * nco_scale + phase_adjust);  // nco_state (:221-222)
}

// guard[s * nchunk + c] = 1 when every sample of the PLL's chunk c of stream
// s passes pllfast::input_ok (0 or 2^-60 <= |v| <= FLT_MAX): the chunk guard
// of the certified step, for all streams and chunks at once.  It sits on the
// stereo back stage's critical path, right before the recurrence, so it reads
// like a streaming kernel: one 16-B load per lane (a chunk is lanes 2c and
// 2c + 1, combined by a lane swap), the rows 16-B aligned
// (pll_guard_vec_ok); pll_guard_kernel below takes any other row layout.
static_assert(kPllChunk == 8, "a chunk is two float4 lanes");
__global__ __launch_bounds__(kWG) void pll_guard_vec_kernel(const float* __restrict__ in, long long in_stride,
                                                            uint8_t* __restrict__ guard, long long nchunk) {
  const int s = blockIdx.y;
  const long long q = (long long)blockIdx.x * kWG + threadIdx.x;  // the stream's q-th float4
  int ok = 1;
  if (q < 2 * nchunk) {
    const float4 v = *reinterpret_cast<const float4*>(in + (long long)s * in_stride + 4 * q);
    ok = (int)pllfast::input_ok(v.x) & (int)pllfast::input_ok(v.y) & (int)pllfast::input_ok(v.z) &
         (int)pllfast::input_ok(v.w);
  }
  ok &= __shfl_xor(ok, 1, 64);
  if (q < 2 * nchunk && (q & 1) == 0) guard[(long long)s * nchunk + (q >> 1)] = (uint8_t)ok;
}
bool pll_guard_vec_ok(const float* in, long long in_stride) {
  return (reinterpret_cast<uintptr_t>(in) & 15) == 0 && (in_stride & 3) == 0;
}
__global__ __launch_bounds__(kWG) void pll_guard_kernel(const float* __restrict__ in, int nstreams, long long in_stride,
                                                        uint8_t* __restrict__ guard, long long nchunk) {
  const int s = blockIdx.y;
  const long long c = (long long)blockIdx.x * kWG + threadIdx.x;
  if (c >= nchunk) return;
  const float* x = in + (long long)s * in_stride + c * kPllChunk;
  int ok = 1;
#pragma unroll
  for (int j = 0; j < kPllChunk; ++j) ok &= (int)pllfast::input_ok(x[j]);
  guard[(long long)s * nchunk + c] = (uint8_t)ok;
}

// ncoOut[k] from the recorded arguments (k = 0: the old nco_state), optionally
// mixed: out = ncoOut * mix * 2 (pointwiseMultiply's gain, src/filter.cpp:264).
__global__ __launch_bounds__(kWG) void nco_kernel(const float* __restrict__ args, long long args_stride, long long n,
                                                  float nco_scale, float phase_adjust, const float* __restrict__ mix,
                                                  long long mix_stride, float* __restrict__ out,
                                                  long long out_stride) {
  const int s = blockIdx.y;
  const long long k = (long long)blockIdx.x * kWG + threadIdx.x;
  if (k >= n) return;
  const float a = args[(long long)s * args_stride + k];
  const float nco = k == 0 ? a : libmx::cos_f(a * nco_scale + phase_adjust);
  out[(long long)s * out_stride + k] = mix ? nco * mix[(long long)s * mix_stride + k] * 2.0f : nco;
}

// L/R + interleave + s16: pcm[2i] = q(a[i] + b[i]), pcm[2i+1] = q(a[i] - b[i])
__global__ __launch_bounds__(kWG) void stereo_pcm_kernel(const float* __restrict__ a, const float* __restrict__ b,
                                                         long long n, long long stride, int16_t* __restrict__ pcm,
                                                         long long pcm_stride) {
  const int s = blockIdx.y;
  const long long i = (long long)blockIdx.x * kWG + threadIdx.x;
  if (i >= n) return;
  const float u = a[(long long)s * stride + i], v = b[(long long)s * stride + i];
  const float l = u + v, r = u - v;
  int16_t* p = pcm + (long long)s * pcm_stride + 2 * i;
  p[0] = pcm_quantise(l);
  p[1] = pcm_quantise(r);
}

}  // namespace

// args: [nstreams][args_stride] with args_stride >= n + 1 (args[s][n] is
// written, a spare slot: the kernel stores every step's argument unguarded)
size_t pll_guard_bytes(long long n, int nstreams) {
  const long long nchunk = n / kPllChunk;
  return (size_t)(nchunk > 0 ? nchunk : 1) * (size_t)(nstreams > 0 ? nstreams : 1);
}

// The guard pre-pass runs when the certified step does and the streams fit
// the grid's y dimension (past the device's grid-y limit the recurrence
// evaluates the guard itself -- same bits); SDR_PLL_FAST=0 runs
// libm_exact.hpp's routines on every step (A/B, tests), SDR_PLL_GUARD=0
// evaluates the input check inside the recurrence (A/B).
static bool pll_guard_pre(long long n, int nstreams) {
  return n / kPllChunk > 0 && sw(kSwPllFast) != 0 && sw(kSwPllGuard) != 0 && nstreams <= device_grid_y_max();
}

hipError_t launch_pll_guard(const float* in, long long n, int nstreams, long long in_stride, uint8_t* guard,
                            hipStream_t st, bool* ready) {
  *ready = false;
  if (!guard || !pll_guard_pre(n, nstreams)) return hipSuccess;
  const long long nchunk = n / kPllChunk;
  if (pll_guard_vec_ok(in, in_stride))
    hipLaunchKernelGGL(pll_guard_vec_kernel, dim3((unsigned)((2 * nchunk + kWG - 1) / kWG), (unsigned)nstreams),
                       dim3(kWG), 0, st, in, in_stride, guard, nchunk);
  else
    hipLaunchKernelGGL(pll_guard_kernel, dim3((unsigned)((nchunk + kWG - 1) / kWG), (unsigned)nstreams), dim3(kWG), 0,
                       st, in, nstreams, in_stride, guard, nchunk);
  const hipError_t e = hipGetLastError();
  *ready = e == hipSuccess;
  return e;
}

hipError_t launch_pll_recurrence(const float* in, long long n, int nstreams, long long in_stride, float freq,
                                 float Fs, float nco_scale, float phase_adjust, float norm_bw, float* pll, float* args,
                                 long long args_stride, hipStream_t st, uint8_t* guard, bool guard_ready) {
  if (args_stride < n + 1) return hipErrorInvalidValue;
  const dim3 grid((unsigned)((nstreams + 63) / 64)), block(64);
  const long long nchunk = n / kPllChunk;
  const int fast = sw(kSwPllFast);  // (mode 2, no re-run path, exists in timing builds only)
  bool pre = guard_ready;
  if (!pre) {
    const hipError_t e = launch_pll_guard(in, n, nstreams, in_stride, guard, st, &pre);
    if (e != hipSuccess) return e;
  }
#ifdef SDR_TIMING_BUILD
  if (fast == 2)
    hipLaunchKernelGGL((pll_kernel<2, 0>), grid, block, 0, st, in, n, nstreams, in_stride, freq, Fs, nco_scale,
                       phase_adjust, norm_bw, pll, args, args_stride, nullptr, 0LL);
  else
#endif
  if (fast && pre)
    hipLaunchKernelGGL((pll_kernel<1, 1>), grid, block, 0, st, in, n, nstreams, in_stride, freq, Fs, nco_scale,
                       phase_adjust, norm_bw, pll, args, args_stride, guard, nchunk);
  else if (fast)
    hipLaunchKernelGGL((pll_kernel<1, 0>), grid, block, 0, st, in, n, nstreams, in_stride, freq, Fs, nco_scale,
                       phase_adjust, norm_bw, pll, args, args_stride, nullptr, 0LL);
  else
    hipLaunchKernelGGL((pll_kernel<0, 0>), grid, block, 0, st, in, n, nstreams, in_stride, freq, Fs, nco_scale,
                       phase_adjust, norm_bw, pll, args, args_stride, nullptr, 0LL);
  return hipGetLastError();
}

hipError_t launch_nco(const float* args, long long args_stride, long long n, int nstreams, float nco_scale,
                      float phase_adjust, const float* mix, long long mix_stride, float* out, long long out_stride,
                      hipStream_t st) {
  hipLaunchKernelGGL(nco_kernel, dim3((unsigned)((n + kWG - 1) / kWG), (unsigned)nstreams), dim3(kWG), 0, st, args,
                     args_stride, n, nco_scale, phase_adjust, mix, mix_stride, out, out_stride);
  return hipGetLastError();
}

hipError_t launch_pll(const float* in, long long n, int nstreams, long long in_stride, float freq, float Fs,
                      float nco_scale, float phase_adjust, float norm_bw, float* pll, const float* mix,
                      long long mix_stride, float* out, long long out_stride, float* args, long long args_stride,
                      hipStream_t st, uint8_t* guard) {
  hipError_t e = launch_pll_recurrence(in, n, nstreams, in_stride, freq, Fs, nco_scale, phase_adjust, norm_bw, pll,
                                       args, args_stride, st, guard);
  if (e != hipSuccess) return e;
  return launch_nco(args, args_stride, n, nstreams, nco_scale, phase_adjust, mix, mix_stride, out, out_stride, st);
}

hipError_t launch_stereo_pcm(const float* a, const float* b, long long n, int nstreams, long long stride,
                             int16_t* pcm, long long pcm_stride, hipStream_t st) {
  hipLaunchKernelGGL(stereo_pcm_kernel, dim3((unsigned)((n + kWG - 1) / kWG), (unsigned)nstreams), dim3(kWG), 0, st,
                     a, b, n, stride, pcm, pcm_stride);
  return hipGetLastError();
}

}  // namespace sdr
