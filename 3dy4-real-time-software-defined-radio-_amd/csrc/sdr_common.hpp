// sdr_common.hpp -- shared launch descriptors and helpers for the gfx950
// RF front-end kernels.  Internal to libsdrhip.so (the public surface is
// include/sdr_hip.h).
#pragma once

#include <hip/hip_runtime.h>

#include <cstdint>

namespace sdr {

// Every FIR-family kernel runs 256-thread workgroups: four wave64s, one per
// SIMD of a CU.
constexpr int kWG = 256;

enum class Src : int { F32 = 0, U8 = 1 };

// One launch = the next block of `nstreams` independent streams.  Stream s:
//   input   x{0,1} + s*x_stride (f32 planar I/Q), or iq + s*x_stride bytes (u8)
//   state   state{0,1} + s*ns          (the reference's `state` vectors)
//   prev    prev{0,1}[s]               (fmDemodArctan's prev_I / prev_Q)
//   output  y0 + s*y_stride            (FIR-only launches)
//           out + s*out_stride         (demodulated, fused launches)
struct FirLaunch {
  const float* x0;
  const float* x1;
  const uint8_t* iq;
  long long x_stride;
  long long n;  // input samples (IQ pairs for the fused path) per stream
  int nstreams;
  int ntaps;
  int D;
  float* state0;
  float* state1;
  int ns;
  float* prev0;
  float* prev1;
  float* y0;
  float* y1;
  long long y_stride;
  float* out;
  long long out_stride;
  int tiles_per_stream;
  int tiles_per_wg;  // fir_tile: tiles per workgroup (see fir_tile.hip)
  int walk;          // fir_tile: 0 a run per workgroup, 1 XCD slabs; fir_tile_grp: 1 XCD slabs, 0 one slab
  int slab;          // fir_tile_grp: tiles per slab
  int ablate;        // timing builds only (SDR_ABL): 1 = no global loads, 2 = no FIR math, 4 = one tap pass of three
  int fma;           // SDR_ARITH_FMA: fused multiply-add FIR arithmetic where a fast path implements it
  // Side copy, done by each stream's tile-0 workgroup after its reads (the
  // fast tile kernels only): side_n floats side_src + s*side_src_stride ->
  // side_dst + s*side_dst_stride.  The device mono pipeline's delay line
  // (sdr_mono_pcm_u8_dev) rides on it: 0 = none.
  const float* side_src;
  float* side_dst;
  long long side_src_stride, side_dst_stride;
  int side_n;
  // FIR-only launches (fir_tile_grp): outputs quantised to s16 PCM
  // (src/project.cpp:311-314) into pcm + s*pcm_stride instead of y0; null = f32
  int16_t* pcm;
  long long pcm_stride;
};

// Exact reference conversion of one wire byte, src/iofunc.cpp:118:
// float(((unsigned char)u - 128) / 128.0).  (u-128)/128 is a multiple of
// 2^-7 with |value| <= 1, so the float product below is the same number.
__device__ __forceinline__ float u8_to_f32(uint32_t u) { return (float)((int)u - 128) * 0.0078125f; }

// Byte b of a packed word, same value: v_cvt_f32_ubyte<b> then one fma --
// u * 2^-7 - 1 is exact, so the single rounding of the fma changes nothing
// (128 gives +0.0, as the reference's (u-128)/128.0 does).
template <int B>
__device__ __forceinline__ float u8_byte_to_f32(uint32_t w) {
  return __builtin_fmaf((float)((w >> (8 * B)) & 0xffu), 0.0078125f, -1.0f);
}


// Compute units of the calling thread's current device, cached per device
// (the launchers run concurrently from several host threads: the drop-in's
// two threads per block, bench.py's one thread per GPU).
int device_cu_count();
int device_lds_bytes();  // LDS bytes per CU of the current device
int device_grid_y_max();  // grid y limit of the current device (kernels put streams on y)
// Integer environment variable, `dflt` when unset.  Read at context creation
// (SDR_STEREO_FORK) and, once, by the switch table below -- never per launch.
int env_int(const char* name, int dflt);

// Kernel-selection switches: which of several bit-identical kernels a
// launcher runs (A/B and the parity tests, which run every kernel).  One
// process-wide table of atomics, initialised once from the environment
// variable of the same name (first use), then changed only through
// sdr_set_switch() (include/sdr_hip.h).  Launchers read it with one relaxed
// atomic load: no environment scan in the launch path, and no getenv racing a
// setenv in a multithreaded caller.
enum Switch : int {
  kSwFirSc = 0,       // SDR_FIR_SC: f32 fused front end on fir_tile_sc (1) or fir_tile (0)
  kSwFirScU8,         // SDR_FIR_SC_U8: u8 front end on fir_tile_sc (1) or persistent fir_tile_grp (0)
  kSwResampleLp,      // SDR_RESAMPLE_LP: lane-phase resample_lp for the shapes it covers
  kSwResampleLoader,  // SDR_RESAMPLE_LOADER: resample_lp with its loader wave
  kSwResampleRs,      // SDR_RESAMPLE_RS: sliding-window resample_rs
  kSwResamplePp,      // SDR_RESAMPLE_PP: phase-major resample_pp
  kSwLongVtap,        // SDR_LONG_VTAP: fir_long with LDS-staged (1) or SGPR (0) taps
  kSwF16Mfma,         // SDR_F16_MFMA: fp16 arm on the MFMA Toeplitz GEMM (1) or v_dot2 (0)
  kSwF16Head,         // SDR_F16_HEAD: fir_long_mfma's first workgroup loads its state in the first batch
  kSwF16W8,           // SDR_F16_W8: fir_long_mfma as 8 waves of one tile (1) or 4 of two (0)
  kSwPllFast,         // SDR_PLL_FAST: certified short-chain PLL step (1) or library routines (0)
  kSwPllGuard,        // SDR_PLL_GUARD: the PLL's chunk input checks as a parallel pre-pass
  kSwLongCommit,      // SDR_LONG_COMMIT: fir_long's first workgroup commits the state (1) or long_commit (0)
  kSwCount
};
int sw(Switch s);

// Timing experiments (ablations that return WRONG outputs, shape overrides)
// exist only in a timing build (make TIMING=1 -> -DSDR_TIMING_BUILD, never
// the shipped library): in the product build the ablation field is the
// constant 0 and the variables are not even named.
#ifdef SDR_TIMING_BUILD
#define SDR_TIMING_ENV(name, dflt) (::sdr::env_int((name), (dflt)))
#define SDR_ABL(v) (v)
#else
#define SDR_TIMING_ENV(name, dflt) (dflt)
#define SDR_ABL(v) 0
#endif

// Host-side launchers, one per kernel family (defined next to the kernels).
// allow_fast = false forces the generic kernel (misaligned buffers).
hipError_t launch_fir(const FirLaunch& a, const float* h, bool demod, int nch, Src src, hipStream_t st,
                      float* scratch_y0, float* scratch_y1, bool allow_fast);
hipError_t launch_demod(const float* I, const float* Q, long long n, int nstreams, long long stride,
                        float* prev_i, float* prev_q, float* out, long long out_stride, hipStream_t st);
// lp_tables: resample_lp's tables prebuilt by resample_lp_tables (a plan),
// or nullptr to build them into scratch_taps for this call
hipError_t launch_resample(int up, int down, const float* x, long long n, int nstreams, long long x_stride,
                           const float* h, int ntaps, float* state, int ns, float* y, long long y_stride,
                           long long ny, float* scratch_taps, hipStream_t st, const float* lp_tables = nullptr);
hipError_t launch_delay(const float* in, long long n, int nstreams, long long in_stride, float* state, int ns,
                        float* out, long long out_stride, hipStream_t st);
hipError_t launch_pcm(const float* x, long long n, int nstreams, long long x_stride, int16_t* pcm,
                      long long pcm_stride, hipStream_t st);
// Stereo back end (stereo.hip): fmPLL one lane per stream, optionally fused
// with the x2 mixer; L/R + interleave + s16 output stage.  guard: scratch of
// pll_guard_bytes(n, nstreams) for the certified step's per-chunk input
// checks (computed in parallel before the recurrence), or nullptr to check
// inside the recurrence.
size_t pll_guard_bytes(long long n, int nstreams);
hipError_t launch_pll(const float* in, long long n, int nstreams, long long in_stride, float freq, float Fs,
                      float nco_scale, float phase_adjust, float norm_bw, float* pll, const float* mix,
                      long long mix_stride, float* out, long long out_stride, float* args, long long args_stride,
                      hipStream_t st, uint8_t* guard);
// the two halves of launch_pll: the per-stream recurrence (records each
// sample's oscillator argument in args) and the parallel NCO (+ mixer)
// guard_ready: launch_pll_guard already wrote this block's guard (stream-ordered
// before this launch; the two-stage stereo front stage does, off the recurrence's
// critical path), else the pre-pass runs here first
hipError_t launch_pll_recurrence(const float* in, long long n, int nstreams, long long in_stride, float freq,
                                 float Fs, float nco_scale, float phase_adjust, float norm_bw, float* pll, float* args,
                                 long long args_stride, hipStream_t st, uint8_t* guard, bool guard_ready = false);
// the recurrence's input guard pre-pass alone; *ready = whether it ran (the
// recurrence then takes the guard as given)
hipError_t launch_pll_guard(const float* in, long long n, int nstreams, long long in_stride, uint8_t* guard,
                            hipStream_t st, bool* ready);
hipError_t launch_nco(const float* args, long long args_stride, long long n, int nstreams, float nco_scale,
                      float phase_adjust, const float* mix, long long mix_stride, float* out, long long out_stride,
                      hipStream_t st);
hipError_t launch_stereo_pcm(const float* a, const float* b, long long n, int nstreams, long long stride,
                             int16_t* pcm, long long pcm_stride, hipStream_t st);
hipError_t launch_synth_fm_u8(uint8_t* iq, long long npairs, int nstreams, long long iq_stride,
                              unsigned long long seed, hipStream_t st);
hipError_t launch_u8_to_planar(const uint8_t* iq, long long npairs, int nstreams, long long iq_stride, float* I,
                               float* Q, long long x_stride, hipStream_t st);

// src/project.cpp:311-314: NaN -> 0, else static_cast<short>(x * 16384) as
// the reference's x86-64 build emits it (cvttss2si to int32, keep the low 16
// bits; values outside int32 give INT_MIN -> 0).
__device__ __forceinline__ int16_t pcm_quantise(float u) {
  if (__builtin_isnan(u)) return 0;
  const float v = u * 16384.0f;
  const int w = (v < 2147483648.0f && v >= -2147483648.0f) ? (int)v : (int)0x80000000u;
  return (int16_t)(uint16_t)((unsigned)w & 0xffffu);
}

// Long FIRs without decimation (fir_long.hip): T a multiple of 32.
bool fir_long_ok(int D, int ntaps, int ns, long long n);
hipError_t launch_fir_long(const FirLaunch& a, const float* h, hipStream_t st);
// fp16-storage arm (not bit-exact; tolerance-tested): x/state are fp16
// [nstreams][x_stride] / [nstreams][ns], y fp32; scratch_pairs holds
// fir_long_h_pairs(ntaps) packed tap pairs.
size_t fir_long_h_pairs(int ntaps);
// whether sdr_fir_block_f16_dev runs the MFMA kernel for ntaps (else v_dot2)
bool fir_f16_uses_mfma(int ntaps);
// plan: the MFMA kernel's tap copies prebuilt by build_fir_f16_plan (a tap
// plan, fir_f16_plan_halves(ntaps) halves), or nullptr to build them per launch
hipError_t launch_fir_long_h(const void* x, long long n, int nstreams, long long x_stride, const float* h, int ntaps,
                             void* state, int ns, float* y, long long y_stride, uint32_t* scratch_pairs,
                             hipStream_t st, const void* plan = nullptr);
// halves of the fp16 MFMA kernel's tap plan for ntaps (0: the shape takes no plan)
size_t fir_f16_plan_halves(int ntaps);
hipError_t build_fir_f16_plan(const float* h, int ntaps, void* plan, hipStream_t st);
hipError_t launch_f32_to_f16(const float* x, long long count, void* y, hipStream_t st);

// Whether the tiled fast path handles (D, ntaps, ns) for this source; false
// means launch_fir takes the generic path (still exact, slower).
bool fir_has_fast_path(int D, int ntaps, int ns, int nch, bool demod, Src src);

// Bytes of scratch the resampler needs for its polyphase tap table.
size_t resample_scratch_floats(int up, int ntaps);
// Sliding-window resampler (resample_rs.hip): false = shape not covered.
size_t resample_rs_scratch_floats(int up, int ntaps);
bool launch_resample_rs(int up, int down, const float* x, long long n, int nstreams, long long x_stride,
                        const float* h, int ntaps, float* state, int ns, float* y, long long y_stride, long long ny,
                        float* scratch, hipStream_t st, hipError_t* err, bool* state_done,
                        const float* lp_tables = nullptr);
// Build resample_lp's tables (shifted tap rows + lane table, resample_rs_scratch_floats
// floats) once for a plan; false (nothing launched) when the shape is not one
// resample_lp covers.
bool resample_lp_tables(int up, int down, const float* h, int ntaps, int ns, float* tables, hipStream_t st,
                        hipError_t* err);

// libm_check.hip: the device transcendental routines in bulk (parity tests)
hipError_t launch_libm_sincos_hash(int mode, unsigned chunk_lo, unsigned nchunks, unsigned long long* hash,
                                   hipStream_t st);
hipError_t launch_libm_sincos_diff(unsigned chunk_lo, unsigned nchunks, unsigned long long* count, unsigned* args,
                                   long long cap, hipStream_t st);
hipError_t launch_libm_eval(int fn, const float* a, const float* b, long long n, float* out, hipStream_t st);
hipError_t launch_libm_atan2_screen(unsigned long long seed, unsigned long long first, unsigned long long count,
                                    unsigned* cand, long long cand_cap, unsigned* out, long long out_cap,
                                    unsigned long long* counters, hipStream_t st);

}  // namespace sdr
