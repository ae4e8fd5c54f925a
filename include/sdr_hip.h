/*
 * sdr_hip.h -- C ABI of the MI355X (gfx950) RF front-end library (libsdrhip.so).
 *
 * This is the drop-in boundary for the hot path of the reference's DSP block
 * library, src/filter.cpp, whose C++ interface is include/filter.h:17-34
 * (ghotrs4/3DY4-Real-Time-Software-defined-Radio-).  Plain pointers and sizes
 * only: no torch, no HIP types in any signature (streams travel as void*).
 *
 * Two families of entry points:
 *
 *  1. Host-pointer, synchronous calls (``sdr_*_f32``): one block of one
 *     stream, exactly the contract of the filter.h function each one
 *     replaces -- outputs valid on return, in/out state arrays updated in
 *     place.  The drop-in filter implementation (host/filter_hip.cpp) is
 *     built on these.  They copy over PCIe; they exist for compatibility and
 *     parity, not for throughput.
 *
 *  2. Device-resident, batched, stream-ordered calls (``*_dev``): nstreams
 *     independent streams in one launch, every pointer is device memory, the
 *     call only enqueues work on the context's HIP stream.  Stream s reads
 *     its n input samples at  x + s*x_stride  and owns row s of each state
 *     array ([nstreams][ns], row stride ns) and element s of each prev array.
 *     One call == the next block of every stream: state carries exactly as
 *     the reference carries it between calls.  These are what bench.py times.
 *
 * Arithmetic contract: every kernel reproduces the reference's fp32 operation
 * order (taps summed k = 0..T-1 from 0.0f with separately rounded multiply
 * and add, discriminator envelope summed in double) so results are
 * bit-identical to the compiled reference; see DESIGN.md "Parity".
 *
 * Errors: every call returns SDR_OK (0) or a negative code.  SDR_EINVAL marks
 * an argument combination for which the reference itself would read or write
 * out of bounds (e.g. n % D != 0 in downsampleBlockConvolveFIR,
 * src/filter.cpp:127-132); sdr_ctx_last_error() says which.
 *
 * Threading: a context (one device + one HIP stream + scratch buffers) must
 * not be used by two threads at once; use one context per thread (the drop-in
 * keeps a thread_local one, matching src/project.cpp:299-302's two threads).
 */
#ifndef SDR_HIP_H
#define SDR_HIP_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDR_OK 0
#define SDR_EINVAL (-1) /* precondition the reference leaves as UB / bad argument */
#define SDR_EHIP (-2)   /* HIP runtime / launch failure */
#define SDR_ENOMEM (-3) /* device allocation failed */
#define SDR_ENODEV (-4) /* no such device */

typedef struct sdr_ctx sdr_ctx;

/* ABI version of this header; sdr_abi_version() returns the library's.  A
 * caller built against version V should refuse a library whose version
 * differs (entry points are added and, rarely, removed between versions --
 * INTEGRATION.md §2 keeps the history).
 *   1  rounds 1-4
 *   2  round 5: the three-stage stereo split (sdr_stereo_pll_dev /
 *      sdr_stereo_post_dev) removed; switch table (sdr_set_switch)
 *   3  round 6: sdr_libm_* verification entry points, the two-stage mono
 *      path (sdr_mono_work_*, sdr_mono_front_u8_dev, sdr_mono_back_dev), the
 *      stereo back stage's halves (sdr_stereo_pll_dev, sdr_stereo_post_dev) */
#define SDR_ABI_VERSION 3
int sdr_abi_version(void);

/* ------------------------------------------------------------ context -- */
const char *sdr_version(void);
const char *sdr_strerror(int code);
int sdr_device_count(int *count);
int sdr_ctx_create(int device, sdr_ctx **ctx);
int sdr_ctx_destroy(sdr_ctx *ctx);
/* Use an external HIP stream (hipStream_t as void*); NULL restores the
 * context's own stream. */
int sdr_ctx_set_stream(sdr_ctx *ctx, void *hip_stream);
void *sdr_ctx_get_stream(sdr_ctx *ctx);
int sdr_ctx_synchronize(sdr_ctx *ctx);
const char *sdr_ctx_last_error(sdr_ctx *ctx);

/* FIR arithmetic of the fused front end (sdr_frontend_*_dev and the calls
 * built on it).  SDR_ARITH_EXACT (default): every product and sum rounded
 * separately in the reference's order -- the bits of src/filter.cpp:123-140.
 * SDR_ARITH_FMA: the same taps in the same order with one fused
 * multiply-add per tap (one rounding instead of two); no reference
 * counterpart, outputs within the fp32 tolerance of DESIGN.md section 2. */
#define SDR_ARITH_EXACT 0
#define SDR_ARITH_FMA 1
int sdr_ctx_set_arith(sdr_ctx *ctx, int mode);

/* Launch order of sdr_stereo_pcm_u8_dev (same outputs either way):
 * SDR_FORK_SIDE runs the branches that do not wait for the PLL recurrence on
 * a second HIP stream beside it, SDR_FORK_SERIAL runs everything on the
 * context's stream, SDR_FORK_AUTO (default) forks while the recurrence
 * occupies at most CUs/4 waves (<= 4,096 streams on MI355X).  The default
 * at creation can be set by the environment variable SDR_STEREO_FORK. */
#define SDR_FORK_AUTO (-1)
#define SDR_FORK_SERIAL 0
#define SDR_FORK_SIDE 1
int sdr_ctx_set_stereo_fork(sdr_ctx *ctx, int mode);

/* Kernel-selection switches (process-wide).  Several calls have more than
 * one kernel with identical outputs (bit-identical, or -- fp16 arm -- the same
 * tolerance contract); a switch picks one, for A/B timing and for the parity
 * tests, which run every kernel.  Each switch starts at the environment
 * variable of the same name if it is set when the library first needs it,
 * else at the measured default, and is then changed only by
 * sdr_set_switch: launches read it without scanning the environment.  Names:
 * SDR_FIR_SC, SDR_FIR_SC_U8, SDR_RESAMPLE_LP, SDR_RESAMPLE_LOADER,
 * SDR_RESAMPLE_RS, SDR_RESAMPLE_PP, SDR_LONG_VTAP, SDR_F16_MFMA,
 * SDR_F16_HEAD, SDR_F16_W8, SDR_PLL_FAST, SDR_PLL_GUARD, SDR_LONG_COMMIT.  An unknown name is
 * SDR_EINVAL.  A change applies to launches enqueued after it. */
int sdr_set_switch(const char *name, int value);
int sdr_get_switch(const char *name, int *value);

/* Device memory helpers so a C/C++ caller needs no HIP headers. */
int sdr_dev_alloc(sdr_ctx *ctx, size_t bytes, void **ptr);
int sdr_dev_free(sdr_ctx *ctx, void *ptr);
int sdr_copy_h2d(sdr_ctx *ctx, void *dst, const void *src, size_t bytes); /* synchronous */
int sdr_copy_d2h(sdr_ctx *ctx, void *dst, const void *src, size_t bytes); /* synchronous */
int sdr_dev_memset(sdr_ctx *ctx, void *dst, int value, size_t bytes);   /* stream-ordered */

/* Pinned host buffers, stream-ordered copies and events, for callers that
 * overlap their own I/O with the device work (host/sdr_project.cpp: the
 * HIP-stream replacement of src/project.cpp's per-block threads + queue). */
typedef struct sdr_event sdr_event;
int sdr_host_alloc(sdr_ctx *ctx, size_t bytes, void **ptr); /* page-locked */
int sdr_host_free(sdr_ctx *ctx, void *ptr);
int sdr_copy_h2d_async(sdr_ctx *ctx, void *dst, const void *src, size_t bytes); /* stream-ordered */
int sdr_copy_d2h_async(sdr_ctx *ctx, void *dst, const void *src, size_t bytes); /* stream-ordered */
int sdr_event_create(sdr_ctx *ctx, sdr_event **ev);
int sdr_event_record(sdr_ctx *ctx, sdr_event *ev);      /* marks the work enqueued so far */
int sdr_event_synchronize(sdr_ctx *ctx, sdr_event *ev); /* blocks until that work is done */
int sdr_event_destroy(sdr_ctx *ctx, sdr_event *ev);
/* The context's stream waits (on the device) for the work an event marked,
 * which may have been recorded on another context's stream of the same device. */
int sdr_ctx_wait_event(sdr_ctx *ctx, sdr_event *ev);

/* HIP-graph capture of the context's stream: sdr_graph_begin, then any
 * stream-ordered *_dev / *_async calls (recorded, not run), then
 * sdr_graph_end instantiates them; sdr_graph_launch replays the recorded
 * sequence on the context's stream with the same pointers (state arrays
 * carry across replays exactly as across direct calls).  Replaces the
 * per-block launch sequence of a streaming caller (src/project.cpp:289-318
 * runs one block at a time) by one launch.  The stream must not be the null
 * stream; calls that synchronise fail while capturing.
 * A graph replays the context's internal scratch buffers it was recorded
 * with, so while any graph of the context is alive (or a capture is in
 * progress) a call that would need larger scratch fails with SDR_EINVAL
 * instead of reallocating under the graph: make one direct call of the
 * largest shape before capturing, or destroy the graphs first.
 * The library only knows the graphs sdr_graph_end made.  A caller that
 * captures the context's stream itself (after sdr_ctx_set_stream, e.g. with
 * torch.cuda.graph) must size the scratch by one direct call of the largest
 * shape first and then pin it with sdr_ctx_pin_scratch(ctx, 1) for as long as
 * its graphs live: while pinned, growth is refused (SDR_EINVAL) instead of
 * freeing buffers the caller's graph still replays.  sdr_ctx_pin_scratch(ctx,
 * 0) unpins. */
int sdr_ctx_pin_scratch(sdr_ctx *ctx, int pinned);
typedef struct sdr_graph sdr_graph;
int sdr_graph_begin(sdr_ctx *ctx);
int sdr_graph_end(sdr_ctx *ctx, sdr_graph **graph);
int sdr_graph_launch(sdr_ctx *ctx, sdr_graph *graph);
int sdr_graph_destroy(sdr_ctx *ctx, sdr_graph *graph);

/* --------------------------------------------------- coefficient design -- */
/* impulseResponseLPF / impulseResponseBPF, src/filter.cpp:14-49
 * (filter.h:17, :27): windowed-sinc taps with the up-factor gain folded in,
 * bit-identical to the reference.  Host code (one-time setup). h: ntaps. */
int sdr_taps_lpf(float Fs, float Fc, int ntaps, int up, float *h);
int sdr_taps_bpf(float Fs, float Fb, float Fe, int ntaps, int up, float *h);

/* ------------------------------------------------------------- sizing -- */
/* Output length of resampleBlockConvolveFIR, src/filter.cpp:149:
 * (size_t)((n / (float)down) * up). */
long long sdr_resample_out_len(int up, int down, long long n);

/* -------------------------------------------- host-pointer, synchronous -- */
/* blockConvolveFIR, src/filter.cpp:66-83 (filter.h:19).  y: n floats. */
int sdr_fir_block_f32(sdr_ctx *ctx, const float *x, long long n, const float *h, int ntaps,
                      float *state, int ns, float *y);
/* downsampleBlockConvolveFIR, src/filter.cpp:123-140 (filter.h:25).
 * y: n/D floats; requires n % D == 0. */
int sdr_fir_decim_f32(sdr_ctx *ctx, int D, const float *x, long long n, const float *h, int ntaps,
                      float *state, int ns, float *y);
/* resampleBlockConvolveFIR, src/filter.cpp:142-173 (filter.h:26).
 * y: sdr_resample_out_len(up, down, n) floats (y_cap is checked against it). */
int sdr_resample_f32(sdr_ctx *ctx, int up, int down, const float *x, long long n, const float *h,
                     int ntaps, float *state, int ns, float *y, long long y_cap);
/* fmDemodArctan, src/filter.cpp:85-102 (filter.h:20).  out: n floats. */
int sdr_fm_demod_f32(sdr_ctx *ctx, const float *I, const float *Q, long long n, float *prev_i,
                     float *prev_q, float *out);
/* The whole front end of src/project.cpp:86-90 fused into one launch:
 * FIR+decimate(I), FIR+decimate(Q), discriminator.  demod: n/D floats. */
int sdr_frontend_f32(sdr_ctx *ctx, int D, const float *I, const float *Q, long long n, const float *h,
                     int ntaps, float *state_i, float *state_q, int ns, float *prev_i, float *prev_q,
                     float *demod);
/* Same, reading the RTL-SDR wire format directly: interleaved u8 I/Q
 * (2*npairs bytes) converted as src/iofunc.cpp:117-119 and de-interleaved as
 * src/project.cpp:78-81, inside the kernel. */
int sdr_frontend_u8(sdr_ctx *ctx, int D, const uint8_t *iq, long long npairs, const float *h, int ntaps,
                    float *state_i, float *state_q, int ns, float *prev_i, float *prev_q, float *demod);

/* -------------------------------- device-resident, batched, stream-ordered -- */
/* The tiled kernels stream 16-B vectors (8-B for u8 input): inputs whose
 * stream rows are not so aligned run on the generic kernel instead -- same
 * bits, lower throughput.  Output rows of any alignment are accepted. */
int sdr_fir_decim_f32_dev(sdr_ctx *ctx, int D, const float *x, long long n, int nstreams, long long x_stride,
                          const float *h, int ntaps, float *state, int ns, float *y, long long y_stride);
int sdr_fir_block_f32_dev(sdr_ctx *ctx, const float *x, long long n, int nstreams, long long x_stride,
                          const float *h, int ntaps, float *state, int ns, float *y, long long y_stride);
int sdr_fm_demod_f32_dev(sdr_ctx *ctx, const float *I, const float *Q, long long n, int nstreams,
                         long long stride, float *prev_i, float *prev_q, float *out, long long out_stride);
int sdr_frontend_f32_dev(sdr_ctx *ctx, int D, const float *I, const float *Q, long long n, int nstreams,
                         long long x_stride, const float *h, int ntaps, float *state_i, float *state_q, int ns,
                         float *prev_i, float *prev_q, float *demod, long long out_stride);
/* iq_stride in bytes (multiple of 8); npairs per stream. */
int sdr_frontend_u8_dev(sdr_ctx *ctx, int D, const uint8_t *iq, long long npairs, int nstreams,
                        long long iq_stride, const float *h, int ntaps, float *state_i, float *state_q, int ns,
                        float *prev_i, float *prev_q, float *demod, long long out_stride);
int sdr_resample_f32_dev(sdr_ctx *ctx, int up, int down, const float *x, long long n, int nstreams,
                         long long x_stride, const float *h, int ntaps, float *state, int ns, float *y,
                         long long y_stride);

/* A resampler plan: the lane-phase kernel's tap tables (each phase's taps,
 * pre-shifted per window alignment, and the bank-aware lane table) built
 * ONCE from the device taps h, instead of by a small launch in every
 * sdr_resample_f32_dev call.  A streaming caller's taps do not change
 * (src/project.cpp:262-266 designs them once), so the per-block call is a
 * single launch.  h is read at creation by that kernel and at each call by
 * the fallback kernels (other shapes): it must not change while the plan
 * lives.  Same outputs, state and preconditions as sdr_resample_f32_dev.
 * sdr_resample_plan_destroy waits for the table build and for the last
 * direct call on every stream that used the plan (one event per stream), not
 * for the whole device; graph replays of calls with the plan must have
 * completed (not only been destroyed) before it. */
typedef struct sdr_resample_plan sdr_resample_plan;
int sdr_resample_plan_create(sdr_ctx *ctx, int up, int down, const float *h, int ntaps,
                             sdr_resample_plan **plan);
int sdr_resample_plan_f32_dev(sdr_ctx *ctx, const sdr_resample_plan *plan, const float *x, long long n,
                              int nstreams, long long x_stride, float *state, int ns, float *y,
                              long long y_stride);
int sdr_resample_plan_destroy(sdr_ctx *ctx, sdr_resample_plan *plan);

/* BASELINE config 5's fp16 arm of blockConvolveFIR (src/filter.cpp:66-83):
 * x and state are fp16 (IEEE binary16, [nstreams][x_stride] / [nstreams][ns]),
 * taps fp32 (rounded to fp16 inside), y fp32.  fp32 accumulation of fp16
 * products: a Toeplitz GEMM on v_mfma_f32_32x32x16_f16 when ntaps % 8 == 0,
 * ntaps <= 4096 and n >= 8 (one launch), else v_dot2_f32_f16.  NOT bit-exact
 * with the reference -- a tolerance arm; the fp32 calls above are the exact
 * path.  Rows must be 16-B aligned. */
/* Which kernel sdr_fir_block_f16_dev runs for ntaps under the current
 * environment (blocks of n >= 8): 1 = the MFMA Toeplitz GEMM, 0 = v_dot2. */
int sdr_fir_block_f16_kernel(int ntaps);
int sdr_fir_block_f16_dev(sdr_ctx *ctx, const void *x, long long n, int nstreams, long long x_stride,
                          const float *h, int ntaps, void *state, int ns, float *y, long long y_stride);
/* A tap plan for the fp16 arm: the MFMA kernel's shifted fp16 tap copies
 * built ONCE from the device taps h (a streaming caller's taps do not change,
 * src/project.cpp:262-266), instead of in every workgroup of every call.  h
 * must stay valid and unchanged while the plan lives (the v_dot2 fallback and
 * shapes without a plan read it per call).  Same outputs, state and
 * preconditions as sdr_fir_block_f16_dev.  Destroy waits for the plan's build
 * and every direct call on every stream that used it; graph replays of calls
 * with the plan must have completed before it. */
typedef struct sdr_fir_f16_plan sdr_fir_f16_plan;
int sdr_fir_f16_plan_create(sdr_ctx *ctx, const float *h, int ntaps, sdr_fir_f16_plan **plan);
int sdr_fir_block_f16_plan_dev(sdr_ctx *ctx, const sdr_fir_f16_plan *plan, const void *x, long long n, int nstreams,
                               long long x_stride, void *state, int ns, float *y, long long y_stride);
int sdr_fir_f16_plan_destroy(sdr_ctx *ctx, sdr_fir_f16_plan *plan);
/* fp32 -> fp16 (round to nearest even), count elements, stream-ordered. */
int sdr_f32_to_f16_dev(sdr_ctx *ctx, const float *x, long long count, void *y);

/* ------------------------------- device-resident mono back end (8(f)) -- */
/* delayBlock (src/filter.cpp, as src/project.cpp:114 uses it), batched:
 * out = state ++ in[0 .. n-ns), state <- in[n-ns .. n).  ns <= 256. */
int sdr_delay_f32_dev(sdr_ctx *ctx, const float *in, long long n, int nstreams, long long in_stride, float *state,
                      int ns, float *out, long long out_stride);
/* The output stage of src/project.cpp:311-314: NaN -> 0, else
 * (short)(x * 16384) with the reference build's x86-64 conversion. */
int sdr_pcm_s16_dev(sdr_ctx *ctx, const float *x, long long n, int nstreams, long long x_stride, int16_t *pcm,
                    long long pcm_stride);
/* The whole mono path of src/project.cpp:72-118 + 304-314 for one block of
 * every stream, device-resident: u8 IQ -> fused front end -> delay ->
 * audio resampler (up/down; up == 1 is FIR + decimate) -> s16 PCM.
 * Bit-identical to the reference program's output (tests). */
int sdr_mono_pcm_u8_dev(sdr_ctx *ctx, int D, const uint8_t *iq, long long npairs, int nstreams, long long iq_stride,
                        const float *h_rf, int rf_taps, float *state_i, float *state_q, int ns_rf, float *prev_i,
                        float *prev_q, float *delay_state, int ns_delay, int up, int down, const float *h_audio,
                        int audio_taps, float *state_audio, int ns_audio, int16_t *pcm, long long pcm_stride);

/* ----------------------------------------------- stereo back end -------- */
/* fmPLL (src/filter.cpp:174-228) for nstreams independent streams, one lane
 * per stream (the recurrence is sequential in time).  pll is [nstreams][6]:
 * {feedbackI, feedbackQ, integrator, phaseEst, trigOffset, nco_state}
 * (src/project.cpp:48-55 initial values 1, 0, 0, 0, 0, 1), updated in place.
 * mix == NULL: out = ncoOut; else out = ncoOut * mix * 2, i.e. fmPLL fused
 * with pointwiseMultiply (src/filter.cpp:253-266) as src/project.cpp:126
 * applies it.  atan2/cos/sin are evaluated in double, as the reference does. */
int sdr_fm_pll_dev(sdr_ctx *ctx, const float *in, long long n, int nstreams, long long in_stride, float freq,
                   float Fs, float nco_scale, float phase_adjust, float norm_bw, float *pll, const float *mix,
                   long long mix_stride, float *out, long long out_stride);
/* pointwiseAdd/Subtract (src/filter.cpp:267-288) + interleave (:289-301) +
 * the s16 stage of src/project.cpp:311-314: pcm[2i] = s16(mono[i] + stereo[i]),
 * pcm[2i+1] = s16(mono[i] - stereo[i]). */
int sdr_stereo_pcm_dev(sdr_ctx *ctx, const float *mono, const float *stereo, long long n, int nstreams,
                       long long stride, int16_t *pcm, long long pcm_stride);

/* Device taps of the stereo back end (src/project.cpp:262-273). */
typedef struct sdr_stereo_taps {
  const float *h_rf;     /* RF low-pass, rf_taps */
  int rf_taps;
  const float *h_audio;  /* audio low-pass (x up gain), audio_taps */
  int audio_taps;
  const float *h_pilot;  /* 18.5-19.5 kHz band-pass, bpf_taps */
  const float *h_stereo; /* 22-54 kHz band-pass, bpf_taps */
  int bpf_taps;
} sdr_stereo_taps;

/* Device state of the stereo back end, one row per stream
 * (src/project.cpp:25-55: RFState, AudioState, PLLState). */
typedef struct sdr_stereo_state {
  float *state_i, *state_q; /* [nstreams][ns_rf] */
  int ns_rf;
  float *prev_i, *prev_q;   /* [nstreams] */
  float *delay_state;       /* [nstreams][ns_delay] mono delay (num_taps/2) */
  int ns_delay;
  float *state_audio;       /* [nstreams][ns_audio] mono resampler */
  float *stereo_lp_state;   /* [nstreams][ns_audio] stereo resampler */
  int ns_audio;
  float *pilot_state, *stereo_state; /* [nstreams][ns_bpf] */
  int ns_bpf;
  float *pll;               /* [nstreams][6], see sdr_fm_pll_dev */
} sdr_stereo_state;

/* The whole stereo path of src/project.cpp:72-132 + 304-314 for one block of
 * every stream, device-resident: u8 IQ -> front end -> {delay -> mono
 * resampler, pilot BPF -> PLL x stereo BPF -> stereo resampler} -> L/R
 * interleaved s16 PCM (2 * audio samples per stream and block).  The PLL
 * constants are project.cpp's (19 kHz, ncoScale 2, phaseAdjust 0, normalised
 * bandwidth 0.01); audio_fs is the IF rate it runs at. */
int sdr_stereo_pcm_u8_dev(sdr_ctx *ctx, int D, const uint8_t *iq, long long npairs, int nstreams, long long iq_stride,
                          int up, int down, float audio_fs, const sdr_stereo_taps *taps, sdr_stereo_state *state,
                          int16_t *pcm, long long pcm_stride);

/* The same stereo path in two stages, cut where the PLL recurrence starts,
 * with one block's intermediates in a work object: sdr_stereo_front_u8_dev
 * runs the front end, delay + mono resampler and both band-pass filters
 * (src/project.cpp:72-121); sdr_stereo_back_dev the PLL recurrence, NCO x
 * stereo band, stereo resampler and the L/R s16 stage (:123-132, 304-314).
 * The stages touch disjoint parts of the state (front: state_i/q, prev_*,
 * delay, state_audio, pilot/stereo band-pass; back: pll, stereo_lp_state), so
 * block b+1's front stage may run on one context's stream while block b's
 * back stage runs on another's -- order them with sdr_event_record /
 * sdr_ctx_wait_event and give each block in flight its own work object
 * (host/sdr_project.cpp).  Outputs equal sdr_stereo_pcm_u8_dev's. */
/* sdr_stereo_work_destroy waits for every direct front / back call on every
 * context's stream that used the work (one event per stream), then frees it;
 * graph replays of calls with the work must have completed before it. */
typedef struct sdr_stereo_work sdr_stereo_work;
int sdr_stereo_work_create(sdr_ctx *ctx, int D, long long npairs, int up, int down, int nstreams,
                           sdr_stereo_work **work);
int sdr_stereo_work_destroy(sdr_ctx *ctx, sdr_stereo_work *work);
int sdr_stereo_front_u8_dev(sdr_ctx *ctx, const uint8_t *iq, long long iq_stride, const sdr_stereo_taps *taps,
                            sdr_stereo_state *state, sdr_stereo_work *work);
int sdr_stereo_back_dev(sdr_ctx *ctx, float audio_fs, const sdr_stereo_taps *taps, sdr_stereo_state *state,
                        sdr_stereo_work *work, int16_t *pcm, long long pcm_stride);
/* The back stage's two halves: the recurrence (PLL state) and the post stage
 * (NCO x stereo band, stereo resampler, L/R s16; the stereo resampler state),
 * so block b's post stage can run on the front stage's stream after block
 * b+1's front stage while block b+1's recurrence runs on the back stream
 * (the caller orders post(b) after pll(b) with an sdr_event).  Together they
 * equal sdr_stereo_back_dev. */
int sdr_stereo_pll_dev(sdr_ctx *ctx, float audio_fs, sdr_stereo_state *state, sdr_stereo_work *work);
int sdr_stereo_post_dev(sdr_ctx *ctx, const sdr_stereo_taps *taps, sdr_stereo_state *state, sdr_stereo_work *work,
                        int16_t *pcm, long long pcm_stride);

/* The mono path in two stages (like the stereo pair above): sdr_mono_front_u8_dev
 * runs the RF front end of one block into the work's row (src/project.cpp:72-93);
 * sdr_mono_back_dev the delay line, the audio filter and the s16 stage
 * (:114-118, 304-314).  The stages touch disjoint state (front: state_i/q,
 * prev_i/q; back: delay_state, state_audio), so block b+1's front stage may run
 * on one context's stream while block b's back stage runs on another's --
 * order them with events and give each block in flight its own work.  The
 * work is created for one shape and one set of tap / state lengths (it picks
 * the fused row layout when up == 1 and the fast kernels cover the filters);
 * outputs equal sdr_mono_pcm_u8_dev's.  destroy waits for every stream that
 * used the work. */
typedef struct sdr_mono_work sdr_mono_work;
int sdr_mono_work_create(sdr_ctx *ctx, int D, long long npairs, int up, int down, int nstreams, int ns_delay,
                         const float *h_rf, int rf_taps, int ns_rf, const float *h_audio, int audio_taps,
                         int ns_audio, sdr_mono_work **work);
int sdr_mono_work_destroy(sdr_ctx *ctx, sdr_mono_work *work);
int sdr_mono_front_u8_dev(sdr_ctx *ctx, const uint8_t *iq, long long iq_stride, const float *h_rf, int rf_taps,
                          float *state_i, float *state_q, int ns_rf, float *prev_i, float *prev_q,
                          sdr_mono_work *work);
int sdr_mono_back_dev(sdr_ctx *ctx, const float *h_audio, int audio_taps, float *state_audio, int ns_audio,
                      float *delay_state, sdr_mono_work *work, int16_t *pcm, long long pcm_stride);

/* ---------------------------------------------------- synthetic input -- */
/* Fill nstreams x npairs interleaved u8 IQ of a noisy FM carrier on the
 * device (counter-based, keyed by (seed, stream, sample)); used by the
 * benchmark so no host traffic is needed.  Not bit-identical to the numpy
 * generator in sdrhip/synth.py -- both are just "FM-like" test signals. */
int sdr_synth_fm_u8_dev(sdr_ctx *ctx, uint8_t *iq, long long npairs, int nstreams, long long iq_stride,
                        unsigned long long seed);
/* u8 interleaved -> planar f32 (src/iofunc.cpp:117-119 + project.cpp:78-81). */
int sdr_u8_to_planar_dev(sdr_ctx *ctx, const uint8_t *iq, long long npairs, int nstreams, long long iq_stride,
                         float *I, float *Q, long long x_stride);

/* ------------------------------------- device transcendental routines -- */
/* The PLL and NCO kernels evaluate fmPLL's atan2 / sin / cos
 * (src/filter.cpp:199-221: glibc's double routines on float arguments, each
 * result stored to float) with csrc/libm_exact.hpp, built to give glibc's
 * float for every argument.  These calls run those same device routines in
 * bulk so the parity tests can prove it on the GPU (tests/test_libm_exact.py):
 *   sdr_libm_sincos_hash_dev: every finite fp32 bit pattern u with u >> 20 in
 *     [chunk_lo, chunk_hi) (2^20 per chunk; 4096 chunks cover all 2^32);
 *     hash[chunk] += sum of a 64-bit mix of (u, sin float, cos float) -- zero
 *     hash[] first.  mode 0: the product routine; 1: the platform library's
 *     double sin / cos rounded to float (for comparison only).
 *   sdr_libm_sincos_diff_dev: the arguments where the two differ:
 *     args[2k] = u, args[2k+1] = 1 (sin) | 2 (cos), k < cap; *count (device,
 *     zero it first) counts them all.
 *   sdr_libm_eval_dev: out[i] = f(a[i] [, b[i]]) with fn 0 sin, 1 cos,
 *     2 atan2(a, b) (product routines), 3 / 4 / 5 the platform library's.
 *   sdr_libm_atan2_screen_dev: pairs first .. first+count-1 of a seeded
 *     family; counters[0] (device, zeroed) counts those the short path does
 *     not certify (offsets into cand, cap cand_cap), counters[1] those whose
 *     exact value lies within 4 double ulps of a float rounding midpoint,
 *     written to out[4k..4k+3] = {y, x, atan2 float, 0} bits (k < out_cap). */
int sdr_libm_sincos_hash_dev(sdr_ctx *ctx, int mode, unsigned chunk_lo, unsigned chunk_hi,
                             unsigned long long *hash);
int sdr_libm_sincos_diff_dev(sdr_ctx *ctx, unsigned chunk_lo, unsigned chunk_hi, unsigned long long *count,
                             unsigned *args, long long cap);
int sdr_libm_eval_dev(sdr_ctx *ctx, int fn, const float *a, const float *b, long long n, float *out);
int sdr_libm_atan2_screen_dev(sdr_ctx *ctx, unsigned long long seed, unsigned long long first,
                              unsigned long long count, unsigned *cand, long long cand_cap, unsigned *out,
                              long long out_cap, unsigned long long *counters);

#ifdef __cplusplus
}
#endif
#endif /* SDR_HIP_H */
