/*
 * sdr_oracle.h -- CPU restatement of the reference DSP block library.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in the product (the HIP library, the
 * drop-in filter implementation) links or calls this.  Only tests/,
 * __graft_entry__.smoke() and bench.py's cpu_baseline leg may use it, and
 * only as the checker / the timed CPU baseline.
 *
 * Every function restates one function of the reference's src/filter.cpp
 * (ghotrs4/3DY4-Real-Time-Software-defined-Radio-) loop for loop, with the
 * same float/double promotion and the same accumulation order, so that its
 * output is bit-identical to the compiled reference on the same machine.
 * That claim is pinned by tests/test_oracle_golden.py against fixtures
 * produced by the compiled reference itself (tests/golden/make_golden.py).
 *
 * Pointer/length form: outputs are caller-allocated; the reference's
 * std::vector resize/clear rules become "write exactly this many elements"
 * (the *_len helpers give the counts).  Return value 0 = ok, -1 = a
 * precondition the reference would violate silently (heap OOB / UB).
 */
#ifndef SDR_ORACLE_H
#define SDR_ORACLE_H

#include <stddef.h>

#ifdef __cplusplus
extern "C" {
#endif

/* src/filter.cpp:14-29 */
long or_taps_lpf(float Fs, float Fc, unsigned short ntaps, int up, float *h);
/* src/filter.cpp:31-49 */
long or_taps_bpf(float Fs, float Fb, float Fe, unsigned short ntaps, int up, float *h);

/* src/filter.cpp:53-64 ; y has nx + nh - 1 elements */
long or_convolve_full(const float *x, long nx, const float *h, int nh, float *y);
/* src/filter.cpp:66-83 ; y has nx elements, state (ns) updated in place */
long or_fir_block(const float *x, long nx, const float *h, int nh, float *state, int ns, float *y);
/* src/filter.cpp:85-102 ; out has n elements, prev_i/prev_q updated */
long or_fm_demod(const float *I, const float *Q, long n, float *prev_i, float *prev_q, float *out);
/* src/filter.cpp:104-110 ; out has ceil(n/factor) elements */
long or_downsample(const float *x, long n, long factor, float *out);
/* src/filter.cpp:112-121 ; out has n*max(factor,1) elements */
long or_upsample(const float *x, long n, long factor, float *out);
/* src/filter.cpp:123-140 ; y has nx/D elements */
long or_fir_decim(int D, const float *x, long nx, const float *h, int nh, float *state, int ns, float *y);
/* src/filter.cpp:149 -- output length of resampleBlockConvolveFIR */
long or_resample_len(int up, int down, long nx);
/* src/filter.cpp:142-173 ; y has or_resample_len() elements */
long or_resample(int up, int down, const float *x, long nx, const float *h, int nh, float *state, int ns, float *y);
/* src/filter.cpp:174-228 ; pll[6] = {feedbackI, feedbackQ, integrator, phaseEst, trigOffset, nco_state} */
long or_fm_pll(const float *in, long n, float freq, float Fs, float nco_scale, float phase_adjust,
              float norm_bw, float *nco_out, float *pll);
/* src/filter.cpp:229-251 */
long or_delay_block(const float *in, long n, float *state, int ns, float *out);
/* src/filter.cpp:253-290 */
long or_pointwise_mul(const float *a, long na, const float *b, long nb, float *out);
long or_pointwise_add(const float *a, long na, const float *b, long nb, float *out);
long or_pointwise_sub(const float *a, long na, const float *b, long nb, float *out);
/* src/filter.cpp:291-301 */
long or_interleave(const float *l, long nl, const float *r, long nr, float *out);
/* src/project.cpp:311-314: float -> s16 PCM (NaN -> 0, x*16384 truncated) */
long or_pcm_s16(const float *x, long n, short *out);

/* src/iofunc.cpp:113-119 + src/project.cpp:78-81: u8 interleaved IQ -> planar float */
long or_u8_to_planar(const unsigned char *iq, long npairs, float *I, float *Q);

/* Fused mode-0 front end exactly as src/project.cpp:72-93 sequences it:
 * FIR+decimate I, FIR+decimate Q, then the discriminator.  Convenience for
 * the CPU baseline; each step is the restatement above. */
long or_frontend(int D, const float *I, const float *Q, long n, const float *h, int nh,
                float *state_i, float *state_q, int ns, float *prev_i, float *prev_q,
                float *scratch_i, float *scratch_q, float *demod);

#ifdef __cplusplus
}
#endif
#endif
