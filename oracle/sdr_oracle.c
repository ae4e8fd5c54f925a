/*
 * sdr_oracle.c -- scalar C restatement of the reference's src/filter.cpp.
 *
 * TEST INFRASTRUCTURE ONLY (see sdr_oracle.h).  Built with
 *   gcc -O2 -std=c11 -ffp-contract=off
 * so that, like the reference (g++ -O3 -std=c++17, src/Makefile:4, which on
 * x86-64 means SSE2 scalar math and no contraction), every float operation is
 * a separately rounded IEEE-754 op.  Accumulation order, float<->double
 * promotion points and sizing rules follow the reference line by line; the
 * citations name the line each block restates.
 */
#include "sdr_oracle.h"

#include <math.h>
#include <string.h>

#define OR_PI 3.14159265358979323846 /* include/dy4.h:14 */

/* ---------------------------------------------------------------- taps -- */

/* src/filter.cpp:14-29.  Norm_cutoff is a float quotient widened to double;
 * the sinc is evaluated in double and stored to float, then the float tap is
 * widened again for the sin^2 window and the gain (pow(.,2) is folded to a
 * product by the compiler at -O3; it is exact-equivalent). */
long or_taps_lpf(float Fs, float Fc, unsigned short ntaps, int up, float *h)
{
    const int T = ntaps;
    const double nc = (double)(Fc / (Fs / 2));
    for (int i = 0; i < T; i++) {
        float v;
        if (i == (T - 1) / 2) {
            v = (float)nc;
        } else {
            const double arg = OR_PI * nc * ((double)i - ((double)(float)T - 1.0) / 2.0);
            v = (float)(nc * sin(arg) / arg);
        }
        const double w = sin((double)i * OR_PI / (double)T);
        v = (float)((double)v * (w * w) * (double)(float)up);
        h[i] = v;
    }
    return 0;
}

/* src/filter.cpp:31-49 */
long or_taps_bpf(float Fs, float Fb, float Fe, unsigned short ntaps, int up, float *h)
{
    const int T = ntaps;
    const double ncent = (double)(((Fe + Fb) / 2) / (Fs / 2));
    const double npass = (double)((Fe - Fb) / (Fs / 2));
    for (int i = 0; i < T; i++) {
        float v;
        if (i == (T - 1) / 2) {
            v = (float)npass;
        } else {
            const double arg = OR_PI * npass / 2 * ((double)i - ((double)(float)T - 1.0) / 2.0);
            v = (float)(npass * sin(arg) / arg);
        }
        v = (float)((double)v * cos((double)(i - (T - 1) / 2) * OR_PI * ncent));
        const double w = sin((double)i * OR_PI / (double)T);
        v = (float)((double)v * (w * w) * (double)(float)up);
        h[i] = v;
    }
    return 0;
}

/* ----------------------------------------------------------- convolution -- */

/* src/filter.cpp:53-64: y[n] = sum_k h[k] x[n-k] over the full support. */
long or_convolve_full(const float *x, long nx, const float *h, int nh, float *y)
{
    const long ny = nx + nh - 1;
    for (long n = 0; n < ny; n++) {
        float acc = 0.0f;
        for (int k = 0; k < nh; k++) {
            const long j = n - k;
            if (j >= 0 && j < nx)
                acc = acc + h[k] * x[j];
        }
        y[n] = acc;
    }
    return 0;
}

/* Read x~[j]: x[j] for j >= 0, else the saved tail state[ns + j]. */
static inline float xt(const float *x, const float *state, int ns, long j)
{
    return j >= 0 ? x[j] : state[ns + j];
}

/* src/filter.cpp:66-83.  Preconditions the reference leaves as UB:
 * ns >= nh-1 (state index ns-(k-n) >= 0) and nx >= ns (state.assign). */
long or_fir_block(const float *x, long nx, const float *h, int nh, float *state, int ns, float *y)
{
    if (ns < nh - 1 || nx < ns) return -1;
    for (long n = 0; n < nx; n++) {
        float acc = 0.0f;
        for (int k = 0; k < nh; k++)
            acc = acc + h[k] * xt(x, state, ns, n - k);
        y[n] = acc;
    }
    memmove(state, x + nx - ns, (size_t)ns * sizeof(float));
    return 0;
}

/* src/filter.cpp:123-140.  Only kept outputs are computed; y has nx/D
 * elements and the loop visits ceil(nx/D) of them, so nx % D != 0 is a heap
 * overflow in the reference -> rejected here. */
long or_fir_decim(int D, const float *x, long nx, const float *h, int nh, float *state, int ns, float *y)
{
    if (D <= 0 || nx % D != 0 || ns < nh - 1 || nx < ns) return -1;
    for (long n = 0; n < nx; n += D) {
        float acc = 0.0f;
        for (int k = 0; k < nh; k++)
            acc = acc + h[k] * xt(x, state, ns, n - k);
        y[n / D] = acc;
    }
    memmove(state, x + nx - ns, (size_t)ns * sizeof(float));
    return 0;
}

/* src/filter.cpp:149: y.resize((x.size()/(float)downFactor)*upFactor) --
 * a float quotient times a float, truncated by the size_t conversion. */
long or_resample_len(int up, int down, long nx)
{
    const float q = (float)nx / (float)down;
    const float f = q * (float)up;
    return (long)f;
}

/* src/filter.cpp:142-173.  For n = 0, M, 2M, ... < nx*L the polyphase
 * branch p = n mod L is summed k = p, p+L, ...; (n-k) is an exact multiple
 * of L.  Negative input indices read state[ns - (k-n)/L]. */
long or_resample(int up, int down, const float *x, long nx, const float *h, int nh, float *state, int ns, float *y)
{
    if (up <= 0 || down <= 0 || nx < ns) return -1;
    const long ny = or_resample_len(up, down, nx);
    const long nlim = nx * (long)up;
    /* outputs written by the loop: ceil(nlim / down) must fit in ny */
    if ((nlim + down - 1) / down > ny) return -1;
    /* deepest state index touched: (nh-1 - 0)/up for n = 0 */
    if (nh > 0 && (long)(nh - 1) / up > ns) return -1;
    for (long n = 0; n < nlim; n += down) {
        const int phase = (int)(n % up);
        float acc = 0.0f;
        for (int k = phase; k < nh; k += up) {
            if (n - k >= 0)
                acc = acc + h[k] * x[(n - k) / up];
            else
                acc = acc + h[k] * state[ns - (k - n) / up];
        }
        y[n / down] = acc;
    }
    memmove(state, x + nx - ns, (size_t)ns * sizeof(float));
    return 0;
}

/* -------------------------------------------------------- discriminator -- */

/* src/filter.cpp:85-102.  Lyons' arctan-free discriminator.  std::pow(float,
 * int) promotes to double, so I^2+Q^2 is summed in double (both squares are
 * exact) and rounded once to float; numerator and divide are float.  A zero
 * envelope yields 0.  prev_* become the last inputs. */
long or_fm_demod(const float *I, const float *Q, long n, float *prev_i, float *prev_q, float *out)
{
    if (n <= 0) return -1; /* reference reads I[I.size()-1] */
    for (long k = 0; k < n; k++) {
        const float p = (float)((double)I[k] * (double)I[k] + (double)Q[k] * (double)Q[k]);
        if (p == 0) {
            out[k] = 0.0f;
            continue;
        }
        const float ip = k > 0 ? I[k - 1] : *prev_i;
        const float qp = k > 0 ? Q[k - 1] : *prev_q;
        const float a = I[k] * (Q[k] - qp);
        const float b = Q[k] * (I[k] - ip);
        out[k] = (a - b) / p;
    }
    *prev_i = I[n - 1];
    *prev_q = Q[n - 1];
    return 0;
}

/* ------------------------------------------------------------ rate glue -- */

/* src/filter.cpp:104-110 */
long or_downsample(const float *x, long n, long factor, float *out)
{
    long m = 0;
    if (factor <= 0) return -1;
    for (long i = 0; i < n; i += factor) out[m++] = x[i];
    return m;
}

/* src/filter.cpp:112-121: each sample followed by factor-1 zeros */
long or_upsample(const float *x, long n, long factor, float *out)
{
    long m = 0;
    for (long i = 0; i < n; i++) {
        out[m++] = x[i];
        for (long j = factor; j > 1; j--) out[m++] = 0.0f;
    }
    return m;
}

/* ----------------------------------------------------------------- PLL -- */

/* src/filter.cpp:174-228.  State carried in float; the trig calls are the C
 * double-precision libm functions applied to float arguments (the reference
 * calls unqualified atan2/cos/sin, which resolve to ::atan2(double,double)
 * etc.), their results rounded back to float. */
long or_fm_pll(const float *in, long n, float freq, float Fs, float nco_scale, float phase_adjust,
              float norm_bw, float *nco_out, float *pll)
{
    if (n <= 0) return -1;
    const float Cp = 2.666f;
    const float Ci = 3.555f;
    const float Kp = norm_bw * Cp;
    const float Ki = norm_bw * norm_bw * Ci;
    float fbI = pll[0], fbQ = pll[1], integ = pll[2], phase = pll[3], toff = pll[4], nco = pll[5];

    nco_out[0] = nco;
    for (long k = 0; k < n; k++) {
        const float eI = (in[k] == 0 ? 1.0f : in[k]) * fbI;
        const float eQ = in[k] * (-1.0f * fbQ);
        const float eD = (float)atan2((double)eQ, (double)eI);
        integ = integ + Ki * eD;
        phase = phase + (Kp * eD + integ);
        toff = toff + 1.0f;
        const float arg = (float)(2 * OR_PI * (double)(freq / Fs) * (double)toff + (double)phase);
        fbI = (float)cos((double)arg);
        fbQ = (float)sin((double)arg);
        const float o = (float)cos((double)(arg * nco_scale + phase_adjust));
        if (k == n - 1)
            nco = o;
        else
            nco_out[k + 1] = o;
    }
    pll[0] = fbI; pll[1] = fbQ; pll[2] = integ; pll[3] = phase; pll[4] = toff; pll[5] = nco;
    return 0;
}

/* ------------------------------------------------------ elementwise glue -- */

/* src/filter.cpp:229-251: out = [state, in[0 .. n-ns)], state = in[n-ns ..) */
long or_delay_block(const float *in, long n, float *state, int ns, float *out)
{
    if (n < ns) return -1;
    memcpy(out, state, (size_t)ns * sizeof(float));
    memcpy(out + ns, in, (size_t)(n - ns) * sizeof(float));
    memcpy(state, in + n - ns, (size_t)ns * sizeof(float));
    return 0;
}

/* src/filter.cpp:253-266 (the x2 mixer gain is part of the op) */
long or_pointwise_mul(const float *a, long na, const float *b, long nb, float *out)
{
    const long n = na < nb ? na : nb;
    for (long i = 0; i < n; i++) out[i] = a[i] * b[i] * 2;
    return n;
}

/* src/filter.cpp:267-278: length follows the first operand */
long or_pointwise_add(const float *a, long na, const float *b, long nb, float *out)
{
    if (nb < na) return -1;
    for (long i = 0; i < na; i++) out[i] = a[i] + b[i];
    return na;
}

/* src/filter.cpp:279-290 */
long or_pointwise_sub(const float *a, long na, const float *b, long nb, float *out)
{
    if (nb < na) return -1;
    for (long i = 0; i < na; i++) out[i] = a[i] - b[i];
    return na;
}

/* src/filter.cpp:291-301: L0 R0 L1 R1 ... */
long or_interleave(const float *l, long nl, const float *r, long nr, float *out)
{
    const long n = nl + nr;
    for (long i = 0; i < n; i += 2) out[i] = l[i / 2];
    for (long i = 1; i < n; i += 2) out[i] = r[i / 2];
    return n;
}

/* src/project.cpp:311-314, the output stage: NaN -> 0, else
 * static_cast<short int>(x * 16384) (float product; the cast as the
 * reference's compiler emits it on x86-64: truncate to int32, keep the low
 * 16 bits; out-of-int32-range values give INT_MIN, i.e. 0). */
long or_pcm_s16(const float *x, long n, short *out)
{
    for (long k = 0; k < n; k++) {
        if (isnan(x[k])) {
            out[k] = 0;
        } else {
            const float v = x[k] * 16384;
            const int i = (v < 2147483648.0f && v >= -2147483648.0f) ? (int)v : (int)0x80000000u;
            out[k] = (short)(unsigned short)((unsigned)i & 0xffffu);
        }
    }
    return n;
}

/* ------------------------------------------------------- ingest + front -- */

/* src/iofunc.cpp:117-119: float(((unsigned char)u - 128) / 128.0), then the
 * de-interleave of src/project.cpp:78-81. */
long or_u8_to_planar(const unsigned char *iq, long npairs, float *I, float *Q)
{
    for (long i = 0; i < npairs; i++) {
        I[i] = (float)((double)((int)iq[2 * i] - 128) / 128.0);
        Q[i] = (float)((double)((int)iq[2 * i + 1] - 128) / 128.0);
    }
    return 0;
}

/* src/project.cpp:86-90 */
long or_frontend(int D, const float *I, const float *Q, long n, const float *h, int nh,
                float *state_i, float *state_q, int ns, float *prev_i, float *prev_q,
                float *scratch_i, float *scratch_q, float *demod)
{
    int rc = or_fir_decim(D, I, n, h, nh, state_i, ns, scratch_i);
    if (rc) return rc;
    rc = or_fir_decim(D, Q, n, h, nh, state_q, ns, scratch_q);
    if (rc) return rc;
    return or_fm_demod(scratch_i, scratch_q, n / D, prev_i, prev_q, demod);
}
