// libm_exact.hpp -- the float the reference stores from glibc's double sin /
// cos / atan2 of fp32 arguments, reproduced on the device (and, from the same
// source, on the host for the CPU proofs).
//
// The reference's fmPLL (src/filter.cpp:199-221) evaluates
//   errorD    = atan2(errorQ, errorI)               (float args, glibc double, stored to float)
//   feedbackI = cos(trigArg), feedbackQ = sin(trigArg)
//   ncoOut[k] = cos(trigArg*ncoScale + phaseAdjust)
// and keeps only the float roundings.  Two ~1-ulp double libraries (glibc
// here, OCML on the device) round to different floats only where the exact
// value lies within about an ulp of a float rounding midpoint, so "ROCm's
// double routines round to glibc's floats" cannot be shown by sampling.  These
// routines are built so that it can be shown:
//   1. fast path: the short-chain kernels of pll_fast.hpp (relative error
//      < 2^-46) with exact IEEE operations only (a true division instead of
//      v_rcp_f64), certified by pll_fast's midpoint windows (atan2: >= 1,024
//      double ulps from every float midpoint: the exact value and glibc's
//      double, both within a few ulps, round to this float; sin / cos: >= 32
//      ulps, their kernels being within ~1.4 ulps -- the exhaustive sweep
//      below checks every certified result);
//   2. otherwise a double-double evaluation accurate to ~2^-70 relative
//      (sin / cos: Payne-Hanek reduction of the fp32 argument against 320 bits
//      of 2/pi, Taylor series in double-double; atan2: one Newton step on
//      x sin(t) - y cos(t) = 0 from the fast result), rounded to the nearest
//      double and then to float -- exactly what glibc does where its double is
//      correctly rounded;
//   (the exhaustive sweep below found no argument where glibc's sin / cos
//   float differs from the correctly rounded double's float).
// Every operation is an IEEE-correct double operation (add, mul, fma, div,
// rint, ldexp, conversions), so host and device compute identical bits.
//
// Proof, not sampling:
//   - sin / cos: tests/libm_sweep.cpp evaluates these routines and glibc on
//     EVERY finite float (2^32 - 2^24 arguments); tests/test_libm_exact.py runs
//     it (CPU) and asserts zero mismatches; the device evaluates every finite
//     float too and its per-chunk hashes must equal glibc's, committed in
//     tests/golden/libm_sincos_hash.npz (tests/test_gpu_parity.py).
//   - atan2 (two arguments, 2^64 pairs): the sweep samples pairs, keeps every
//     pair whose exact value lies near a float midpoint, and the device and
//     host must reproduce glibc's float on each (committed fixture); the GPU
//     test additionally screens ~2^37 seeded pairs on the device and checks
//     every near-midpoint one against the box's glibc.
// Non-finite arguments, and atan2 with a zero argument, take the platform
// library (the results are the C standard's exact values or NaN).
#pragma once

#include <cmath>

#include "pll_fast.hpp"

#ifndef SDR_HD
#define SDR_HD __host__ __device__
#endif

namespace sdr {
namespace libmx {

// IEEE-exact operations for pll_fast's kernels (a true division, not v_rcp_f64)
struct ExactOps {
  SDR_HD static double fma(double a, double b, double c) { return __builtin_fma(a, b, c); }
  SDR_HD static double rcp(double u) { return 1.0 / u; }
};

// ---- double-double ---------------------------------------------------------
struct dd {
  double hi, lo;
};
SDR_HD inline dd two_sum(double a, double b) {
  const double s = a + b, bb = s - a;
  return {s, (a - (s - bb)) + (b - bb)};
}
SDR_HD inline dd fast_two_sum(double a, double b) {  // |a| >= |b| (or a == 0)
  const double s = a + b;
  return {s, b - (s - a)};
}
SDR_HD inline dd two_prod(double a, double b) {
  const double p = a * b;
  return {p, __builtin_fma(a, b, -p)};
}
SDR_HD inline dd dd_add(dd a, dd b) {
  dd s = two_sum(a.hi, b.hi);
  const dd t = two_sum(a.lo, b.lo);
  s.lo += t.hi;
  s = fast_two_sum(s.hi, s.lo);
  s.lo += t.lo;
  return fast_two_sum(s.hi, s.lo);
}
SDR_HD inline dd dd_neg(dd a) { return {-a.hi, -a.lo}; }
SDR_HD inline dd dd_mul(dd a, dd b) {
  dd p = two_prod(a.hi, b.hi);
  p.lo += a.hi * b.lo + a.lo * b.hi;
  return fast_two_sum(p.hi, p.lo);
}
SDR_HD inline dd dd_mul_d(dd a, double b) {
  dd p = two_prod(a.hi, b);
  p.lo += a.lo * b;
  return fast_two_sum(p.hi, p.lo);
}

// pi/2 = kP1 + kP2 + kP3 (+ 5.6e-50); 1/n! as double-doubles (exact rationals
// rounded twice: scripts in the commit that added this file)
constexpr double kP3 = -0x1.f1976b7ed8fbcp-110;
// 2/pi, fraction bits 1..384, big-endian 32-bit words
constexpr unsigned kTwoOverPiW[12] = {0xa2f9836eu, 0x4e441529u, 0xfc2757d1u, 0xf534ddc0u, 0xdb629599u, 0x3c439041u,
                                      0xfe5163abu, 0xdebbc561u, 0xb7246e3au, 0x424dd2e0u, 0x06492eeau, 0x09d1921cu};
// sin r = r * sum_k (-1)^k z^k / (2k+1)!,  cos r = sum_k (-1)^k z^k / (2k)!,  z = r^2, |r| <= pi/4:
// 14 / 15 terms leave < 2^-110 of the result
constexpr double kInvFact[29][2] = {
    {1.0, 0.0},
    {1.0, 0.0},
    {0x1.0000000000000p-1, 0.0},
    {0x1.5555555555555p-3, 0x1.5555555555555p-57},
    {0x1.5555555555555p-5, 0x1.5555555555555p-59},
    {0x1.1111111111111p-7, 0x1.1111111111111p-63},
    {0x1.6c16c16c16c17p-10, -0x1.f49f49f49f49fp-65},
    {0x1.a01a01a01a01ap-13, 0x1.a01a01a01a01ap-73},
    {0x1.a01a01a01a01ap-16, 0x1.a01a01a01a01ap-76},
    {0x1.71de3a556c734p-19, -0x1.c154f8ddc6c00p-73},
    {0x1.27e4fb7789f5cp-22, 0x1.cbbc05b4fa99ap-76},
    {0x1.ae64567f544e4p-26, -0x1.c062e06d1f209p-80},
    {0x1.1eed8eff8d898p-29, -0x1.2aec959e14c06p-83},
    {0x1.6124613a86d09p-33, 0x1.f28e0cc748ebep-87},
    {0x1.93974a8c07c9dp-37, 0x1.05d6f8a2efd1fp-92},
    {0x1.ae7f3e733b81fp-41, 0x1.1d8656b0ee8cbp-97},
    {0x1.ae7f3e733b81fp-45, 0x1.1d8656b0ee8cbp-101},
    {0x1.952c77030ad4ap-49, 0x1.ac981465ddc6cp-103},
    {0x1.6827863b97d97p-53, 0x1.eec01221a8b0bp-107},
    {0x1.2f49b46814157p-57, 0x1.2650f61dbdcb4p-112},
    {0x1.e542ba4020225p-62, 0x1.ea72b4afe3c2fp-120},
    {0x1.71b8ef6dcf572p-66, -0x1.d043ae40c4647p-120},
    {0x1.0ce396db7f853p-70, -0x1.aebcdbd20331cp-124},
    {0x1.761b41316381ap-75, -0x1.3423c7d91404fp-130},
    {0x1.f2cf01972f578p-80, -0x1.9ada5fcc1ab14p-135},
    {0x1.3f3ccdd165fa9p-84, -0x1.58ddadf344487p-139},
    {0x1.88e85fc6a4e5ap-89, -0x1.71c37ebd16540p-143},
    {0x1.d1ab1c2dccea3p-94, 0x1.054d0c78aea14p-149},
    {0x1.0a18a2635085dp-98, 0x1.b9e2e28e1aa54p-153}};

SDR_HD inline dd inv_fact(int n, bool neg) {
  return neg ? dd{-kInvFact[n][0], -kInvFact[n][1]} : dd{kInvFact[n][0], kInvFact[n][1]};
}

// sin r, cos r for |r| <= ~pi/4 (r a double-double), relative error < 2^-70:
// Horner in z = r^2 with the small high-order terms in plain double (sine
// k >= 4, cosine k >= 5: each below 2^-18 of the sum, so their roundings
// stay below 2^-71 of it) and the leading ones in double-double.  Enough to
// round to the nearest double wherever that decides the float: the sweep
// over every finite float confirms sin / cos, the atan2 samples the Newton
// step built on it (tests/test_libm_exact.py).
SDR_HD inline void dd_sincos_kernel(dd r, dd& s, dd& c) {
  const dd z = dd_mul(r, r);
  double ts = -kInvFact[27][0];  // k = 13: (-1)^13 / 27!
  for (int k = 12; k >= 4; --k) ts = __builtin_fma(ts, z.hi, (k & 1) ? -kInvFact[2 * k + 1][0] : kInvFact[2 * k + 1][0]);
  dd ps{ts, 0.0};
  for (int k = 3; k >= 0; --k) ps = dd_add(dd_mul(ps, z), inv_fact(2 * k + 1, k & 1));
  s = dd_mul(ps, r);
  double tc = kInvFact[28][0];  // k = 14
  for (int k = 13; k >= 5; --k) tc = __builtin_fma(tc, z.hi, (k & 1) ? -kInvFact[2 * k][0] : kInvFact[2 * k][0]);
  dd pc{tc, 0.0};
  for (int k = 4; k >= 0; --k) pc = dd_add(dd_mul(pc, z), inv_fact(2 * k, k & 1));
  c = pc;
}

// Payne-Hanek: a finite float ax >= 0.78 as (q + f) pi/2, |f| <= 1/2 quarter
// turns; returns q mod 4 and r = f pi/2 as a double-double.  ax = m 2^E (m
// the 24-bit significand); only the 192 bits of 2/pi from bit s = max(1, E-1)
// matter mod 4 (earlier bits give multiples of 4), and the ones after them
// change ax * 2/pi by < 2^-166 -- against a reduced argument never below
// ~2^-35 for fp32 inputs.
SDR_HD inline int reduce_pio2(float ax, dd& r) {
  const unsigned u = __builtin_bit_cast(unsigned, ax);
  const int E = (int)(u >> 23) - 150;
  const unsigned long long m = (u & 0x7fffffu) | 0x800000u;
  const int s = E >= 2 ? E - 1 : 1;
  const int F = s + 191 - E;  // ax * (2/pi)_window = P * 2^-F, F in [190, 216]
  const int w0 = (s - 1) >> 5, sh = (s - 1) & 31;
  unsigned P[7];
  unsigned long long carry = 0;
  for (int j = 5; j >= 0; --j) {
    const unsigned long long pair = ((unsigned long long)kTwoOverPiW[w0 + j] << 32) | kTwoOverPiW[w0 + j + 1];
    const unsigned win = (unsigned)(pair >> (32 - sh));
    const unsigned long long t = m * win + carry;
    P[j + 1] = (unsigned)t;
    carry = t >> 32;
  }
  P[0] = (unsigned)carry;
  // bits F-1 .. F+1 (F in [190, 216]) lie in the top two words: bit b of P
  // (b = 0 the least significant) is bit b - 160 of top = P[0]:P[1]
  const unsigned long long top = ((unsigned long long)P[0] << 32) | P[1];
  int q = (int)((top >> (F - 160)) & 3u);
  const bool neg = ((top >> (F - 161)) & 1u) != 0u;  // f >= 1/2: take q + 1 and f - 1
  // keep the F fraction bits; negate them (2^F - frac) when f >= 1/2
  for (int k = 0; k < 7; ++k) {
    const int lo = 32 * (6 - k);  // bit index of this word's least significant bit
    if (lo >= F)
      P[k] = 0u;
    else if (lo + 32 > F)
      P[k] &= (1u << (F - lo)) - 1u;
  }
  if (neg) {
    q += 1;
    unsigned long long c = 1;
    for (int k = 6; k >= 0; --k) {
      const unsigned long long t = (unsigned long long)(~P[k]) + c;
      P[k] = (unsigned)t;
      c = t >> 32;
    }
    for (int k = 0; k < 7; ++k) {  // mask again (the complement set the bits above F)
      const int lo = 32 * (6 - k);
      if (lo >= F)
        P[k] = 0u;
      else if (lo + 32 > F)
        P[k] &= (1u << (F - lo)) - 1u;
    }
  }
  // |f| as a double-double: the words are exact doubles of decreasing weight
  dd acc{0.0, 0.0};
  for (int k = 0; k < 7; ++k) {
    const double wv = __builtin_ldexp((double)P[k], 32 * (6 - k) - F);
    const dd t = two_sum(acc.hi, wv);
    acc = fast_two_sum(t.hi, t.lo + acc.lo);
  }
  r = dd_mul(acc, dd{pllfast::kP1, pllfast::kP2});
  if (neg) r = dd_neg(r);
  return q & 3;
}

// sin / cos of q pi/2 + r from the kernel values of r
SDR_HD inline void quadrant(int q, dd s, dd c, dd& S, dd& C) {
  switch (q & 3) {
    case 0: S = s; C = c; break;
    case 1: S = c; C = dd_neg(s); break;
    case 2: S = dd_neg(s); C = dd_neg(c); break;
    default: S = dd_neg(c); C = s; break;
  }
}

// the nearest double to a double-double, then the float (glibc's float when
// its double is the correctly rounded one)
SDR_HD inline double dd_round(dd a) { return fast_two_sum(a.hi, a.lo).hi; }

// No exception table is needed: the exhaustive sweep over every finite float
// (tests/libm_sweep.cpp, committed in tests/golden/libm_sincos.npz) found
// glibc's float equal to the correctly rounded double's float for sin and cos
// on every argument, so the double-double path alone reproduces it.  (If a
// glibc update ever broke that, tests/test_libm_exact.py fails and the
// arguments it prints would go into a lookup here.)

// a double result whose float rounding the midpoint certificate decides: the
// float range's rounding drops 29 bits (|d| >= 2^-126) or d is a float
SDR_HD inline bool normal_or_float(double d) {
  return __builtin_fabs(d) >= 0x1p-126 || (double)(float)d == d;
}

// whether the finite, non-float double d lies within w of its own ulps of a
// float rounding midpoint (subnormal floats included): the only doubles two
// libraries within an ulp of each other can round to different floats
SDR_HD inline bool near_float_mid(double d, double w) {
  const float f = (float)d;
  const double fd = (double)f;
  if (fd == d || !(__builtin_fabs(d) <= 0x1.fffffep127)) return false;
  // the float neighbour on d's side of f
  const unsigned b = __builtin_bit_cast(unsigned, f);
  const bool away = (d > fd) == (f > 0.0f);  // the neighbour is larger in magnitude
  float g;
  if (f == 0.0f)
    g = d > 0.0 ? 0x1p-149f : -0x1p-149f;
  else
    g = __builtin_bit_cast(float, away ? b + 1u : b - 1u);
  const double mid = 0.5 * (fd + (double)g);  // exact: 25 significant bits
  const double ulp = __builtin_fabs(d) * 0x1p-52;
  return __builtin_fabs(d - mid) <= w * ulp;
}

struct SinCos {
  float s, c;
};

// the double-double path of sincos_f: |x| finite (out of line: rare, and
// large; the short path is what callers inline)
SDR_HD inline __attribute__((noinline)) SinCos sincos_slow(float x) {
  const float ax = __builtin_fabsf(x);
  dd r;
  int q = 0;
  if (ax < 0.78f)
    r = dd{(double)ax, 0.0};
  else
    q = reduce_pio2(ax, r);
  dd s, c, S, C;
  dd_sincos_kernel(r, s, c);
  quadrant(q, s, c, S, C);
  const double sd = dd_round(S);
  return {(float)(x < 0.0f ? -sd : sd), (float)dd_round(C)};
}

// (float)sin((double)x), (float)cos((double)x) as glibc computes them
SDR_HD inline __attribute__((always_inline)) SinCos sincos_f(float x) {
  const float ax = __builtin_fabsf(x);
  if (!(ax <= 0x1.fffffep127f))  // Inf, NaN: the library's NaN
    return {(float)::sin((double)x), (float)::cos((double)x)};
  if (x == 0.0f) return {x, 1.0f};  // sin(+-0) = +-0, cos = 1
  if (ax < 0x1p26f) {
    unsigned score = ~0u;
    pllfast::Osc o;
    float s, c;
    pllfast::sincos_fast<ExactOps>(x, s, c, score, o);
    if (score >= pllfast::kCertifiedSc && normal_or_float(o.S) && normal_or_float(o.C)) return {s, c};
  } else {
    // beyond the fast reduction's checked range: Payne-Hanek, then the same
    // short kernels on the reduced argument's leading double
    dd r;
    const int q = reduce_pio2(ax, r);
    const double z = r.hi * r.hi, z2 = z * z;
    using pllfast::kS1, pllfast::kS2, pllfast::kS3, pllfast::kS4, pllfast::kS5;
    using pllfast::kC1, pllfast::kC2, pllfast::kC3, pllfast::kC4, pllfast::kC5;
    const double sp = __builtin_fma(z2, __builtin_fma(kS5, z2, __builtin_fma(kS4, z, kS3)), __builtin_fma(kS2, z, kS1));
    const double sr = __builtin_fma(r.hi * z, sp, r.hi + r.lo);
    const double cp = __builtin_fma(z2, __builtin_fma(kC5, z2, __builtin_fma(kC4, z, kC3)), __builtin_fma(kC2, z, kC1));
    const double cr = __builtin_fma(z2, cp, __builtin_fma(z, -0.5, 1.0));
    dd S, C;
    quadrant(q, dd{sr, 0.0}, dd{cr, 0.0}, S, C);
    const unsigned score = pllfast::umin(pllfast::mid_score_sc(sr), pllfast::mid_score_sc(cr));
    if (score >= pllfast::kCertifiedSc && normal_or_float(sr) && normal_or_float(cr))
      return {(float)(x < 0.0f ? -S.hi : S.hi), (float)C.hi};
  }
  return sincos_slow(x);
}
SDR_HD inline float cos_f(float x) { return sincos_f(x).c; }
SDR_HD inline float sin_f(float x) { return sincos_f(x).s; }

// the double-double path of atan2_f: x, y finite and nonzero; t0 the fast
// double result (relative error < 2^-46); returns the nearest double to the
// exact value (the tests read it to find the near-midpoint cases)
SDR_HD inline __attribute__((noinline)) double atan2_slow_d(float y, float x, double t0) {
  const double X = (double)x, Y = (double)y;
  // sin / cos of t0 (|t0| <= pi) in double-double: t0 - k pi/2 with k in
  // -2..2 is exact in its first step (Sterbenz), then the two tails
  const double kd = __builtin_rint(t0 * pllfast::kTwoOverPi);
  const double t1 = __builtin_fma(-kd, pllfast::kP1, t0);
  dd r = two_sum(t1, -kd * pllfast::kP2);
  r = dd_add(r, dd{-kd * kP3, 0.0});
  dd s, c, S, C;
  dd_sincos_kernel(r, s, c);
  quadrant((int)kd, s, c, S, C);
  // Newton on g(t) = x sin t - y cos t (g'' = -g vanishes at the root: the
  // step's own error is cubic in t0's)
  const dd num = dd_add(dd_mul_d(S, X), dd_neg(dd_mul_d(C, Y)));
  const double den = __builtin_fma(X, C.hi, Y * S.hi);
  const double delta = -(num.hi / den);
  return two_sum(t0, delta).hi;
}
SDR_HD inline float atan2_slow(float y, float x, double t0) { return (float)atan2_slow_d(y, x, t0); }

// (float)atan2((double)y, (double)x) as glibc computes it
SDR_HD inline __attribute__((always_inline)) float atan2_f(float y, float x) {
  const float ax = __builtin_fabsf(x), ay = __builtin_fabsf(y);
  if (!(ax <= 0x1.fffffep127f && ay <= 0x1.fffffep127f) || x == 0.0f || y == 0.0f)
    return (float)::atan2((double)y, (double)x);  // the C standard's exact values, or NaN
  unsigned score = ~0u;
  const double a = pllfast::atan2_abs<ExactOps>(y, x, score);
  if (score >= pllfast::kCertified && normal_or_float(a)) return __builtin_copysignf((float)a, y);
  return atan2_slow(y, x, __builtin_copysign(a, (double)y));
}

}  // namespace libmx
}  // namespace sdr
