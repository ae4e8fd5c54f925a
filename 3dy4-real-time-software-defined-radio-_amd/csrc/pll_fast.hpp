// pll_fast.hpp -- short-chain atan2 / sincos for the fmPLL recurrence, with a
// certificate that the float the reference stores is the one computed.
//
// The reference evaluates errorD = atan2(errorQ, errorI) and
// feedbackI/Q = cos/sin(trigArg) in double on float arguments and rounds each
// result to float (src/filter.cpp:199, :216-217).  Only those floats feed the
// recurrence, so any double approximation d of the exact value f gives the
// same float as long as no float rounding boundary (a midpoint between two
// adjacent floats) lies between d and f, nor between f and the library's
// double result.  These routines keep the library's algorithms (OCML's
// atan2/sincos polynomial coefficients) with fewer instructions and shorter
// dependency chains -- one wave per SIMD issues every instruction of the
// recurrence on its own, so the count is what the time is:
//   - atan2: v/u by one reciprocal and a second-order correction instead of
//     the IEEE division sequence; a degree-15 polynomial in t^2 (error
//     < 2^-46.8) by Estrin's scheme (depth 5) instead of OCML's degree 19 by
//     Horner's (depth 20);
//   - sincos: a two-term FMA Cody-Waite reduction of the fp32 argument
//     (exact first step; a third term changes no result, see kP1 below)
//     instead of the double-double reduction; sine and
//     cosine kernels one term shorter than fdlibm's, by Estrin's scheme;
//     quadrant signs applied before the rounding to float.
// Each double result is within ~2^-46.3 (relative) of the exact value: the
// atan polynomial's fit error or the rotation's reciprocal plus a few ulps of
// rounding (tests/pll_cert.cpp measures 2^-46.4 / 2^-46.7 / 2^-51.5 against
// glibc for atan2_abs / atan2_rot / sincos).
//
// Certificate.  mid_score() measures a result's distance to the nearest float
// midpoint; the caller keeps the running unsigned minimum over a chunk, which
// is certified while it stays >= kCertified, i.e. every result lies more than
// kCertW = 1,024 double ulps (>= 2^-43 relative, 10x the error above) from a
// midpoint -- so it, the exact value and the library's result (within
// ~2^-46.3 and 1-2 ulps of the exact value) round to one float.  (The round-2
// window of 4,096 ulps re-ran 4x as many chunks: 2.3 % of 64-lane chunks, a
// 5 % slower recurrence.)  The remaining cases are guarded by chunk_ok on the
// state before and after each chunk (finite and in range, so |trigArg| <
// 2^26, trigArg != -0, the feedback floats are 0 or >= 2^-60, and errorD is
// never subnormal), and by input_ok on the chunk's samples (0 or 2^-60 <=
// |v| <= FLT_MAX, so the phase detector's products are normal or exact
// zeros); a NaN from x = y = 0 reaches phaseEst and fails the closing check.  Within those guards a certified
// step's floats are the reference's; an uncertified chunk is re-run with the
// library routines.  DESIGN.md section 4.7 has the argument.
//
// Host/device: SDR_HD is __host__ __device__ under hipcc; the CPU test of the
// certificate (tests/pll_cert.cpp) defines it empty.  Ops supplies fma(a, b, c)
// and rcp(u) (relative error <= 2^-20): the kernel's are a VOP3 v_fma_f64
// (one instruction; the compiler's VOP2 fmac form costs a v_mov_b64 per
// polynomial pair) and v_rcp_f64; the CPU test's are std fma and a
// deliberately coarse reciprocal.
#pragma once

#ifndef SDR_HD
#define SDR_HD __host__ __device__
#endif

namespace sdr {
namespace pllfast {
// atan(t) = t + t*z*P(z), z = t^2, t in [0, 1], P of degree 15: a weighted
// least-squares fit (scripts/fit_atan.py) with relative error < 2^-46.8 on
// [0, 1] -- 4 terms fewer than OCML's degree 19 (< 2^-54), well inside the
// certificate's 2^-40 margin.  Coefficients c0..c15.
constexpr double kAtanC[16] = {
    -0x1.5555555548634p-2, 0x1.9999998dcb71cp-3, -0x1.2492473aa1d47p-3, 0x1.c71c204d48085p-4,
    -0x1.7459013f32a55p-4, 0x1.3af102625a079p-4, -0x1.1042b16ee39eep-4, 0x1.dae1c88757e5cp-5,
    -0x1.9852ad76ae65cp-5, 0x1.4cd7d6822d40bp-5, -0x1.e72bb0e3e1c37p-6, 0x1.2c694cfa120d0p-6,
    -0x1.231ab51098098p-7, 0x1.97372e16c0db6p-9, -0x1.68e74a9b5111ap-11, 0x1.2ddb1bd53fd3fp-14};
// Sine / cosine kernels on [-pi/4, pi/4], one term shorter than OCML's
// (fdlibm's, error 2^-58): weighted least-squares fits (scripts/fit_sincos.py)
// with relative error < 2^-47.4 (sine) and 2^-53.1 (cosine), inside the
// certificate's margin like the atan fit.
//   sin r = r + r z (S1 + S2 z + ... + S5 z^4),  cos r = 1 - z/2 + z^2 (C1 + ... + C5 z^4)
constexpr double kS1 = -0x1.55555555520b6p-3, kS2 = 0x1.1111110c7394ep-7, kS3 = -0x1.a019f92438b3ep-13,
                 kS4 = 0x1.71d763ba62162p-19, kS5 = -0x1.a95eb720c4661p-26;
constexpr double kC1 = 0x1.5555555552c07p-5, kC2 = -0x1.6c16c166fb086p-10, kC3 = 0x1.a019fa3cf03c1p-16,
                 kC4 = -0x1.27dffdd9599aap-22, kC5 = 0x1.1bbaabead14f7p-29;
// pi/2 = P1 + P2 (+ -1.5e-33); 2/pi; pi.  A third Cody-Waite term is not
// needed: over every float in [pi/4, 2^26) the reduced argument is at least
// 2^-27.83 (exhaustive search, at x = 0x1.f9cbe2p+7), so |kd| * 1.5e-33 <=
// 2^-84 changes none of them (scripts/min_reduced_arg.c).
constexpr double kP1 = 0x1.921fb54442d18p+0, kP2 = 0x1.1a62633145c07p-54;
constexpr double kTwoOverPi = 0x1.45f306dc9c883p-1;
constexpr double kPi = 0x1.921fb54442d18p+1;

// mid_score(d) = ((lo29 - (2^28 - W)) mod 2^29) << 3 for the 29 mantissa
// bits double -> float drops: < kCertified <=> lo29 within [-W, W) of the
// midpoint 2^28 (W = kCertW).  One shift-add per result.
#ifndef SDR_PLL_CERT_W
#define SDR_PLL_CERT_W 1024
#endif
constexpr unsigned kCertW = SDR_PLL_CERT_W;  // the window's half width in double ulps (a power of 2)
constexpr unsigned kCertified = (2u * kCertW) << 3;
constexpr unsigned kMidBias = 0u - (((1u << 28) - kCertW) << 3);  // -((2^28 - W) << 3) mod 2^32

SDR_HD inline unsigned lo_bits(double d) { return (unsigned)__builtin_bit_cast(unsigned long long, d); }
SDR_HD inline unsigned umin(unsigned a, unsigned b) { return a < b ? a : b; }
SDR_HD inline unsigned mid_score(double d) { return (lo_bits(d) << 3) + kMidBias; }
// The sine / cosine results keep their own, narrower window (round 6): their
// kernels are accurate to ~2^-51.5 (about 1.4 double ulps, tests/pll_cert.cpp)
// and, with a one-argument function, the window is PROVED rather than
// sampled -- tests/libm_sweep.cpp runs sincos_fast on every finite float and
// every result certified at kCertWSc ulps equals glibc's float.  Callers keep
// a separate running minimum for it, compared against kCertifiedSc; a chunk
// of the PLL then re-runs ~3x less often (the atan2 window stays 1,024 ulps).
#ifndef SDR_PLL_CERT_W_SC
#define SDR_PLL_CERT_W_SC 32
#endif
constexpr unsigned kCertWSc = SDR_PLL_CERT_W_SC;
constexpr unsigned kCertifiedSc = (2u * kCertWSc) << 3;
constexpr unsigned kMidBiasSc = 0u - (((1u << 28) - kCertWSc) << 3);
SDR_HD inline unsigned mid_score_sc(double d) { return (lo_bits(d) << 3) + kMidBiasSc; }

// The oscillator's argument over the next chunk's 8 steps stays inside the
// reduction's exhaustively checked range, |trigArg| < 2^26:
//   trigArg = step * trigOffset' + phaseEst',  trigOffset' <= trigOffset + 8,
//   |phaseEst'| <= |phaseEst| + 8 |integrator| + 138  (|Kp|, |Ki| <= 1, |errorD| <= pi),
// bounded here in fp32 with stepf >= |step| (step_bound) and margins well
// above the few roundings of the bound itself (a NaN or Inf anywhere fails
// it).  This bound is all |phaseEst| needs: past 2^24 samples the loop's
// phase keeps growing in phaseEst, and the fast step follows it up to
// |trigArg| < 2^26.  trigOffset may sit AT 2^24:
// there the reference's `trigOffset++` stops advancing (fp32), which the
// fast step computes the same way -- a receiver reaches it after 2^24
// samples (70 s at 240 kHz) and stays there.
SDR_HD inline bool arg_ok(float integrator, float phaseEst, float trigOffset, float stepf) {
  const float ph = __builtin_fmaf(__builtin_fabsf(integrator), 16.0f, __builtin_fabsf(phaseEst) + 256.0f);
  return __builtin_fmaf(stepf, trigOffset + 8.0f, ph) < 0x1p26f;
}
// |step| rounded up to fp32 with a relative margin (once per launch)
SDR_HD inline float step_bound(double step) { return (float)(__builtin_fabs(step) * (1.0 + 0x1p-20)); }

// Chunk guard: the state at a chunk's start keeps every step of the next 8
// inside the certified domain (|Kp|, |Ki| <= 1 is the caller's launch-time
// condition).  Written with & so it is straight-line code.
SDR_HD inline bool chunk_ok(float fbI, float fbQ, float integrator, float phaseEst, float trigOffset, float stepf) {
  const float aI = __builtin_fabsf(fbI), aQ = __builtin_fabsf(fbQ);
  return (int)(trigOffset >= 0.0f) & (int)(trigOffset <= 0x1p24f) &
         (int)(__builtin_fabsf(integrator) < 0x1p20f) & (int)arg_ok(integrator, phaseEst, trigOffset, stepf) &
         (int)(aI <= 1.0f) & (int)(aQ <= 1.0f) & ((int)(aI >= 0x1p-60f) | (int)(fbI == 0.0f)) &
         ((int)(aQ >= 0x1p-60f) | (int)(fbQ == 0.0f));
}

// Chunk guard on the inputs: every sample v of a certified chunk is 0 or
// 2^-60 <= |v| <= FLT_MAX.  With chunk_ok's feedback floats (0 or >= 2^-60)
// the phase detector's products v * fbI and v * fbQ are then normal floats
// (>= 2^-120, each within 2^-24 of the exact product) or exact zeros, which
// atan2_rot's error bound assumes; a tiny or subnormal v can round a product
// to a subnormal or to 0 (v = 2^-149 once gave a residual of 3e-3 rad), and
// a non-finite v has no product at all.  A chunk with any other input is
// re-run with the library routines.
SDR_HD inline bool input_ok(float v) {
  const float a = __builtin_fabsf(v);
  return (int)(v == 0.0f) | ((int)(a >= 0x1p-60f) & (int)(a <= 0x1.fffffep127f));
}

// A float that is NaN, Inf or subnormal.  In chunk_ok's domain errorD is
// never subnormal (|errorQ / errorI| >= 2^-83 unless errorQ = 0, then the
// result is exact) and x = y = 0 or a non-finite input gives NaN, which
// reaches phaseEst and fails the chunk's closing chunk_ok; the CPU test
// checks these claims with this predicate.
SDR_HD inline bool float_special(float f) {
  const unsigned e = __builtin_bit_cast(unsigned, f) >> 23 & 0xffu;
  return (e == 0xffu) | ((e == 0u) & (__builtin_bit_cast(unsigned, f) << 1 != 0u));
}

// (float)atan2(y, x) for fp32 y, x: OCML's algorithm with fewer double
// operations; folds the double result's midpoint distance into score.  A
// double op is what the recurrence pays for (a single wave issues each one
// on its own), so the float parts stay float: |x|, |y|, their max / min and
// the quadrant tests are exact in fp32.
template <class Ops>
SDR_HD inline double atan2_abs(float y, float x, unsigned& score);
template <class Ops>
SDR_HD inline float atan2_fast(float y, float x, unsigned& score) {
  return __builtin_copysignf((float)atan2_abs<Ops>(y, x, score), y);
}
// |atan2(y, x)| in double (the CPU test reads it to bound the error)
template <class Ops>
SDR_HD inline double atan2_abs(float y, float x, unsigned& score) {
  const float ax = __builtin_fabsf(x), ay = __builtin_fabsf(y);
  const double u = (double)__builtin_fmaxf(ax, ay), v = (double)__builtin_fminf(ax, ay);
  // v / u: r0 = (1 - e) / u exactly with |e| <= 2^-24.37 (v_rcp_f64, measured),
  // so t = q0 (1 + e) = v/u (1 - e^2): relative error <= 2^-48.7 + 2 ulp
  const double r0 = Ops::rcp(u);
  const double q0 = v * r0;
  const double e = Ops::fma(-u, r0, 1.0);
  const double t = Ops::fma(q0, e, q0);
  // P(z): the pairs c_2i + c_2i+1 z, then Horner in z^2
  const double z = t * t;
  const double z2 = z * z;
  double p[8];
#pragma unroll
  for (int i = 0; i < 8; ++i) p[i] = Ops::fma(kAtanC[2 * i + 1], z, kAtanC[2 * i]);
  double P = p[7];
#pragma unroll
  for (int i = 6; i >= 0; --i) P = Ops::fma(P, z2, p[i]);
  // OCML's fixups (|y| > |x|: pi/2 - a; x negative (sign bit): pi - that) on
  // a = t + t z P, folded into C + s (t + t z P) with s = +-1:
  //   (swap, neg) = (0,0): 0 + a, (1,0): pi/2 - a, (0,1): pi - a, (1,1): pi/2 + a
  const bool swap = ay > ax, neg = __builtin_signbit(x);
  const double C = swap ? kP1 : (neg ? kPi : 0.0);
  const unsigned long long sflip = (unsigned long long)(swap != neg) << 63;  // s = -1
  const double st = __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, t) ^ sflip);
  const double stz = __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, t * z) ^ sflip);
  const double res = Ops::fma(stz, P, Ops::fma(1.0, st, C));  // C + s t is one rounding
  score = umin(score, mid_score(res));
  return res;
}

// The oscillator a fast step hands the next step's phase detector: the
// reduced argument r (trigArg = r + q pi/2 + ~2^-84 |q|) and the double
// sine S and cosine C of trigArg (the quadrant applied to the sine and cosine kernels
// of r), from which atan2_rot rotates.
struct Osc {
  double r, S, C;
  int q;
};

// (float)sin(x), (float)cos(x) for x an fp32 value in chunk_ok's domain
// (|x| < 2^26, x != -0); folds both double results into score -- the
// sine / cosine running minimum, certified at >= kCertifiedSc -- and leaves
// the oscillator in o.
template <class Ops>
SDR_HD inline void sincos_fast(float xf, float& sf, float& cf, unsigned& score, Osc& o) {
  const double x = (double)xf;
  const double kd = __builtin_rint(x * kTwoOverPi);
  // x and kd*P1 are multiples of 2^-52 and |x - kd*P1| < 2, so r1 is exact
  const double r1 = Ops::fma(-kd, kP1, x);
  const double r = Ops::fma(-kd, kP2, r1);
  const int q = (int)kd;
  const double z = r * r;
  const double z2 = z * z;
  // sin r = r + r z S(z), S = (S1 + S2 z) + z^2 ((S3 + S4 z) + z^2 S5)  (Estrin)
  const double sp = Ops::fma(z2, Ops::fma(kS5, z2, Ops::fma(kS4, z, kS3)), Ops::fma(kS2, z, kS1));
  const double sr = Ops::fma(r * z, sp, r);
  // cos r = (1 - z/2) + z^2 C(z), C = (C1 + C2 z) + z^2 ((C3 + C4 z) + z^2 C5);
  // 1 - z/2 in one rounding (cos r >= 0.7: 1 ulp, no compensation needed)
  const double cp = Ops::fma(z2, Ops::fma(kC5, z2, Ops::fma(kC4, z, kC3)), Ops::fma(kC2, z, kC1));
  const double cr = Ops::fma(z2, cp, Ops::fma(z, -0.5, 1.0));
  score = umin(score, umin(mid_score_sc(sr), mid_score_sc(cr)));
  // quadrant q mod 4: (sin, cos) = (s, c), (c, -s), (-s, -c), (-c, s), applied
  // to the doubles (kept for atan2_rot) and then rounded (rounding commutes
  // with negation, so the floats are those of the rounded kernels)
  const double sw = (q & 1) ? cr : sr;
  const double cw = (q & 1) ? sr : cr;
  o.S = __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, sw) ^
                                       ((unsigned long long)((unsigned)q << 30 & 0x80000000u) << 32));
  o.C = __builtin_bit_cast(double, __builtin_bit_cast(unsigned long long, cw) ^
                                       ((unsigned long long)((unsigned)(q + 1) << 30 & 0x80000000u) << 32));
  o.r = r;
  o.q = q;
  sf = (float)o.S;
  cf = (float)o.C;
}
template <class Ops>
SDR_HD inline void sincos_fast(float xf, float& sf, float& cf, unsigned& score) {
  Osc o;
  sincos_fast<Ops>(xf, sf, cf, score, o);
}

// (float)atan2(y, x) for the phase detector of the step after the one that
// left oscillator o: y = v * -fbQ, x = v' * fbI with fbI, fbQ the float
// cos / sin of o's angle theta (v' = v for v != 0).  Instead of an atan
// polynomial, (x, y) is rotated back by the known angle
//   beta = -theta (+ pi for v < 0) = k pi/2 - r,  k in {-2, ..., 2}, beta in (-pi, pi]
// (cos, sin of beta are +-(C, -S) of o): the residual angle is
//   delta = atan((y C + x S) / (x C - y S)),  C, S = cos, sin theta,
// which only the float roundings of fbI, fbQ, x and y make nonzero:
// |delta| <= 2^-22 |sin theta cos theta| <= 2^-22 |beta|, so atan(t) = t
// (t^3/3 is < 2^-66 |beta|) and v_rcp_f64's 2^-24.4 costs < 2^-46 |beta|;
// the numerator's one rounding costs 2^-53 |S C|.  So the result
// beta + delta is within ~2^-45 |result| of the exact atan2 -- as tight as
// the polynomial's -- in ~10 double operations instead of ~27.  y = 0 (v = 0,
// where x = fbI is a different geometry, or fbQ = 0) takes atan2's exact
// values on the axis, +-0 or +-pi (x != 0 here: fbI is never 0).  Not
// certified (score 0, the chunk re-runs): a result that rounds to +-pi_f
// (beta + delta may have crossed +-pi, where atan2 wraps).
template <class Ops>
SDR_HD inline float atan2_rot(float y, float x, float v, const Osc& o, unsigned& score, double& res);
template <class Ops>
SDR_HD inline float atan2_rot(float y, float x, float v, const Osc& o, unsigned& score) {
  double res;
  return atan2_rot<Ops>(y, x, v, o, score, res);
}
// res: the double result (the CPU test reads it to bound the error)
template <class Ops>
SDR_HD inline float atan2_rot(float y, float x, float v, const Osc& o, unsigned& score, double& res) {
  const int q4 = o.q & 3;
  const double S = o.S, C = o.C;
  const double X = (double)x, Y = (double)y;
  const double num = Ops::fma(Y, C, X * S);
  const double den = Ops::fma(X, C, -(Y * S));
  const double rc = Ops::rcp(den);
  // k = (2 [v < 0] - q4) mod 4 as a representative in (-pi, pi]
  int k = ((v < 0.0f ? 2 : 0) - q4) & 3;
  k = k == 3 ? -1 : k;
  k = (k == 2 && __builtin_signbit(o.r)) ? -2 : k;
  const double kd = (double)k;
  // beta + delta = k P1 + (delta - r): k P2 (<= 2^-52.5 of the result when k != 0,
  // absent when k = 0) is dropped; two roundings of at most 2^-53 each
  res = Ops::fma(kd, kP1, Ops::fma(num, rc, -o.r));
  const float f = (float)res;
  const bool axis = y == 0.0f;
  // atan2(+-0, x) = +-0 for x > 0, +-pi (rounded: pi_f) for x < 0
  const float fa = x > 0.0f ? y : __builtin_copysignf(0x1.921fb6p+1f, y);
  // branch-free: umin(score, mid) on the rotation's result, 0 if it rounds to
  // +-pi_f, unchanged on the axis
  const unsigned in_pi = 0u - (unsigned)(__builtin_fabsf(f) < 0x1.921fb6p+1f);
  const unsigned cand = umin(score, mid_score(res)) & in_pi;
  score = axis ? score : cand;
  return axis ? fa : f;
}

// The closing check of a chunk that ran the fast path from a chunk_ok state:
// phaseEst, integrator and trigOffset finite and small enough for the next
// chunk (trigOffset only grows, up to 2^24; the feedback floats are sin /
// cos results of arguments in the domain, so 0 or >= 2^-54 -- see
// chunk_ok).  A NaN anywhere in the chunk reaches phaseEst, and fails here.
SDR_HD inline bool chunk_end_ok(float integrator, float phaseEst, float trigOffset, float stepf) {
  return (int)(__builtin_fabsf(integrator) < 0x1p20f) & (int)(trigOffset <= 0x1p24f) &
         (int)arg_ok(integrator, phaseEst, trigOffset, stepf);
}

}  // namespace pllfast
}  // namespace sdr
