// CPU check of the PLL's short-chain transcendentals (csrc/pll_fast.hpp):
// wherever they certify a result, its float rounding must equal the
// reference's, (float)atan2 / (float)sin / (float)cos of glibc's double
// routines (src/filter.cpp:199, :216-217).  Built and run by
// tests/test_pll_cert.py (g++, no GPU).  The device reciprocal
// (v_rcp_f64, measured max error 2^-24.37: tools/ubench_rcp.hip) is modelled
// by 1/u with its low 28 mantissa bits cleared (error up to 2^-24), so the
// division's correction term is exercised at least as hard as on the device.
//
// usage: pll_cert <samples> <seed>; prints one JSON line of counts.
#define SDR_HD
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <random>

#include "pll_fast.hpp"

using namespace sdr::pllfast;

struct HostOps {
  static double fma(double a, double b, double c) { return std::fma(a, b, c); }
  static double rcp(double u) {  // 1/u with its low 28 mantissa bits cleared (error <= 2^-24)
    double r = 1.0 / u;
    uint64_t b;
    std::memcpy(&b, &r, 8);
    b &= ~((1ull << 28) - 1);
    std::memcpy(&r, &b, 8);
    return r;
  }
};

static uint32_t fbits(float f) {
  uint32_t b;
  std::memcpy(&b, &f, 4);
  return b;
}

struct Counts {
  long long n = 0, certified = 0, mismatch = 0, special = 0;
  double max_rel = 0.0;  // max |fast - glibc| / |glibc| over certified results
};
static void track(Counts& c, double fast, double ref) {
  if (ref != 0.0 && std::isfinite(ref)) c.max_rel = std::fmax(c.max_rel, std::fabs(fast - ref) / std::fabs(ref));
}

// atan2 on the kernel's domain: y = v * -fbQ, x = v' * fbI with |v| in
// {0} U [2^-60, 2^60] and feedback floats in {0} U [2^-60, 1] (chunk_ok)
static void check_atan2(float y, float x, Counts& c) {
  unsigned score = ~0u;
  const double a = std::copysign(atan2_abs<HostOps>(y, x, score), (double)y);
  const float eD = std::copysign((float)std::fabs(a), y);
  const double refd = std::atan2((double)y, (double)x);
  const float ref = (float)refd;
  ++c.n;
  // the kernel never sees a subnormal errorD in this domain; NaN only from
  // x = y = 0 (caught there by the closing chunk_ok): counted if it shows
  if (float_special(eD)) {
    if (!(x == 0.0f && y == 0.0f)) ++c.special;
    return;
  }
  if (score < kCertified) return;
  ++c.certified;
  track(c, a, refd);
  if (fbits(eD) != fbits(ref)) {
    if (c.mismatch < 5) std::fprintf(stderr, "atan2 mismatch y=%a x=%a fast=%a ref=%a\n", y, x, a, (double)ref);
    ++c.mismatch;
  }
}

// sincos on the kernel's domain: x = +0 or 2^-60 <= |x| < 2^26
static void check_sincos(float x, Counts& c) {
  unsigned score = ~0u;
  float s, co;
  Osc o;
  sincos_fast<HostOps>(x, s, co, score, o);
  const float rs = (float)std::sin((double)x), rc = (float)std::cos((double)x);
  ++c.n;
  if (score < kCertifiedSc) return;
  ++c.certified;
  track(c, o.S, std::sin((double)x));
  track(c, o.C, std::cos((double)x));
  if (fbits(s) != fbits(rs) || fbits(co) != fbits(rc)) {
    if (c.mismatch < 5) std::fprintf(stderr, "sincos mismatch x=%a s=%a/%a c=%a/%a\n", x, s, rs, co, rc);
    ++c.mismatch;
  }
}

// atan2_rot: the phase detector of the step after sincos_fast(arg) -- y =
// v * -fbQ, x = v' * fbI from that step's floats -- against glibc's atan2 of
// the same floats (the kernel's steps 2..8 of a chunk)
static void check_atan2_rot(float arg, float v, Counts& c) {
  unsigned sc = ~0u;
  float fbQ, fbI;
  Osc o;
  sincos_fast<HostOps>(arg, fbQ, fbI, sc, o);
  const float eI = (v == 0.0f ? 1.0f : v) * fbI;
  const float eQ = v * (-1.0f * fbQ);
  unsigned score = ~0u;
  double res;
  const float eD = atan2_rot<HostOps>(eQ, eI, v, o, score, res);
  const double refd = std::atan2((double)eQ, (double)eI);
  const float ref = (float)refd;
  ++c.n;
  if (float_special(eD)) ++c.special;
  if (score < kCertified) return;
  ++c.certified;
  if (eQ != 0.0f) track(c, res, refd);
  if (fbits(eD) != fbits(ref)) {
    if (c.mismatch < 5)
      std::fprintf(stderr, "atan2_rot mismatch arg=%a v=%a fast=%a ref=%a\n", arg, v, (double)eD, (double)ref);
    ++c.mismatch;
  }
}

// src/filter.cpp:174-228's recurrence, the reference's way and the kernel's
// way (chunks of 8 fast steps, a chunk re-run with the library routines when
// any step was not certified; here one "wave" = one stream).  States and
// recorded arguments must be bit-equal.
struct Pll {
  float fbI = 1, fbQ = 0, integ = 0, phase = 0, trig = 0;
};

static long long pll_compare(const float* in, long long n, float trig0, long long* reruns, float phase0 = 0.0f) {
  const float Kp = 0.01f * 2.666f, Ki = 0.01f * 0.01f * 3.555f;
  const double step = 2.0 * 3.14159265358979323846 * (double)(19e3f / 240e3f);
  Pll r, f;
  r.trig = f.trig = trig0;
  r.phase = f.phase = phase0;
  long long bad_args = 0;
  const float stepf = step_bound(step);
  bool start_ok = chunk_ok(f.fbI, f.fbQ, f.integ, f.phase, f.trig, stepf);
  Osc osc{};  // the kernel's: every step but the first rotates back from the previous step's oscillator
  auto lib_step = [&](Pll& p, float v) {
    const float eI = (v == 0.0f ? 1.0f : v) * p.fbI;
    const float eQ = v * (-1.0f * p.fbQ);
    const float eD = (float)std::atan2((double)eQ, (double)eI);
    p.integ = p.integ + Ki * eD;
    p.phase = p.phase + (Kp * eD + p.integ);
    p.trig = p.trig + 1.0f;
    const float arg = (float)(step * (double)p.trig + (double)p.phase);
    p.fbI = (float)std::cos((double)arg);
    p.fbQ = (float)std::sin((double)arg);
    return arg;
  };
  for (long long k0 = 0; k0 < n; k0 += 8) {
    const long long m = n - k0 < 8 ? n - k0 : 8;
    float ra[8], fa[8];
    for (long long j = 0; j < m; ++j) ra[j] = lib_step(r, in[k0 + j]);
    const Pll saved = f;
    bool in_ok = true;
    for (long long j = 0; j < m; ++j) in_ok = in_ok && input_ok(in[k0 + j]);
    unsigned score = start_ok && in_ok ? ~0u : 0u, score_sc = score;
    for (long long j = 0; j < m; ++j) {
      const float v = in[k0 + j];
      const float eI = (v == 0.0f ? 1.0f : v) * f.fbI;
      const float eQ = v * (-1.0f * f.fbQ);
      const float eD =
          (j > 0 || k0 > 0) ? atan2_rot<HostOps>(eQ, eI, v, osc, score) : atan2_fast<HostOps>(eQ, eI, score);
      f.integ = f.integ + Ki * eD;
      f.phase = f.phase + (Kp * eD + f.integ);
      f.trig = f.trig + 1.0f;
      fa[j] = (float)(step * (double)f.trig + (double)f.phase);
      sincos_fast<HostOps>(fa[j], f.fbQ, f.fbI, score_sc, osc);
    }
    start_ok = chunk_end_ok(f.integ, f.phase, f.trig, stepf);
    const bool bad = score < kCertified || score_sc < kCertifiedSc || !start_ok;
    if (bad) {
      ++*reruns;
      f = saved;
      for (long long j = 0; j < m; ++j) fa[j] = lib_step(f, in[k0 + j]);
      start_ok = chunk_ok(f.fbI, f.fbQ, f.integ, f.phase, f.trig, stepf);
      float tq, ti;
      unsigned unused = 0u;
      sincos_fast<HostOps>(fa[m - 1], tq, ti, unused, osc);  // the kernel's refresh after a re-run
    }
    for (long long j = 0; j < m; ++j) bad_args += fbits(ra[j]) != fbits(fa[j]);
  }
  const bool st = fbits(r.fbI) == fbits(f.fbI) && fbits(r.fbQ) == fbits(f.fbQ) && fbits(r.integ) == fbits(f.integ) &&
                  fbits(r.phase) == fbits(f.phase) && fbits(r.trig) == fbits(f.trig);
  return bad_args + (st ? 0 : 1);
}

int main(int argc, char** argv) {
  const long long N = argc > 1 ? std::atoll(argv[1]) : 1000000;
  const unsigned seed = argc > 2 ? (unsigned)std::atoi(argv[2]) : 1;
  std::mt19937_64 g(seed);
  std::uniform_real_distribution<double> U(-1.0, 1.0), E(-60.0, 60.0);
  std::bernoulli_distribution coin(0.5), rare(0.001);
  Counts at, sc, scw, ar;
  auto logu = [&](double lo, double hi) {
    std::uniform_real_distribution<double> L(lo, hi);
    return (coin(g) ? -1.0 : 1.0) * std::exp2(L(g));
  };
  for (long long i = 0; i < N; ++i) {
    // atan2: PLL-like products (|.| <= 0.3), and the kernel's whole domain:
    // v in {0} U [2^-60, 2^60] times feedback floats in {0} U [2^-60, 1]
    float y, x;
    if (i % 2 == 0) {
      y = (float)(0.3 * U(g));
      x = (float)(0.3 * U(g));
    } else {
      const float v = rare(g) ? 0.0f : (float)logu(-60, 60);
      const float fq = rare(g) ? 0.0f : (float)logu(-60, 0), fi = rare(g) ? 0.0f : (float)logu(-60, 0);
      y = v * (-1.0f * fq);
      x = (v == 0.0f ? 1.0f : v) * fi;
    }
    check_atan2(y, x, at);
    // sincos: small and PLL-sized arguments, and magnitudes 2^-60 .. 2^26
    float a;
    switch (i % 3) {
      case 0: a = (float)(8.0 * U(g)); break;
      case 1: a = (float)(0.4974 * (double)(i % 20000000) + U(g)); break;
      default: a = (float)logu(-60, 25.99); break;
    }
    if (rare(g)) a = 0.0f;
    check_sincos(a, sc);
    // the rotation: pilot-sized and whole-domain v (and exact zeros)
    const float v = rare(g) ? 0.0f : (i % 2 ? (float)(0.3 * U(g)) : (float)logu(-60, 60));
    check_atan2_rot(a, v, ar);
  }
  // the floats nearest to multiples of pi/2 (and their neighbours): the
  // reduction's hardest arguments (tiny reduced values)
  const long double halfpi = 1.5707963267948966192313216916397514L;
  for (long long k = 1; k <= N / 8 && k < (1ll << 26); ++k) {
    const long long kk = (long long)((double)k * 40000000.0 / (double)(N / 8 + 1)) + 1;
    const float c = (float)(kk * halfpi);
    check_sincos(c, scw);
    check_sincos(std::nextafter(c, 1e30f), scw);
    check_sincos(std::nextafter(c, -1e30f), scw);
    // tiny reduced arguments: beta near 0 or +-pi (the rotation's hardest)
    const float v = (float)(0.3 * U(g));
    check_atan2_rot(c, v, ar);
    check_atan2_rot(std::nextafter(c, 1e30f), -v, ar);
  }
  // whole recurrences: noisy 19 kHz pilots, exact zeros, a large trigOffset start
  long long pll_bad = 0, reruns = 0, steps = 0;
  std::normal_distribution<double> G(0.0, 0.01);
  const long long L = 20000;
  float* pil = (float*)std::malloc(sizeof(float) * L);
  for (int s = 0; s < 24; ++s) {
    const double amp = 0.01 + 0.29 * (U(g) + 1) / 2, f = 19e3 + 40 * U(g), ph = 3.2 * U(g);
    for (long long k = 0; k < L; ++k)
      pil[k] = (float)(amp * std::cos(2 * M_PI * f / 240e3 * (double)k + ph) + G(g));
    for (long long k = 0; k < L; k += 997) pil[k] = 0.0f;
    // 16,770,000: trigOffset reaches 2^24 (where fp32 ++ stops) mid-run
    const float trig0 = s % 4 == 0 ? 0.0f : (s % 4 == 1 ? 3.0e6f : (s % 4 == 2 ? 1.6e7f : 16770000.0f));
    // s = 23: a saturated trigOffset with phaseEst past 2^24 (the loop's
    // phase keeps growing there, src/filter.cpp:210)
    pll_bad += pll_compare(pil, L, s == 23 ? 16777216.0f : trig0, &reruns, s == 23 ? 2.5e7f : 0.0f);
    steps += L;
  }
  // tiny, subnormal and non-finite pilot samples (input_ok's excluded range,
  // 2^-149 .. 2^-60, +-0, Inf, NaN): such chunks must re-run, never certify
  long long tiny_bad = 0, tiny_reruns = 0;
  for (int s = 0; s < 12; ++s) {
    for (long long k = 0; k < L; ++k) {
      const double amp = 0.2 * std::cos(2 * M_PI * 19e3 / 240e3 * (double)k + s);
      pil[k] = (float)amp;
      if (k % 61 == s) pil[k] = (float)logu(-149.0, -60.0);  // tiny and subnormal
      if (k % 499 == 7) pil[k] = (k & 1) ? -0.0f : 0.0f;
    }
    if (s == 10) pil[L / 2] = INFINITY;
    if (s == 11) pil[L / 3] = NAN;
    tiny_bad += pll_compare(pil, L, s % 2 ? 0.0f : 1.6e7f, &tiny_reruns);
  }
  std::free(pil);
  std::printf("{\"pll_tiny_mismatch\": %lld, \"pll_tiny_reruns\": %lld}\n", tiny_bad, tiny_reruns);
  std::printf(
      "{\"atan2\": [%lld, %lld, %lld], \"atan2_special\": %lld, \"atan2_rot\": [%lld, %lld, %lld], \"atan2_rot_special\": %lld, \"sincos\": [%lld, %lld, %lld], \"sincos_worst\": [%lld, %lld, %lld], "
      "\"atan2_max_rel_log2\": %.2f, \"atan2_rot_max_rel_log2\": %.2f, \"sincos_max_rel_log2\": %.2f, \"cert_window_ulps\": %u, \"pll_mismatch\": %lld, \"pll_chunks_rerun\": %lld, \"pll_steps\": %lld}\n",
      at.n, at.certified, at.mismatch, at.special, ar.n, ar.certified, ar.mismatch, ar.special, sc.n, sc.certified, sc.mismatch, scw.n, scw.certified, scw.mismatch, std::log2(at.max_rel), std::log2(ar.max_rel),
      std::log2(std::fmax(sc.max_rel, scw.max_rel)), kCertW, pll_bad,
      reruns, steps);
  return 0;
}
