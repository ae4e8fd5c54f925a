// CPU proof for csrc/libm_exact.hpp: its float sin / cos / atan2 against
// glibc's double routines rounded to float -- what the reference's fmPLL
// stores (src/filter.cpp:199-221; the compiled reference calls glibc's
// atan2, sincos and cos: objdump of oracle/_ref/libref_filter.so).
// Test infrastructure (tests/test_libm_exact.py, tests/golden/make_libm_golden.py).
//
//   libm_sweep sincos <chunk_lo> <chunk_hi> <threads> [<out_prefix>]
//       every finite float whose bits u have u >> 20 in [chunk_lo, chunk_hi)
//       (4,096 chunks of 2^20 arguments cover all 2^32 bit patterns):
//       libm_exact's sincos_f against glibc's sin, cos and sincos.  Prints one
//       JSON line of counts.  With out_prefix: <p>.hash (per-chunk u64 hashes
//       of glibc's floats, the device test's reference) and <p>.near (every
//       argument whose glibc double lies within 4 double ulps of a float
//       rounding midpoint: u32 argument bits, u32 glibc sin float, u32 glibc
//       cos float, u32 flags).
//   libm_sweep atan2 <seed> <log2 samples> <threads> [<out>]
//       seeded pairs (PLL-like phase-detector products and the whole float
//       range): atan2_f against glibc; with out: every pair whose glibc double
//       lies within 4 ulps of a float midpoint (u32 y, u32 x, u32 glibc float).
//   libm_sweep eval <in> <out>
//       evaluate sin_f / cos_f / atan2_f on records of (u32 fn, u32 a, u32 b):
//       fn 0 sin(a), 1 cos(a), 2 atan2(a, b); writes u32 float bits.
#define SDR_HD
#include <algorithm>
#include <atomic>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <random>
#include <thread>
#include <vector>

#include "libm_exact.hpp"

using namespace sdr;

static inline uint32_t fbits(float f) {
  uint32_t b;
  std::memcpy(&b, &f, 4);
  return b;
}
static inline float bfloat(uint32_t b) {
  float f;
  std::memcpy(&f, &b, 4);
  return f;
}
static inline uint64_t dbits(double d) {
  uint64_t b;
  std::memcpy(&b, &d, 8);
  return b;
}
// the hash the device test recomputes (csrc/capi.hip sdr_libm_sincos_hash)
static inline uint64_t sm64(uint64_t z) {
  z += 0x9e3779b97f4a7c15ull;
  z = (z ^ (z >> 30)) * 0xbf58476d1ce4e5b9ull;
  z = (z ^ (z >> 27)) * 0x94d049bb133111ebull;
  return z ^ (z >> 31);
}
static inline uint64_t rec_hash(uint32_t u, uint32_t s, uint32_t c) {
  return sm64(((uint64_t)u << 32) | s) + sm64((((uint64_t)u << 32) | c) ^ 0x5bd1e9955bd1e995ull);
}
// within 4 double ulps of a float rounding midpoint
static inline bool near_mid(double d) { return libmx::near_float_mid(d, 4.0); }

static int sweep_sincos(int clo, int chi, int nth, const char* out) {
  std::atomic<int> next{clo};
  std::atomic<long long> n{0}, bad_s{0}, bad_c{0}, bad_sc{0}, slow{0}, fast_cert_bad{0};
  std::vector<uint64_t> hash(4096, 0);
  std::vector<uint32_t> near;
  std::mutex mu;
  auto work = [&] {
    std::vector<uint32_t> loc;
    long long ln = 0, bs = 0, bc = 0, bsc = 0, sl = 0, fcm = 0;
    for (int ch; (ch = next.fetch_add(1)) < chi;) {
      uint64_t h = 0;
      for (uint32_t k = 0; k < (1u << 20); ++k) {
        const uint32_t u = ((uint32_t)ch << 20) | k;
        if ((u & 0x7f800000u) == 0x7f800000u) continue;  // Inf / NaN
        const float x = bfloat(u);
        const double sd = std::sin((double)x), cd = std::cos((double)x);
        double ssd, scd;
        sincos((double)x, &ssd, &scd);
        const float gs = (float)sd, gc = (float)cd;
        const libmx::SinCos m = libmx::sincos_f(x);
        const float ms = m.s, mc = m.c;
        ++ln;
        if (fbits(ms) != fbits(gs)) {
          if (bs < 20) std::fprintf(stderr, "sin mismatch x=%a (0x%08x) glibc=%a mine=%a d=%a\n", x, u, gs, ms, sd);
          ++bs;
        }
        if (fbits(mc) != fbits(gc)) {
          if (bc < 20) std::fprintf(stderr, "cos mismatch x=%a (0x%08x) glibc=%a mine=%a d=%a\n", x, u, gc, mc, cd);
          ++bc;
        }
        if (dbits(ssd) != dbits(sd) || dbits(scd) != dbits(cd)) ++bsc;
        h += rec_hash(u, fbits(gs), fbits(gc));
        const bool ns = near_mid(sd), nc = near_mid(cd);
        if (ns || nc) {
          loc.push_back(u);
          loc.push_back(fbits(gs));
          loc.push_back(fbits(gc));
          loc.push_back((ns ? 1u : 0u) | (nc ? 2u : 0u));
        }
        // the fast step the PLL kernel runs (pll_fast.hpp sincos_fast: fma
        // only, the device's bits too) on its whole domain |x| < 2^26: every
        // result its window certifies must be glibc's float -- the proof of
        // kCertWSc -- and the rest is the double-double path's share
        if (std::fabs(x) < 0x1p26f && x != 0.0f) {
          unsigned score = ~0u;
          pllfast::Osc o;
          float a, b;
          pllfast::sincos_fast<libmx::ExactOps>(x, a, b, score, o);
          if (score < pllfast::kCertifiedSc)
            ++sl;
          else if (fbits(a) != fbits(gs) || fbits(b) != fbits(gc))
            ++fcm;
        }
      }
      hash[ch] = h;
    }
    std::lock_guard<std::mutex> g(mu);
    near.insert(near.end(), loc.begin(), loc.end());
    n += ln;
    bad_s += bs;
    bad_c += bc;
    bad_sc += bsc;
    slow += sl;
    fast_cert_bad += fcm;
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nth; ++t) th.emplace_back(work);
  for (auto& t : th) t.join();
  std::printf(
      "{\"args\": %lld, \"sin_mismatch\": %lld, \"cos_mismatch\": %lld, \"sincos_vs_sin_cos\": %lld, "
      "\"near_midpoint\": %zu, \"fast_uncertified\": %lld, \"fast_certified_mismatch\": %lld, "
      "\"cert_window_sc_ulps\": %u}\n",
      n.load(), bad_s.load(), bad_c.load(), bad_sc.load(), near.size() / 4, slow.load(), fast_cert_bad.load(),
      pllfast::kCertWSc);
  if (out) {
    // records sorted by argument bits (threads interleave chunks)
    std::vector<size_t> idx(near.size() / 4);
    for (size_t i = 0; i < idx.size(); ++i) idx[i] = i;
    std::sort(idx.begin(), idx.end(), [&](size_t a, size_t b) { return near[4 * a] < near[4 * b]; });
    std::string p(out);
    FILE* f = std::fopen((p + ".hash").c_str(), "wb");
    std::fwrite(hash.data(), 8, hash.size(), f);
    std::fclose(f);
    f = std::fopen((p + ".near").c_str(), "wb");
    for (size_t i : idx) std::fwrite(&near[4 * i], 4, 4, f);
    std::fclose(f);
  }
  return 0;
}

// a float with sign, exponent in [elo, ehi] (unbiased) and a uniform mantissa
static inline float rand_float(std::mt19937_64& g, int elo, int ehi) {
  const uint64_t r = g();
  const int e = elo + (int)((r >> 32) % (uint64_t)(ehi - elo + 1));
  const uint32_t be = e < -126 ? 0u : (uint32_t)(e + 127);  // below 2^-126: subnormal
  const uint32_t u = ((uint32_t)(r >> 63) << 31) | (be << 23) | ((uint32_t)r & 0x7fffffu);
  return bfloat(u);
}

static int sweep_atan2(uint64_t seed, int lg, int nth, const char* out) {
  const long long N = 1ll << lg;
  std::atomic<long long> next{0}, bad{0}, slow{0};
  std::vector<uint32_t> near;
  std::mutex mu;
  const long long CH = 1 << 20;
  auto work = [&] {
    std::vector<uint32_t> loc;
    long long lb = 0, ls = 0;
    for (long long c; (c = next.fetch_add(1)) * CH < N;) {
      std::mt19937_64 g(seed * 0x9e3779b97f4a7c15ull + (uint64_t)c);
      for (long long i = 0; i < CH; ++i) {
        float y, x;
        switch (i & 3) {
          case 0: {  // the phase detector: v * -fbQ, v * fbI with a pilot-sized v and unit feedback
            const float v = rand_float(g, -12, -1);
            const double th = (double)(g() >> 11) * 0x1p-53 * 6.283185307179586;
            y = v * -(float)std::sin(th);
            x = v * (float)std::cos(th);
            break;
          }
          case 1:  // products of the kernel's domain
            y = rand_float(g, -60, 60);
            x = rand_float(g, -60, 60);
            break;
          case 2:  // near the diagonal and the axes (the fast path's branch points)
            y = rand_float(g, -4, 4);
            x = bfloat(fbits(y) ^ (uint32_t)(g() & 0x800000ffu));
            break;
          default:  // the whole float range, subnormals included
            y = rand_float(g, -149, 127);
            x = rand_float(g, -149, 127);
            break;
        }
        if (!std::isfinite(x) || !std::isfinite(y) || x == 0.0f || y == 0.0f) continue;
        const double d = std::atan2((double)y, (double)x);
        const float gf = (float)d;
        const float mf = libmx::atan2_f(y, x);
        if (fbits(mf) != fbits(gf)) {
          if (lb < 20) std::fprintf(stderr, "atan2 mismatch y=%a x=%a glibc=%a mine=%a d=%a\n", y, x, gf, mf, d);
          ++lb;
        }
        if (near_mid(d)) {
          loc.push_back(fbits(y));
          loc.push_back(fbits(x));
          loc.push_back(fbits(gf));
        }
        unsigned score = ~0u;
        const double a = pllfast::atan2_abs<libmx::ExactOps>(y, x, score);
        ls += score < pllfast::kCertified || !libmx::normal_or_float(a);
      }
    }
    std::lock_guard<std::mutex> gd(mu);
    near.insert(near.end(), loc.begin(), loc.end());
    bad += lb;
    slow += ls;
  };
  std::vector<std::thread> th;
  for (int t = 0; t < nth; ++t) th.emplace_back(work);
  for (auto& t : th) t.join();
  std::printf("{\"pairs\": %lld, \"atan2_mismatch\": %lld, \"near_midpoint\": %zu, \"fast_uncertified\": %lld}\n", N,
              bad.load(), near.size() / 3, slow.load());
  if (out) {
    FILE* f = std::fopen(out, "wb");
    std::fwrite(near.data(), 4, near.size(), f);
    std::fclose(f);
  }
  return 0;
}

static int eval(const char* in, const char* out) {
  FILE* f = std::fopen(in, "rb");
  if (!f) return 1;
  std::vector<uint32_t> rec;
  uint32_t r[3];
  while (std::fread(r, 4, 3, f) == 3) rec.insert(rec.end(), r, r + 3);
  std::fclose(f);
  std::vector<uint32_t> res(rec.size() / 3);
  for (size_t i = 0; i < res.size(); ++i) {
    const float a = bfloat(rec[3 * i + 1]), b = bfloat(rec[3 * i + 2]);
    float v;
    switch (rec[3 * i]) {
      case 0: v = libmx::sin_f(a); break;
      case 1: v = libmx::cos_f(a); break;
      default: v = libmx::atan2_f(a, b); break;
    }
    res[i] = fbits(v);
  }
  f = std::fopen(out, "wb");
  std::fwrite(res.data(), 4, res.size(), f);
  std::fclose(f);
  return 0;
}

int main(int argc, char** argv) {
  if (argc >= 5 && !std::strcmp(argv[1], "sincos"))
    return sweep_sincos(std::atoi(argv[2]), std::atoi(argv[3]), std::atoi(argv[4]), argc > 5 ? argv[5] : nullptr);
  if (argc >= 5 && !std::strcmp(argv[1], "atan2"))
    return sweep_atan2(std::strtoull(argv[2], nullptr, 10), std::atoi(argv[3]), std::atoi(argv[4]),
                       argc > 5 ? argv[5] : nullptr);
  if (argc == 4 && !std::strcmp(argv[1], "eval")) return eval(argv[2], argv[3]);
  std::fprintf(stderr, "usage: libm_sweep sincos|atan2|eval ...\n");
  return 2;
}
