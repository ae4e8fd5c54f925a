// dropin_harness.cpp -- drives the drop-in filter.h implementation
// (host/filter_hip.cpp, libdy4filter_hip.so) through its C++ std::vector
// API exactly the way src/project.cpp does (persistent state vectors, block
// after block), so tests/test_dropin.py can compare every function with the
// golden fixtures the compiled reference produced.  Raw little-endian f32 /
// u8 files in and out; parameters on the command line.
//
//   taps_lpf Fs Fc T U out
//   taps_bpf Fs Fb Fe T U out
//   fir_block  x h ns block nblk y states
//   fir_decim  D x h ns block nblk y states
//   resample   U M x h ns block nblk y states
//   demod      I Q prev_i prev_q out prevs  a0 b0 a1 b1 ...   (segments)
//   frontend   D iq_u8 h block nblk out states
//   threads    D iq_a iq_b h h_bpf block nblk out_a out_b   (two threads at once)
//   glue       x pilot outdir
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "sdr_filter_api.h"

namespace {

template <class T>
std::vector<T> load(const char* path) {
  FILE* f = std::fopen(path, "rb");
  if (!f) {
    std::fprintf(stderr, "cannot open %s\n", path);
    std::exit(2);
  }
  std::fseek(f, 0, SEEK_END);
  const long bytes = std::ftell(f);
  std::fseek(f, 0, SEEK_SET);
  std::vector<T> v(bytes / sizeof(T));
  if (!v.empty() && std::fread(v.data(), sizeof(T), v.size(), f) != v.size()) std::exit(2);
  std::fclose(f);
  return v;
}

void save(const std::string& path, const std::vector<float>& v) {
  FILE* f = std::fopen(path.c_str(), "wb");
  if (!f) std::exit(3);
  if (!v.empty()) std::fwrite(v.data(), sizeof(float), v.size(), f);
  std::fclose(f);
}

void append(std::vector<float>& dst, const std::vector<float>& src) { dst.insert(dst.end(), src.begin(), src.end()); }

std::vector<float> slice(const std::vector<float>& x, long a, long b) { return std::vector<float>(x.begin() + a, x.begin() + b); }

}  // namespace

int main(int argc, char** argv) {
  if (argc < 2) return 1;
  const std::string op = argv[1];
  if (op == "taps_lpf") {
    std::vector<float> h;
    impulseResponseLPF(std::strtof(argv[2], nullptr), std::strtof(argv[3], nullptr), (unsigned short)std::atoi(argv[4]),
                       h, std::atoi(argv[5]));
    save(argv[6], h);
  } else if (op == "taps_bpf") {
    std::vector<float> h;
    impulseResponseBPF(std::strtof(argv[2], nullptr), std::strtof(argv[3], nullptr), std::strtof(argv[4], nullptr),
                       (unsigned short)std::atoi(argv[5]), h, std::atoi(argv[6]));
    save(argv[7], h);
  } else if (op == "fir_block" || op == "fir_decim" || op == "resample") {
    int a = 2, D = 1, U = 1, M = 1;
    if (op == "fir_decim") D = std::atoi(argv[a++]);
    if (op == "resample") {
      U = std::atoi(argv[a++]);
      M = std::atoi(argv[a++]);
    }
    const auto x = load<float>(argv[a]);
    const auto h = load<float>(argv[a + 1]);
    const int ns = std::atoi(argv[a + 2]);
    const long block = std::atol(argv[a + 3]);
    const int nblk = std::atoi(argv[a + 4]);
    std::vector<float> state(ns, 0.0f), y, ys, sts;
    for (int b = 0; b < nblk; b++) {
      const auto xb = slice(x, b * block, (b + 1) * block);
      if (op == "fir_block")
        blockConvolveFIR(y, xb, h, state);
      else if (op == "fir_decim")
        downsampleBlockConvolveFIR(D, y, xb, h, state);
      else
        resampleBlockConvolveFIR(U, M, y, xb, h, state);
      append(ys, y);
      append(sts, state);
    }
    save(argv[a + 5], ys);
    save(argv[a + 6], sts);
  } else if (op == "demod") {
    const auto I = load<float>(argv[2]);
    const auto Q = load<float>(argv[3]);
    float pi = std::strtof(argv[4], nullptr), pq = std::strtof(argv[5], nullptr);
    std::vector<float> out, prevs, d;
    for (int a = 8; a + 1 < argc; a += 2) {
      const long s0 = std::atol(argv[a]), s1 = std::atol(argv[a + 1]);
      fmDemodArctan(slice(I, s0, s1), slice(Q, s0, s1), pi, pq, d);
      append(out, d);
      prevs.push_back(pi);
      prevs.push_back(pq);
    }
    save(argv[6], out);
    save(argv[7], prevs);
  } else if (op == "frontend") {
    // src/project.cpp:72-93: u8 -> float (iofunc.cpp:117-119), de-interleave,
    // FIR+decimate I and Q, discriminate -- block after block.
    const int D = std::atoi(argv[2]);
    const auto iq = load<unsigned char>(argv[3]);
    const auto h = load<float>(argv[4]);
    const long block = std::atol(argv[5]);
    const int nblk = std::atoi(argv[6]);
    std::vector<float> si(100, 0.0f), sq(100, 0.0f), yi, yq, dm, out, sts;
    float pi = 0, pq = 0;
    for (int b = 0; b < nblk; b++) {
      std::vector<float> xi(block), xq(block);
      for (long k = 0; k < block; k++) {
        xi[k] = float(((unsigned char)iq[2 * (b * block + k)] - 128) / 128.0);
        xq[k] = float(((unsigned char)iq[2 * (b * block + k) + 1] - 128) / 128.0);
      }
      downsampleBlockConvolveFIR(D, yi, xi, h, si);
      downsampleBlockConvolveFIR(D, yq, xq, h, sq);
      fmDemodArctan(yi, yq, pi, pq, dm);
      append(out, dm);
      append(sts, si);
      append(sts, sq);
      sts.push_back(pi);
      sts.push_back(pq);
    }
    save(argv[7], out);
    save(argv[8], sts);
  } else if (op == "threads") {
    // Two host threads inside the drop-in at once, each with its own stream
    // and state vectors (src/project.cpp:299-302 calls it from two threads
    // per block; here both run their whole block loops concurrently):
    // per block, the front end (as "frontend" above) and blockConvolveFIR of
    // the demodulated block -- out: demod ++ band-passed, block after block.
    const int D = std::atoi(argv[2]);
    const auto iqa = load<unsigned char>(argv[3]);
    const auto iqb = load<unsigned char>(argv[4]);
    const auto h = load<float>(argv[5]);
    const auto hb = load<float>(argv[6]);
    const long block = std::atol(argv[7]);
    const int nblk = std::atoi(argv[8]);
    auto work = [&](const std::vector<unsigned char>& iq, std::vector<float>& out) {
      std::vector<float> si(100, 0.0f), sq(100, 0.0f), sb(100, 0.0f), yi, yq, dm, bp;
      float pi = 0, pq = 0;
      for (int b = 0; b < nblk; b++) {
        std::vector<float> xi(block), xq(block);
        for (long k = 0; k < block; k++) {
          xi[k] = float(((unsigned char)iq[2 * (b * block + k)] - 128) / 128.0);
          xq[k] = float(((unsigned char)iq[2 * (b * block + k) + 1] - 128) / 128.0);
        }
        downsampleBlockConvolveFIR(D, yi, xi, h, si);
        downsampleBlockConvolveFIR(D, yq, xq, h, sq);
        fmDemodArctan(yi, yq, pi, pq, dm);
        blockConvolveFIR(bp, dm, hb, sb);
        append(out, dm);
        append(out, bp);
      }
    };
    std::vector<float> outa, outb;
    std::thread ta(work, std::cref(iqa), std::ref(outa));
    std::thread tb(work, std::cref(iqb), std::ref(outb));
    ta.join();
    tb.join();
    save(argv[9], outa);
    save(argv[10], outb);
  } else if (op == "glue") {
    // the host-side rows, in the order tests/golden/make_golden.py ran them
    const auto x = load<float>(argv[2]);
    const auto pf = load<float>(argv[3]);
    const std::string dir = argv[4];
    std::vector<float> nco, ncos, plls;
    float fI = 1, fQ = 0, integ = 0, ph = 0, toff = 0, ncs = 1;
    for (int b = 0; b < 2; b++) {
      fmPLL(slice(pf, b * 1024, (b + 1) * 1024), 19e3f, 240e3f, 2.0f, 0.0f, 0.01f, nco, fI, fQ, integ, ph, toff, ncs);
      append(ncos, nco);
      for (float v : {fI, fQ, integ, ph, toff, ncs}) plls.push_back(v);
    }
    save(dir + "/nco.f32", ncos);
    save(dir + "/pll_states.f32", plls);
    std::vector<float> dst(50, 0.0f), d1, d2, dd;
    delayBlock(slice(x, 0, 1024), dst, d1);
    delayBlock(slice(x, 1024, 2048), dst, d2);
    append(dd, d1);
    append(dd, d2);
    save(dir + "/delay.f32", dd);
    save(dir + "/delay_state.f32", dst);
    std::vector<float> y(x.rbegin(), x.rend()), o;
    pointwiseMultiply(x, slice(y, 0, 2000), o);
    save(dir + "/mul.f32", o);
    pointwiseAdd(x, y, o);
    save(dir + "/add.f32", o);
    pointwiseSubtract(x, y, o);
    save(dir + "/sub.f32", o);
    interleave(slice(x, 0, 100), slice(y, 0, 100), o);
    save(dir + "/inter.f32", o);
    std::vector<float> hp;
    impulseResponseBPF(240e3f, 18.5e3f, 19.5e3f, 101, hp, 1);
    convolveFIR(o, slice(x, 0, 300), hp);
    save(dir + "/conv.f32", o);
    downsample(slice(x, 0, 303), 10, o);
    save(dir + "/down.f32", o);
    upsample(slice(x, 0, 40), 3, o);
    save(dir + "/up.f32", o);
  } else {
    std::fprintf(stderr, "unknown op %s\n", op.c_str());
    return 1;
  }
  return 0;
}
