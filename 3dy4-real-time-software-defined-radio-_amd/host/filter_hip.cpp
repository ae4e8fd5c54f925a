// filter_hip.cpp -- drop-in implementation of the reference's DSP block
// library API (include/filter.h:17-34 / src/filter.cpp), MI355X edition.
//
// Link it in place of src/filter.cpp:
//     g++ -O3 -std=c++17 project.cpp iofunc.cpp ... filter_hip.cpp -lsdrhip
// (oracle/Makefile, target `dropin`, does exactly that with the reference's
// unmodified src/project.cpp).  The four data-parallel functions run on the
// GPU through the C ABI of include/sdr_hip.h; coefficient design and the
// sequential / O(n) glue stay on the host, written to the reference's exact
// float/double promotion rules so every output is bit-identical.
//
// Threading: src/project.cpp:299-302 spawns a front-end and a back-end
// thread per block and calls into this library from both at once.  Device
// contexts (stream + scratch) come from a process-wide pool, leased per
// call, so the per-block thread churn never recreates HIP streams.
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <mutex>
#include <vector>

#include "sdr_filter_api.h"
#include "sdr_hip.h"

namespace {

constexpr double kPi = 3.14159265358979323846;  // include/dy4.h:14 (PLL)

class CtxPool {
 public:
  sdr_ctx* take() {
    {
      std::lock_guard<std::mutex> g(mu_);
      if (!free_.empty()) {
        sdr_ctx* c = free_.back();
        free_.pop_back();
        return c;
      }
    }
    const char* env = std::getenv("SDR_DEVICE");
    const int dev = env ? std::atoi(env) : 0;
    sdr_ctx* c = nullptr;
    const int rc = sdr_ctx_create(dev, &c);
    if (rc != SDR_OK) {
      std::fprintf(stderr, "filter_hip: cannot open GPU %d: %s\n", dev, sdr_strerror(rc));
      std::abort();
    }
    return c;
  }
  void give(sdr_ctx* c) {
    std::lock_guard<std::mutex> g(mu_);
    free_.push_back(c);
  }

 private:
  std::mutex mu_;
  std::vector<sdr_ctx*> free_;
};

CtxPool& pool() {
  static CtxPool* p = new CtxPool();  // intentionally leaked: outlives detached threads
  return *p;
}

struct Lease {
  sdr_ctx* c;
  Lease() : c(pool().take()) {}
  ~Lease() { pool().give(c); }
};

void check(int rc, sdr_ctx* c, const char* fn) {
  if (rc == SDR_OK) return;
  std::fprintf(stderr, "filter_hip: %s: %s (%s)\n", fn, sdr_strerror(rc), sdr_ctx_last_error(c));
  std::abort();
}

}  // namespace

// src/filter.cpp:14-29 / :31-49 -- windowed-sinc taps (setup, host C++ in
// libsdrhip: one implementation for the drop-in and the C ABI).
void impulseResponseLPF(float Fs, float Fc, unsigned short int num_taps, std::vector<float>& h, int upFactor) {
  h.assign(num_taps, 0.0f);
  if (num_taps) check(sdr_taps_lpf(Fs, Fc, num_taps, upFactor, h.data()), nullptr, "impulseResponseLPF");
}

void impulseResponseBPF(float Fs, float Fb, float Fe, unsigned short int num_taps, std::vector<float>& h,
                        int upFactor) {
  h.assign(num_taps, 0.0f);
  if (num_taps) check(sdr_taps_bpf(Fs, Fb, Fe, num_taps, upFactor, h.data()), nullptr, "impulseResponseBPF");
}

// src/filter.cpp:53-64 -- one-shot full convolution; not on the streaming
// path (project.cpp never calls it), so it stays a host loop.
void convolveFIR(std::vector<float>& y, const std::vector<float>& x, const std::vector<float>& h) {
  const long nx = (long)x.size(), nh = (long)h.size();
  y.assign(nx + nh - 1, 0.0f);
  for (long n = 0; n < (long)y.size(); n++) {
    float acc = 0.0f;
    const long k0 = n - nx + 1 > 0 ? n - nx + 1 : 0;
    const long k1 = n < nh - 1 ? n : nh - 1;
    // only 0 <= n-k < nx contributes; ascending k as in the reference
    for (long k = k0; k <= k1; k++) acc = acc + h[k] * x[n - k];
    y[n] = acc;
  }
}

// src/filter.cpp:66-83 -- stateful block FIR (GPU).
void blockConvolveFIR(std::vector<float>& y, const std::vector<float>& x, const std::vector<float>& h,
                      std::vector<float>& state) {
  y.assign(x.size(), 0.0f);
  Lease l;
  check(sdr_fir_block_f32(l.c, x.data(), (long long)x.size(), h.data(), (int)h.size(), state.data(),
                          (int)state.size(), y.data()),
        l.c, "blockConvolveFIR");
}

// src/filter.cpp:85-102 -- arctan-free FM discriminator (GPU).
void fmDemodArctan(const std::vector<float>& I, const std::vector<float>& Q, float& prev_I, float& prev_Q,
                   std::vector<float>& fm_demod) {
  fm_demod.resize(I.size());
  if (Q.size() < I.size()) {
    std::fprintf(stderr, "filter_hip: fmDemodArctan: Q shorter than I (%zu < %zu)\n", Q.size(), I.size());
    std::abort();
  }
  Lease l;
  check(sdr_fm_demod_f32(l.c, I.data(), Q.data(), (long long)I.size(), &prev_I, &prev_Q, fm_demod.data()), l.c,
        "fmDemodArctan");
}

// src/filter.cpp:104-110 (host; unused by project.cpp)
void downsample(const std::vector<float> data, size_t factor, std::vector<float>& downsampled) {
  downsampled.clear();
  if (factor == 0) {
    std::fprintf(stderr, "filter_hip: downsample: factor 0\n");
    std::abort();
  }
  downsampled.reserve(data.size() / factor + 1);
  for (size_t i = 0; i < data.size(); i += factor) downsampled.push_back(data[i]);
}

// src/filter.cpp:112-121 (host; unused by project.cpp)
void upsample(const std::vector<float> data, size_t factor, std::vector<float>& upsampled) {
  const size_t stretch = factor > 1 ? factor : 1;
  upsampled.assign(data.size() * stretch, 0.0f);
  for (size_t i = 0; i < data.size(); i++) upsampled[i * stretch] = data[i];
}

// src/filter.cpp:123-140 -- FIR + decimate, only kept outputs computed (GPU).
void downsampleBlockConvolveFIR(int factor, std::vector<float>& y, const std::vector<float>& x,
                                const std::vector<float>& h, std::vector<float>& state) {
  if (factor <= 0) {
    std::fprintf(stderr, "filter_hip: downsampleBlockConvolveFIR: factor %d\n", factor);
    std::abort();
  }
  y.assign(x.size() / factor, 0.0f);
  Lease l;
  check(sdr_fir_decim_f32(l.c, factor, x.data(), (long long)x.size(), h.data(), (int)h.size(), state.data(),
                          (int)state.size(), y.data()),
        l.c, "downsampleBlockConvolveFIR");
}

// src/filter.cpp:142-173 -- polyphase rational resampler (GPU).
void resampleBlockConvolveFIR(int upFactor, int downFactor, std::vector<float>& y, const std::vector<float>& x,
                              const std::vector<float>& h, std::vector<float>& state) {
  const long long ny = sdr_resample_out_len(upFactor, downFactor, (long long)x.size());
  if (ny < 0) {
    std::fprintf(stderr, "filter_hip: resampleBlockConvolveFIR: factors %d/%d\n", upFactor, downFactor);
    std::abort();
  }
  y.assign((size_t)ny, 0.0f);
  Lease l;
  check(sdr_resample_f32(l.c, upFactor, downFactor, x.data(), (long long)x.size(), h.data(), (int)h.size(),
                         state.data(), (int)state.size(), y.data(), ny),
        l.c, "resampleBlockConvolveFIR");
}

// src/filter.cpp:174-228 -- pilot PLL + NCO.  A per-sample recurrence, so
// it stays on the host.  State is float; atan2/cos/sin are the libm double
// functions applied to the float arguments (the reference's unqualified
// calls resolve to ::atan2(double,double) and friends), rounded to float.
void fmPLL(const std::vector<float>& PLLin, const float freq, const float Fs, const float ncoScale,
           const float phaseAdjust, const float normBandwidth, std::vector<float>& ncoOut, float& feedbackI,
           float& feedbackQ, float& integrator, float& phaseEst, float& trigOffset, float& nco_state) {
  const float Kp = normBandwidth * 2.666f;
  const float Ki = normBandwidth * normBandwidth * 3.555f;
  const long n = (long)PLLin.size();
  ncoOut.resize(PLLin.size(), 0.0f);
  if (n == 0) {
    std::fprintf(stderr, "filter_hip: fmPLL: empty block\n");
    std::abort();
  }
  ncoOut[0] = nco_state;
  const double step = 2 * kPi * (double)(freq / Fs);
  for (long k = 0; k < n; k++) {
    const float in = PLLin[k];
    const float eI = (in == 0 ? 1.0f : in) * feedbackI;
    const float eQ = in * (-1.0f * feedbackQ);
    const float eD = (float)std::atan2((double)eQ, (double)eI);
    integrator = integrator + Ki * eD;
    phaseEst = phaseEst + (Kp * eD + integrator);
    trigOffset = trigOffset + 1.0f;
    const float arg = (float)(step * (double)trigOffset + (double)phaseEst);
    feedbackI = (float)std::cos((double)arg);
    feedbackQ = (float)std::sin((double)arg);
    const float nco = (float)std::cos((double)(arg * ncoScale + phaseAdjust));
    if (k == n - 1)
      nco_state = nco;
    else
      ncoOut[k + 1] = nco;
  }
}

// src/filter.cpp:229-251 -- delay line: out = [state, in[0..n-S)], state = in[n-S..n)
void delayBlock(const std::vector<float>& input_block, std::vector<float>& state_block,
                std::vector<float>& output_block) {
  const size_t n = input_block.size(), S = state_block.size();
  if (n < S) {
    std::fprintf(stderr, "filter_hip: delayBlock: block %zu shorter than delay %zu\n", n, S);
    std::abort();
  }
  output_block.resize(n);
  for (size_t i = 0; i < S; i++) output_block[i] = state_block[i];
  for (size_t i = S; i < n; i++) output_block[i] = input_block[i - S];
  for (size_t i = 0; i < S; i++) state_block[i] = input_block[n - S + i];
}

// src/filter.cpp:253-266 -- stereo mixer with its x2 gain
void pointwiseMultiply(const std::vector<float>& block1, const std::vector<float>& block2,
                       std::vector<float>& output) {
  const size_t n = block1.size() < block2.size() ? block1.size() : block2.size();
  output.resize(n);
  for (size_t i = 0; i < n; i++) output[i] = block1[i] * block2[i] * 2;
}

// src/filter.cpp:267-290 -- L = M + S, R = M - S (length of the first operand)
void pointwiseAdd(const std::vector<float>& block1, const std::vector<float>& block2, std::vector<float>& output) {
  if (block2.size() < block1.size()) {
    std::fprintf(stderr, "filter_hip: pointwiseAdd: operand sizes %zu/%zu\n", block1.size(), block2.size());
    std::abort();
  }
  output.resize(block1.size());
  for (size_t i = 0; i < block1.size(); i++) output[i] = block1[i] + block2[i];
}

void pointwiseSubtract(const std::vector<float>& block1, const std::vector<float>& block2,
                       std::vector<float>& output) {
  if (block2.size() < block1.size()) {
    std::fprintf(stderr, "filter_hip: pointwiseSubtract: operand sizes %zu/%zu\n", block1.size(), block2.size());
    std::abort();
  }
  output.resize(block1.size());
  for (size_t i = 0; i < block1.size(); i++) output[i] = block1[i] - block2[i];
}

// src/filter.cpp:291-301 -- L0 R0 L1 R1 ...
void interleave(const std::vector<float>& left, const std::vector<float>& right, std::vector<float>& output) {
  const size_t n = left.size() + right.size();
  output.resize(n);
  for (size_t i = 0; i < n; i += 2) output[i] = left[i / 2];
  for (size_t i = 1; i < n; i += 2) output[i] = right[i / 2];
}
