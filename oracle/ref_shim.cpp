// ref_shim.cpp -- C-callable wrappers around the REFERENCE's own compiled
// src/filter.cpp, used only to generate golden fixtures and to time the
// reference as the CPU baseline.  TEST INFRASTRUCTURE ONLY.
//
// Built by oracle/Makefile (target `ref`) together with
// $(REF)/src/filter.cpp straight from /root/reference -- the reference source
// is compiled where it lies and never copied; the output goes to
// oracle/_ref/ (git-ignored).  Each wrapper marshals plain pointers into the
// std::vector API declared in the reference's include/filter.h:17-34 and
// back, preserving its in-place state semantics.
#include "filter.h"

#include <cstring>
#include <vector>

namespace {
std::vector<float> vec(const float* p, long n) { return std::vector<float>(p, p + (n > 0 ? n : 0)); }
void out(const std::vector<float>& v, float* p) { if (!v.empty()) std::memcpy(p, v.data(), v.size() * sizeof(float)); }
}  // namespace

extern "C" {

long ref_taps_lpf(float Fs, float Fc, unsigned short T, int up, float* h) {
  std::vector<float> v;
  impulseResponseLPF(Fs, Fc, T, v, up);
  out(v, h);
  return (long)v.size();
}

long ref_taps_bpf(float Fs, float Fb, float Fe, unsigned short T, int up, float* h) {
  std::vector<float> v;
  impulseResponseBPF(Fs, Fb, Fe, T, v, up);
  out(v, h);
  return (long)v.size();
}

long ref_convolve_full(const float* x, long nx, const float* h, int nh, float* y) {
  std::vector<float> yv;
  convolveFIR(yv, vec(x, nx), vec(h, nh));
  out(yv, y);
  return (long)yv.size();
}

long ref_fir_block(const float* x, long nx, const float* h, int nh, float* state, int ns, float* y) {
  std::vector<float> yv, st = vec(state, ns);
  blockConvolveFIR(yv, vec(x, nx), vec(h, nh), st);
  out(yv, y);
  out(st, state);
  return (long)yv.size();
}

long ref_fir_decim(int D, const float* x, long nx, const float* h, int nh, float* state, int ns, float* y) {
  std::vector<float> yv, st = vec(state, ns);
  downsampleBlockConvolveFIR(D, yv, vec(x, nx), vec(h, nh), st);
  out(yv, y);
  out(st, state);
  return (long)yv.size();
}

long ref_resample(int up, int down, const float* x, long nx, const float* h, int nh, float* state, int ns, float* y) {
  std::vector<float> yv, st = vec(state, ns);
  resampleBlockConvolveFIR(up, down, yv, vec(x, nx), vec(h, nh), st);
  out(yv, y);
  out(st, state);
  return (long)yv.size();
}

long ref_fm_demod(const float* I, const float* Q, long n, float* prev_i, float* prev_q, float* o) {
  std::vector<float> dv;
  fmDemodArctan(vec(I, n), vec(Q, n), *prev_i, *prev_q, dv);
  out(dv, o);
  return (long)dv.size();
}

long ref_downsample(const float* x, long n, long factor, float* o) {
  std::vector<float> dv;
  downsample(vec(x, n), (size_t)factor, dv);
  out(dv, o);
  return (long)dv.size();
}

long ref_upsample(const float* x, long n, long factor, float* o) {
  std::vector<float> uv;
  upsample(vec(x, n), (size_t)factor, uv);
  out(uv, o);
  return (long)uv.size();
}

long ref_fm_pll(const float* in, long n, float freq, float Fs, float nco_scale, float phase_adjust, float norm_bw,
                float* nco_out, float* pll) {
  std::vector<float> nv;
  fmPLL(vec(in, n), freq, Fs, nco_scale, phase_adjust, norm_bw, nv, pll[0], pll[1], pll[2], pll[3], pll[4], pll[5]);
  out(nv, nco_out);
  return (long)nv.size();
}

long ref_delay_block(const float* in, long n, float* state, int ns, float* o) {
  std::vector<float> ov, st = vec(state, ns);
  delayBlock(vec(in, n), st, ov);
  out(ov, o);
  out(st, state);
  return (long)ov.size();
}

long ref_pointwise_mul(const float* a, long na, const float* b, long nb, float* o) {
  std::vector<float> ov;
  pointwiseMultiply(vec(a, na), vec(b, nb), ov);
  out(ov, o);
  return (long)ov.size();
}

long ref_pointwise_add(const float* a, long na, const float* b, long nb, float* o) {
  std::vector<float> ov;
  pointwiseAdd(vec(a, na), vec(b, nb), ov);
  out(ov, o);
  return (long)ov.size();
}

long ref_pointwise_sub(const float* a, long na, const float* b, long nb, float* o) {
  std::vector<float> ov;
  pointwiseSubtract(vec(a, na), vec(b, nb), ov);
  out(ov, o);
  return (long)ov.size();
}

long ref_interleave(const float* l, long nl, const float* r, long nr, float* o) {
  std::vector<float> ov;
  interleave(vec(l, nl), vec(r, nr), ov);
  out(ov, o);
  return (long)ov.size();
}

// The reference's own front end sequence (src/project.cpp:86-90), called
// block after block by the CPU-baseline timer with persistent vectors, the
// way project.cpp's loop does.
struct ref_front {
  std::vector<float> h, si, sq, yi, yq, dm, xi, xq;
  float pi = 0, pq = 0;
};

void* ref_front_new(const float* h, int nh, int ns) {
  ref_front* f = new ref_front();
  f->h.assign(h, h + nh);
  f->si.assign(ns, 0.0f);
  f->sq.assign(ns, 0.0f);
  return f;
}

void ref_front_free(void* p) { delete static_cast<ref_front*>(p); }

long ref_front_run(void* p, int D, const float* I, const float* Q, long n, float* demod) {
  ref_front* f = static_cast<ref_front*>(p);
  f->xi.assign(I, I + n);
  f->xq.assign(Q, Q + n);
  downsampleBlockConvolveFIR(D, f->yi, f->xi, f->h, f->si);
  downsampleBlockConvolveFIR(D, f->yq, f->xq, f->h, f->sq);
  fmDemodArctan(f->yi, f->yq, f->pi, f->pq, f->dm);
  if (demod) out(f->dm, demod);
  return (long)f->dm.size();
}

// The resampler (src/filter.cpp:142-173, cfg3) and the 1024-tap block FIR on
// I and Q (:66-83, cfg5), block after block with persistent vectors, for the
// CPU baseline of those configs.
struct ref_resample_state {
  int up = 1, down = 1;
  std::vector<float> h, st, x, y;
};

void* ref_resample_new(int up, int down, const float* h, int nh, int ns) {
  auto* r = new ref_resample_state();
  r->up = up;
  r->down = down;
  r->h.assign(h, h + nh);
  r->st.assign(ns, 0.0f);
  return r;
}

void ref_resample_free(void* p) { delete static_cast<ref_resample_state*>(p); }

long ref_resample_run(void* p, const float* x, long n, float* y) {
  auto* r = static_cast<ref_resample_state*>(p);
  r->x.assign(x, x + n);
  resampleBlockConvolveFIR(r->up, r->down, r->y, r->x, r->h, r->st);
  if (y) out(r->y, y);
  return (long)r->y.size();
}

struct ref_block_state {
  std::vector<float> h, si, sq, xi, xq, yi, yq;
};

void* ref_block_new(const float* h, int nh, int ns) {
  auto* r = new ref_block_state();
  r->h.assign(h, h + nh);
  r->si.assign(ns, 0.0f);
  r->sq.assign(ns, 0.0f);
  return r;
}

void ref_block_free(void* p) { delete static_cast<ref_block_state*>(p); }

long ref_block_run(void* p, const float* I, const float* Q, long n, float* yi, float* yq) {
  auto* r = static_cast<ref_block_state*>(p);
  r->xi.assign(I, I + n);
  r->xq.assign(Q, Q + n);
  blockConvolveFIR(r->yi, r->xi, r->h, r->si);
  blockConvolveFIR(r->yq, r->xq, r->h, r->sq);
  if (yi) out(r->yi, yi);
  if (yq) out(r->yq, yq);
  return (long)r->yi.size();
}

}  // extern "C"
