/*
 * c_abi_example.c -- a plain-C caller of libsdrhip.so (include/sdr_hip.h),
 * the binding INTEGRATION.md section 2 describes, compiled with gcc and run
 * by tests/test_capi.py on the GPU box.
 *
 * 8 independent streams x 3 consecutive 65,540-pair blocks of the RTL-SDR
 * wire format go through the batched device call sdr_frontend_u8_dev; every
 * stream is then replayed block by block through the one-block host call
 * sdr_frontend_u8 (the filter.h contract) with its own state, and the two
 * must agree bit for bit, outputs and carried state.  Prints "ok <checksum>".
 */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "sdr_hip.h"

#define CHECK(call)                                                                    \
  do {                                                                                 \
    int rc_ = (call);                                                                  \
    if (rc_ != SDR_OK) {                                                               \
      fprintf(stderr, "%s failed: %s (%s)\n", #call, sdr_strerror(rc_),                \
              ctx ? sdr_ctx_last_error(ctx) : "");                                     \
      return 1;                                                                        \
    }                                                                                  \
  } while (0)

enum { NS = 8, NBLK = 3, D = 10, T = 101, NST = 100 };
static const long long NP = 65540; /* pairs per block (multiple of D) */

int main(void) {
  sdr_ctx *ctx = NULL;
  CHECK(sdr_ctx_create(0, &ctx));
  const long long nout = NP / D, iq_stride = 2 * NP;
  float h[T];
  CHECK(sdr_taps_lpf(2.4e6f, 100e3f, T, 1, h));

  /* device buffers: the whole recording of every stream, states, outputs */
  void *d_iq, *d_h, *d_si, *d_sq, *d_pi, *d_pq, *d_out;
  CHECK(sdr_dev_alloc(ctx, (size_t)NS * NBLK * iq_stride, &d_iq));
  CHECK(sdr_dev_alloc(ctx, sizeof h, &d_h));
  CHECK(sdr_dev_alloc(ctx, (size_t)NS * NST * 4, &d_si));
  CHECK(sdr_dev_alloc(ctx, (size_t)NS * NST * 4, &d_sq));
  CHECK(sdr_dev_alloc(ctx, (size_t)NS * 4, &d_pi));
  CHECK(sdr_dev_alloc(ctx, (size_t)NS * 4, &d_pq));
  CHECK(sdr_dev_alloc(ctx, (size_t)NS * nout * 4, &d_out));
  CHECK(sdr_copy_h2d(ctx, d_h, h, sizeof h));
  CHECK(sdr_dev_memset(ctx, d_si, 0, (size_t)NS * NST * 4));
  CHECK(sdr_dev_memset(ctx, d_sq, 0, (size_t)NS * NST * 4));
  CHECK(sdr_dev_memset(ctx, d_pi, 0, (size_t)NS * 4));
  CHECK(sdr_dev_memset(ctx, d_pq, 0, (size_t)NS * 4));
  /* stream s, block b at d_iq + (b*NS + s)*iq_stride: a synthetic FM signal per stream */
  for (int b = 0; b < NBLK; ++b)
    CHECK(sdr_synth_fm_u8_dev(ctx, (uint8_t *)d_iq + (size_t)b * NS * iq_stride, NP, NS, iq_stride, 77 + b));

  uint8_t *iq = malloc((size_t)NS * NBLK * iq_stride);
  float *dev_out = malloc((size_t)NBLK * NS * nout * 4);
  float *host_out = malloc((size_t)nout * 4);
  CHECK(sdr_copy_d2h(ctx, iq, d_iq, (size_t)NS * NBLK * iq_stride));

  for (int b = 0; b < NBLK; ++b) {
    CHECK(sdr_frontend_u8_dev(ctx, D, (uint8_t *)d_iq + (size_t)b * NS * iq_stride, NP, NS, iq_stride, d_h, T,
                              d_si, d_sq, NST, d_pi, d_pq, d_out, nout));
    CHECK(sdr_copy_d2h(ctx, dev_out + (size_t)b * NS * nout, d_out, (size_t)NS * nout * 4)); /* synchronous */
  }
  float dev_si[NS * NST], dev_sq[NS * NST], dev_pi[NS], dev_pq[NS];
  CHECK(sdr_copy_d2h(ctx, dev_si, d_si, sizeof dev_si));
  CHECK(sdr_copy_d2h(ctx, dev_sq, d_sq, sizeof dev_sq));
  CHECK(sdr_copy_d2h(ctx, dev_pi, d_pi, sizeof dev_pi));
  CHECK(sdr_copy_d2h(ctx, dev_pq, d_pq, sizeof dev_pq));

  unsigned long long sum = 0;
  for (int s = 0; s < NS; ++s) {
    float si[NST] = {0}, sq[NST] = {0}, pi = 0.0f, pq = 0.0f;
    for (int b = 0; b < NBLK; ++b) {
      CHECK(sdr_frontend_u8(ctx, D, iq + ((size_t)b * NS + s) * iq_stride, NP, h, T, si, sq, NST, &pi, &pq,
                            host_out));
      const float *d = dev_out + ((size_t)b * NS + s) * nout;
      if (memcmp(d, host_out, (size_t)nout * 4) != 0) {
        fprintf(stderr, "stream %d block %d: batched and one-block calls differ\n", s, b);
        return 1;
      }
      for (long long k = 0; k < nout; ++k) {
        uint32_t u;
        memcpy(&u, d + k, 4);
        sum = sum * 1000003ULL + u;
      }
    }
    if (memcmp(si, dev_si + s * NST, sizeof si) || memcmp(sq, dev_sq + s * NST, sizeof sq) ||
        memcmp(&pi, dev_pi + s, 4) || memcmp(&pq, dev_pq + s, 4)) {
      fprintf(stderr, "stream %d: carried state differs\n", s);
      return 1;
    }
  }
  printf("ok %016llx\n", sum);
  free(iq);
  free(dev_out);
  free(host_out);
  void *bufs[] = {d_iq, d_h, d_si, d_sq, d_pi, d_pq, d_out};
  for (int i = 0; i < 7; ++i) CHECK(sdr_dev_free(ctx, bufs[i]));
  CHECK(sdr_ctx_destroy(ctx));
  return 0;
}
