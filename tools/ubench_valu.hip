// Microbenchmark: issue rate of v_mul_f32 / v_add_f32 vs v_pk_mul_f32 /
// v_pk_add_f32 on gfx950 (is packed fp32 a 2x throughput lever?).
#include <hip/hip_runtime.h>
#include <cstdio>

typedef float float2v __attribute__((ext_vector_type(2)));

template <int MODE>
__global__ __launch_bounds__(256) void k(float* out, float a, float b, int iters) {
  float2v x0 = {a, b}, x1 = {b, a}, x2 = {a + 1, b}, x3 = {a, b + 1};
  float2v x4 = x0 * 0.5f, x5 = x1 * 0.5f, x6 = x2 * 0.5f, x7 = x3 * 0.5f;
  const float2v m = {1.0000001f, 0.9999999f};
  for (int i = 0; i < iters; ++i) {
#pragma unroll
    for (int u = 0; u < 8; ++u) {
      if (MODE == 0) {  // scalar mul + add, 8 independent chains per component
        asm volatile(
            "v_mul_f32 %0, %0, %8\n v_mul_f32 %1, %1, %8\n v_mul_f32 %2, %2, %8\n v_mul_f32 %3, %3, %8\n"
            "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8\n"
            : "+v"(x0.x), "+v"(x1.x), "+v"(x2.x), "+v"(x3.x), "+v"(x4.x), "+v"(x5.x), "+v"(x6.x), "+v"(x7.x)
            : "v"(m.x));
      } else if (MODE == 2) {  // scalar mul with a row_newbcast DPP operand + plain add
        asm volatile(
            "v_mul_f32_dpp %0, %8, %0 row_newbcast:1 row_mask:0xf bank_mask:0xf\n"
            "v_mul_f32_dpp %1, %8, %1 row_newbcast:2 row_mask:0xf bank_mask:0xf\n"
            "v_mul_f32_dpp %2, %8, %2 row_newbcast:3 row_mask:0xf bank_mask:0xf\n"
            "v_mul_f32_dpp %3, %8, %3 row_newbcast:4 row_mask:0xf bank_mask:0xf\n"
            "v_add_f32 %4, %4, %8\n v_add_f32 %5, %5, %8\n v_add_f32 %6, %6, %8\n v_add_f32 %7, %7, %8\n"
            : "+v"(x0.x), "+v"(x1.x), "+v"(x2.x), "+v"(x3.x), "+v"(x4.x), "+v"(x5.x), "+v"(x6.x), "+v"(x7.x)
            : "v"(m.x));
      } else {  // packed: same number of instructions, two lanes of work each
        asm volatile(
            "v_pk_mul_f32 %0, %0, %8\n v_pk_mul_f32 %1, %1, %8\n v_pk_mul_f32 %2, %2, %8\n v_pk_mul_f32 %3, %3, %8\n"
            "v_pk_add_f32 %4, %4, %8\n v_pk_add_f32 %5, %5, %8\n v_pk_add_f32 %6, %6, %8\n v_pk_add_f32 %7, %7, %8\n"
            : "+v"(x0), "+v"(x1), "+v"(x2), "+v"(x3), "+v"(x4), "+v"(x5), "+v"(x6), "+v"(x7)
            : "v"(m));
      }
    }
  }
  float2v s = x0 + x1 + x2 + x3 + x4 + x5 + x6 + x7;
  out[blockIdx.x * 256 + threadIdx.x] = s.x + s.y;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 256 * 4096 * 4 * sizeof(float));
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const int iters = 4000;
  for (int blocks : {1024, 4096}) {
    for (int mode = 0; mode < 3; ++mode) {
      for (int rep = 0; rep < 2; ++rep) {
        (void)hipEventRecord(e0);
        if (mode == 0)
          hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, 1.0f, 2.0f, iters);
        else if (mode == 2)
          hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, 1.0f, 2.0f, iters);
        else
          hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, 1.0f, 2.0f, iters);
        (void)hipEventRecord(e1);
        (void)hipEventSynchronize(e1);
        float ms = 0;
        (void)hipEventElapsedTime(&ms, e0, e1);
        const double instr = (double)blocks * 4 /*waves*/ * iters * 8 * 8;  // wave-instructions
        const double lanes = instr * 64 * (mode == 1 ? 2 : 1);
        if (rep)
          printf("blocks %5d mode %s: %.3f ms, %.1f T wave-instr/s, %.1f T lane-ops/s\n", blocks,
                 mode == 1 ? "pk " : mode == 2 ? "dpp" : "f32", ms, instr / ms / 1e9, lanes / ms / 1e9);
      }
    }
  }
  return 0;
}
