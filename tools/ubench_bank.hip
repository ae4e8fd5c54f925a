// VGPR bank micro-benchmark (gfx950): cycles per wave-instruction per SIMD
// for v_add_f32 / v_mul_f32 whose two VGPR sources sit in the same register
// bank (index mod 4) or in different banks, W waves per SIMD, every CU busy.
// Destinations rotate over 8 registers, so no instruction depends on the one
// before it.  Build: python3 scripts/gen_ubench_scan.py && hipcc --offload-arch=gfx950 -O3 -Itools tools/ubench_bank.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#include "ubench_bank_scan.h"

#define CLOB "v32", "v33", "v34", "v35", "v36", "v37", "v38", "v39", "v40", "v41", "v42", "v43", "v44", "v45", "v46", "v47", \
             "v48", "v49", "v50", "v51", "v52", "v53", "v54", "v55"

// 8 independent instructions; sources v40..v55, destinations v32..v39
#define SAME8(OP)                        \
  OP " v32, v40, v44\n\t" OP " v33, v41, v45\n\t" OP " v34, v42, v46\n\t" OP " v35, v43, v47\n\t" \
  OP " v36, v48, v52\n\t" OP " v37, v49, v53\n\t" OP " v38, v50, v54\n\t" OP " v39, v51, v55\n\t"
#define DIFF8(OP)                        \
  OP " v32, v40, v45\n\t" OP " v33, v41, v46\n\t" OP " v34, v42, v47\n\t" OP " v35, v43, v44\n\t" \
  OP " v36, v48, v53\n\t" OP " v37, v49, v54\n\t" OP " v38, v50, v55\n\t" OP " v39, v51, v52\n\t"
// the FIR/resampler MAC: product into a temporary, then the sum with the
// accumulator in the same bank as the temporary (as the compiler allocated it
// in resample_lp) or in a different one
#define MACSAME                                                                                        \
  "v_mul_f32 v40, v44, v48\n\tv_add_f32 v32, v32, v40\n\tv_mul_f32 v41, v45, v49\n\tv_add_f32 v33, v33, v41\n\t" \
  "v_mul_f32 v42, v46, v50\n\tv_add_f32 v34, v34, v42\n\tv_mul_f32 v43, v47, v51\n\tv_add_f32 v35, v35, v43\n\t"
#define MACDIFF                                                                                        \
  "v_mul_f32 v41, v44, v49\n\tv_add_f32 v32, v32, v41\n\tv_mul_f32 v42, v45, v50\n\tv_add_f32 v33, v33, v42\n\t" \
  "v_mul_f32 v43, v46, v51\n\tv_add_f32 v34, v34, v43\n\tv_mul_f32 v40, v47, v48\n\tv_add_f32 v35, v35, v40\n\t"

template <int OP>
__global__ __launch_bounds__(512) void bank(float* out, int iters) {
  asm volatile(
      "v_mov_b32 v40, 1.0\n\tv_mov_b32 v41, 1.0\n\tv_mov_b32 v42, 1.0\n\tv_mov_b32 v43, 1.0\n\t"
      "v_mov_b32 v44, 1.0\n\tv_mov_b32 v45, 1.0\n\tv_mov_b32 v46, 1.0\n\tv_mov_b32 v47, 1.0\n\t"
      "v_mov_b32 v48, 1.0\n\tv_mov_b32 v49, 1.0\n\tv_mov_b32 v50, 1.0\n\tv_mov_b32 v51, 1.0\n\t"
      "v_mov_b32 v52, 1.0\n\tv_mov_b32 v53, 1.0\n\tv_mov_b32 v54, 1.0\n\tv_mov_b32 v55, 1.0\n\t"
      "v_mov_b32 v32, 0\n\tv_mov_b32 v33, 0\n\tv_mov_b32 v34, 0\n\tv_mov_b32 v35, 0" ::: CLOB);
  for (int i = 0; i < iters; ++i) {
    if constexpr (OP == 0) asm volatile(SAME8("v_add_f32") SAME8("v_add_f32") SAME8("v_add_f32") SAME8("v_add_f32") ::: CLOB);
    if constexpr (OP == 1) asm volatile(DIFF8("v_add_f32") DIFF8("v_add_f32") DIFF8("v_add_f32") DIFF8("v_add_f32") ::: CLOB);
    if constexpr (OP == 2) asm volatile(SAME8("v_mul_f32") SAME8("v_mul_f32") SAME8("v_mul_f32") SAME8("v_mul_f32") ::: CLOB);
    if constexpr (OP == 3) asm volatile(DIFF8("v_mul_f32") DIFF8("v_mul_f32") DIFF8("v_mul_f32") DIFF8("v_mul_f32") ::: CLOB);
    if constexpr (OP == 4) asm volatile(MACSAME MACSAME MACSAME MACSAME ::: CLOB);
    if constexpr (OP == 5) asm volatile(MACDIFF MACDIFF MACDIFF MACDIFF ::: CLOB);
    // the same MACs as straight-line code of 8 KB / 32 KB per loop trip (a
    // fully unrolled scan's footprint in the instruction cache)
    if constexpr (OP == 6) asm volatile(".rept 256\n\t" MACDIFF ".endr\n\t" ::: CLOB);
    if constexpr (OP == 7) asm volatile(".rept 1024\n\t" MACDIFF ".endr\n\t" ::: CLOB);
    // resample_lp's register pattern: 128 tap registers, 7 chains (ubench_bank_scan.h)
    if constexpr (OP == 8) asm volatile(".rept 4\n\t" SCAN_BODY ".endr\n\t" ::: SCAN_CLOB);
    if constexpr (OP == 9) asm volatile(".rept 4\n\t" SCAN_BODY_B ".endr\n\t" ::: SCAN_CLOB);
    if constexpr (OP == 10) asm volatile(".rept 4\n\t" SCAN_BODY_C ".endr\n\t" ::: SCAN_CLOB);
    if constexpr (OP == 11) asm volatile(".rept 4\n\t" SCAN_BODY_D ".endr\n\t" ::: SCAN_CLOB);
  }
  float r;
  asm volatile("v_mov_b32 %0, v32" : "=v"(r)::CLOB);
  out[blockIdx.x * 256 + threadIdx.x] = r;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 64 << 20);
  int ncu = 0, clk = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  printf("CUs %d, clock %d kHz\n", ncu, clk);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[] = {"v_add_f32 same-bank srcs", "v_add_f32 diff-bank srcs", "v_mul_f32 same-bank srcs",
                         "v_mul_f32 diff-bank srcs", "mul+add, sum srcs same bank", "mul+add, sum srcs diff bank",
                         "mul+add, 8 KB loop body", "mul+add, 32 KB loop body",
                         "resample scan, 128 tap regs", "scan, one product reg", "scan, products then sums",
                         "scan, product over its input"};
  for (int op = 0; op < 12; ++op) {
    const int per_iter = op == 6 ? 2048 : op == 7 ? 8192 : op >= 8 ? 4 * SCAN_N : 32;  // instructions per loop trip
    const int iters = 128000 / per_iter;
    for (int w : {1, 2, 4, 8}) {  // waves per SIMD (256-thread WGs = 1 wave per SIMD each)
      const int grid = ncu * w;
      auto launch = [&] {
        switch (op) {
          case 0: hipLaunchKernelGGL(bank<0>, dim3(grid), dim3(256), 0, 0, out, iters); break;
          case 1: hipLaunchKernelGGL(bank<1>, dim3(grid), dim3(256), 0, 0, out, iters); break;
          case 2: hipLaunchKernelGGL(bank<2>, dim3(grid), dim3(256), 0, 0, out, iters); break;
          case 3: hipLaunchKernelGGL(bank<3>, dim3(grid), dim3(256), 0, 0, out, iters); break;
          case 4: hipLaunchKernelGGL(bank<4>, dim3(grid), dim3(256), 0, 0, out, iters); break;
          case 5: hipLaunchKernelGGL(bank<5>, dim3(grid), dim3(256), 0, 0, out, iters); break;
          case 6: hipLaunchKernelGGL(bank<6>, dim3(grid), dim3(256), 0, 0, out, iters); break;
          case 7: hipLaunchKernelGGL(bank<7>, dim3(grid), dim3(256), 0, 0, out, iters); break;
          case 8: hipLaunchKernelGGL(bank<8>, dim3(grid), dim3(256), 0, 0, out, iters); break;
          case 9: hipLaunchKernelGGL(bank<9>, dim3(grid), dim3(256), 0, 0, out, iters); break;
          case 10: hipLaunchKernelGGL(bank<10>, dim3(grid), dim3(256), 0, 0, out, iters); break;
          case 11: hipLaunchKernelGGL(bank<11>, dim3(grid), dim3(256), 0, 0, out, iters); break;
        }
      };
      launch();
      (void)hipEventRecord(e0);
      for (int r = 0; r < 5; ++r) launch();
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      ms /= 5;
      const double inst = (double)iters * per_iter;  // per wave
      const double per_simd = inst * w / (ms * 1e-3);
      printf("%-30s W=%d  %8.3f ms  %5.2f cyc/instr/SIMD @%.2f GHz\n", names[op], w, ms, clk * 1e3 / per_simd,
             clk / 1e6);
      fflush(stdout);
    }
  }
  // resample_lp's workgroup shape: one workgroup of 7 (or 8) waves per CU, so
  // three SIMDs hold 2 waves and one holds 1 (or all hold 2); optionally a
  // workgroup barrier every 1,792 instructions (one per 'item')
  for (int nw : {7, 8}) {
    const int iters = 128000 / (4 * SCAN_N) * 4;
    hipLaunchKernelGGL(bank<8>, dim3(ncu), dim3(64 * nw), 0, 0, out, iters);
    (void)hipEventRecord(e0);
    for (int r = 0; r < 5; ++r) hipLaunchKernelGGL(bank<8>, dim3(ncu), dim3(64 * nw), 0, 0, out, iters);
    (void)hipEventRecord(e1);
    (void)hipEventSynchronize(e1);
    float ms;
    (void)hipEventElapsedTime(&ms, e0, e1);
    ms /= 5;
    const double per_busiest = (double)iters * 4 * SCAN_N * 2 / (ms * 1e-3);  // 2 waves on the busiest SIMD
    printf("scan, %d-wave workgroup/CU     %8.3f ms  %5.2f cyc/instr on a 2-wave SIMD @%.2f GHz\n", nw, ms,
           clk * 1e3 / per_busiest, clk / 1e6);
    fflush(stdout);
  }
  // sustained: the scan-shaped body at 2 waves/SIMD for ~0.5 s; a falling
  // rate means the clock drops under sustained VALU load
  {
    const int w = 2, grid = ncu * w, iters = 128000 / (4 * SCAN_N) * 4;
    float ms_first = 0, ms_last = 0;
    for (int r = 0; r < 400; ++r) {
      (void)hipEventRecord(e0);
      hipLaunchKernelGGL(bank<8>, dim3(grid), dim3(256), 0, 0, out, iters);
      (void)hipEventRecord(e1);
      (void)hipEventSynchronize(e1);
      float ms;
      (void)hipEventElapsedTime(&ms, e0, e1);
      if (r == 1) ms_first = ms;
      if (r == 399) ms_last = ms;
      if (r % 50 == 0 || r == 399) {
        const double per_simd = (double)iters * 4 * SCAN_N * w / (ms * 1e-3);
        printf("sustained scan W=2 launch %3d  %8.3f ms  %5.2f cyc/instr/SIMD @%.2f GHz\n", r, ms,
               clk * 1e3 / per_simd, clk / 1e6);
        fflush(stdout);
      }
    }
    printf("sustained: last/first = %.3f\n", ms_last / ms_first);
  }
  return 0;
}
