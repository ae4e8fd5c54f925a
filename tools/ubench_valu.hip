// VALU issue rates on MI355X (gfx950): cycles per wave-instruction per SIMD
// for the FIR's candidate instruction forms, with W waves per SIMD, every CU
// busy.  Each wave runs NCH independent chains (no dependency stall).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_valu.hip
#include <hip/hip_runtime.h>

#include <cstdio>

#define REP8(x) x x x x x x x x

template <int OP>
__global__ __launch_bounds__(256) void valu(float* out, int iters, float s) {
  // 8 independent 64-bit register pairs
  typedef float f2 __attribute__((ext_vector_type(2)));
  f2 a0 = {1.f + threadIdx.x, 2.f}, a1 = a0 + 1.f, a2 = a0 + 2.f, a3 = a0 + 3.f;
  f2 a4 = a0 + 4.f, a5 = a0 + 5.f, a6 = a0 + 6.f, a7 = a0 + 7.f;
  const f2 b = {s, s * 0.5f};
  const f2 c = {s * 0.25f + threadIdx.x, s * 0.125f};
  for (int i = 0; i < iters; ++i) {
    if constexpr (OP == 0) {  // v_add_f32 v, v, v  (both halves: 16 instr per 8 pairs)
#define A(V) asm volatile("v_add_f32 %0, %2, %0\n\tv_add_f32 %1, %2, %1" : "+v"(V.x), "+v"(V.y) : "v"(b.y));
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 1) {  // v_mul_f32 v, s, v
#define A(V) asm volatile("v_mul_f32 %0, %2, %0\n\tv_mul_f32 %1, %2, %1" : "+v"(V.x), "+v"(V.y) : "s"(s));
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 2) {  // v_fma_f32
#define A(V) asm volatile("v_fma_f32 %0, %2, %0, %3\n\tv_fma_f32 %1, %2, %1, %3" : "+v"(V.x), "+v"(V.y) : "s"(s), "v"(b.y));
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 3) {  // v_pk_add_f32 (one instr per pair: 8 instr per 8 pairs, x2 for parity)
#define A(V) asm volatile("v_pk_add_f32 %0, %1, %0\n\tv_pk_add_f32 %0, %1, %0" : "+v"(V) : "v"(b));
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 4) {  // v_pk_mul_f32 v, s[pair] (broadcast lo), v
#define A(V) asm volatile("v_pk_mul_f32 %0, %1, %0 op_sel_hi:[0,1]\n\tv_pk_mul_f32 %0, %1, %0 op_sel_hi:[0,1]" : "+v"(V) : "s"(b));
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 5) {  // v_pk_fma_f32
#define A(V) asm volatile("v_pk_fma_f32 %0, %1, %0, %1\n\tv_pk_fma_f32 %0, %1, %0, %1" : "+v"(V) : "v"(b));
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 6) {  // alternating pk_mul (s) / pk_add: the packed exact FIR step
#define A(V) { f2 t; asm volatile("v_pk_mul_f32 %1, %2, %3 op_sel_hi:[0,1]\n\tv_pk_add_f32 %0, %1, %0" : "+v"(V), "=&v"(t) : "s"(b), "v"(c)); }
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 7) {  // alternating v_mul (s) / v_add: the unpacked exact FIR step
#define A(V) { float t; asm volatile("v_mul_f32 %1, %2, %3\n\tv_add_f32 %0, %1, %0" : "+v"(V.x), "=&v"(t) : "s"(s), "v"(c.x)); }
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 8) {  // v_fma_f32 v, v, v, v (VOP3, no SGPR)
#define A(V) asm volatile("v_fma_f32 %0, %2, %0, %3\n\tv_fma_f32 %1, %2, %1, %3" : "+v"(V.x), "+v"(V.y) : "v"(c.x), "v"(b.y));
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 9) {  // v_mul_f32 v, v, v
#define A(V) asm volatile("v_mul_f32 %0, %2, %0\n\tv_mul_f32 %1, %2, %1" : "+v"(V.x), "+v"(V.y) : "v"(c.x));
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 10) {  // v_fmac_f32 v, v, v (VOP2)
#define A(V) asm volatile("v_fmac_f32 %0, %2, %3\n\tv_fmac_f32 %1, %2, %3" : "+v"(V.x), "+v"(V.y) : "v"(c.x), "v"(c.y));
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 11) {  // v_fmac_f32 v, s, v (VOP2, SGPR src0)
#define A(V) asm volatile("v_fmac_f32 %0, %2, %3\n\tv_fmac_f32 %1, %2, %3" : "+v"(V.x), "+v"(V.y) : "s"(s), "v"(c.y));
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 12) {  // v_add_f32 v, s, v
#define A(V) asm volatile("v_add_f32 %0, %2, %0\n\tv_add_f32 %1, %2, %1" : "+v"(V.x), "+v"(V.y) : "s"(s));
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 13) {  // mul v,v,v + add: the exact FIR step with VGPR taps
#define A(V) { float t; asm volatile("v_mul_f32 %1, %2, %3\n\tv_add_f32 %0, %1, %0" : "+v"(V.x), "=&v"(t) : "v"(c.y), "v"(c.x)); }
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 14) {  // mul (s) + add, the add's chain dependent on the mul (as the FIR)
#define A(V) { float t; asm volatile("v_mul_f32 %1, %2, %3\n\tv_add_f32 %0, %1, %0" : "+v"(V.x), "=&v"(t) : "s"(s), "v"(V.y)); }
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 15) {  // v_mul_f32_dpp row_newbcast (tap broadcast from a 16-lane row)
#define A(V) asm volatile("v_mul_f32_dpp %0, %2, %0 row_newbcast:3 row_mask:0xf bank_mask:0xf\n\tv_mul_f32_dpp %1, %2, %1 row_newbcast:5 row_mask:0xf bank_mask:0xf" : "+v"(V.x), "+v"(V.y) : "v"(c.y));
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 16) {  // dpp mul + add, the add's chain dependent on the mul (resample_sw's MAC)
#define A(V) { float t; asm volatile("v_mul_f32_dpp %1, %2, %3 row_newbcast:7 row_mask:0xf bank_mask:0xf\n\tv_add_f32 %0, %1, %0" : "+v"(V.x), "=&v"(t) : "v"(c.y), "v"(V.y)); }
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 17) {  // v_fma_mix_f32 v, s, v(f16 lo), v(-0): an exact product from an f16 operand
#define A(V) asm volatile("v_fma_mix_f32 %0, %2, %0, %3 op_sel_hi:[0,1,0]\n\tv_fma_mix_f32 %1, %2, %1, %3 op_sel:[0,1,0] op_sel_hi:[0,1,0]" : "+v"(V.x), "+v"(V.y) : "s"(s), "v"(-0.0f));
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    } else if constexpr (OP == 18) {  // fma_mix product (s, f16) + add, the add's chain dependent (the f16-staged FIR step)
#define A(V) { float t; asm volatile("v_fma_mix_f32 %1, %2, %3, %4 op_sel_hi:[0,1,0]\n\tv_add_f32 %0, %1, %0" : "+v"(V.x), "=&v"(t) : "s"(s), "v"(V.y), "v"(-0.0f)); }
      REP8(A(a0) A(a1) A(a2) A(a3) A(a4) A(a5) A(a6) A(a7))
#undef A
    }
  }
  const f2 t = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7;
  out[blockIdx.x * 256 + threadIdx.x] = t.x + t.y;
}

int main() {
  float* out;
  (void)hipMalloc(&out, 64 << 20);
  int ncu = 0;
  (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, 0);
  int clk = 0;
  (void)hipDeviceGetAttribute(&clk, hipDeviceAttributeClockRate, 0);
  printf("CUs %d, clock %d kHz\n", ncu, clk);
  hipEvent_t e0, e1;
  (void)hipEventCreate(&e0);
  (void)hipEventCreate(&e1);
  const char* names[] = {"v_add_f32", "v_mul_f32 (s)", "v_fma_f32", "v_pk_add_f32", "v_pk_mul_f32 (s bcast)",
                         "v_pk_fma_f32", "pk_mul+pk_add", "mul+add",
                         "v_fma_f32 vvv", "v_mul_f32 vv", "v_fmac_f32 vv", "v_fmac_f32 sv", "v_add_f32 sv",
                         "mul vv + add", "mul(s)+add (dep)", "v_mul_f32_dpp bcast", "mul_dpp+add (dep)",
                         "v_fma_mix_f32 (s, f16, -0)", "fma_mix(s,f16)+add (dep)"};
  const int iters = 2000;
  for (int op = 0; op < 19; ++op) {
    for (int w : {1, 2, 3, 4, 8}) {  // waves per SIMD (256-thread WGs = 1 wave per SIMD each)
      const int grid = ncu * w;
      auto launch = [&] {
        switch (op) {
          case 0: hipLaunchKernelGGL(valu<0>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 1: hipLaunchKernelGGL(valu<1>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 2: hipLaunchKernelGGL(valu<2>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 3: hipLaunchKernelGGL(valu<3>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 4: hipLaunchKernelGGL(valu<4>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 5: hipLaunchKernelGGL(valu<5>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 6: hipLaunchKernelGGL(valu<6>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 7: hipLaunchKernelGGL(valu<7>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 8: hipLaunchKernelGGL(valu<8>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 9: hipLaunchKernelGGL(valu<9>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 10: hipLaunchKernelGGL(valu<10>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 11: hipLaunchKernelGGL(valu<11>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 12: hipLaunchKernelGGL(valu<12>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 13: hipLaunchKernelGGL(valu<13>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 14: hipLaunchKernelGGL(valu<14>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 15: hipLaunchKernelGGL(valu<15>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 16: hipLaunchKernelGGL(valu<16>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 17: hipLaunchKernelGGL(valu<17>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
          case 18: hipLaunchKernelGGL(valu<18>, dim3(grid), dim3(256), 0, 0, out, iters, 1.0001f); break;
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
      // instructions per wave: iters * 8 (REP8) * 8 pairs * 2
      const double inst = (double)iters * 8 * 8 * 2;
      const double wave_inst_per_s = inst * grid * 4 / (ms * 1e-3);
      const double per_simd = wave_inst_per_s / (ncu * 4);
      printf("%-24s W=%d  %8.3f ms  %7.3f T wave-instr/s  %5.2f cyc/instr/SIMD @%.2f GHz\n", names[op], w, ms,
             wave_inst_per_s / 1e12, clk * 1e3 / per_simd, clk / 1e6);
      fflush(stdout);
    }
  }
  return 0;
}
