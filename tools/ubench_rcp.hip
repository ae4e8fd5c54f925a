// Accuracy of v_rcp_f64 (__builtin_amdgcn_rcp) on MI355X: max |1 - u*rcp(u)|
// over 2^24 arguments spread over [1, 2) and a few binades (the PLL's
// short-chain division, csrc/pll_fast.hpp, relies on it being <= 2^-20).
// Build: hipcc --offload-arch=gfx950 -O3 tools/ubench_rcp.hip -o tools/ubench_rcp
#include <hip/hip_runtime.h>

#include <cmath>
#include <cstdio>

__global__ void rcp_err(double* out, int n) {
  const int i = blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n) return;
  // mantissa sweep with a pseudo-random low part, exponent in [-60, 60]
  const unsigned long long h = (unsigned long long)i * 0x9E3779B97F4A7C15ull;
  const double m = 1.0 + (double)(h >> 11) * 0x1p-53;
  const double u = ldexp(m, (int)(i % 121) - 60);
  const double r = __builtin_amdgcn_rcp(u);
  out[i] = fabs(fma(-u, r, 1.0));
}

int main() {
  const int n = 1 << 24;
  double* d;
  (void)hipMalloc(&d, n * sizeof(double));
  hipLaunchKernelGGL(rcp_err, dim3(n / 256), dim3(256), 0, 0, d, n);
  double* h = new double[n];
  (void)hipMemcpy(h, d, n * sizeof(double), hipMemcpyDeviceToHost);
  double mx = 0;
  for (int i = 0; i < n; ++i) mx = h[i] > mx ? h[i] : mx;
  printf("v_rcp_f64: max |1 - u*rcp(u)| = %.3e = 2^%.2f over %d arguments\n", mx, std::log2(mx), n);
  return 0;
}
