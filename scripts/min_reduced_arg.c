// Exhaustive search over every float x in [0.78, 2^26): the smallest reduced
// argument |x - k pi/2| of the PLL fast path's Cody-Waite reduction
// (csrc/pll_fast.hpp), and whether a third pi/2 term would change any result.
// Build: gcc -O2 scripts/min_reduced_arg.c -lm
#include <math.h>
#include <stdio.h>
#include <stdint.h>
#include <string.h>
int main(void) {
  const double P1 = 0x1.921fb54442d18p+0, P2 = 0x1.1a62633145c07p-54, P3 = -0x1.f1976b7ed8fbcp-110;
  float x = 0.78f; uint32_t b; memcpy(&b, &x, 4);
  double minr = 1, minrx = 0, maxdrop = 0; 
  for (; ; ++b) {
    float f; memcpy(&f, &b, 4);
    if (f >= 0x1p26f) break;
    double xd = f;
    double kd = rint(xd * 0x1.45f306dc9c883p-1);
    double r1 = fma(-kd, P1, xd), r2 = fma(-kd, P2, r1), r = fma(-kd, P3, r2);
    double ar = fabs(r);
    if (ar < minr) { minr = ar; minrx = xd; }
    double rel = fabs(r - r2) / ar;  // what dropping the P3 term would cost
    if (rel > maxdrop) maxdrop = rel;
  }
  printf("min |r| = %a = 2^%.2f at x = %a; max rel effect of P3 term 2^%.2f\n", minr, log2(minr), minrx, log2(maxdrop));
  return 0;
}
