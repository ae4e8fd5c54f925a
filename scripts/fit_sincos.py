"""Weighted least-squares fits of the PLL's sine / cosine kernels on
|r| <= pi/4 (+ slack) with one term fewer than fdlibm's, for
csrc/pll_fast.hpp (the certificate needs ~2^-46, fdlibm gives 2^-58):
  sin r = r + r z S(z),            z = r^2, S of degree 4
  cos r = 1 - z/2 + z^2 C(z),      C of degree 4
prints each max relative error and the coefficients as hex doubles.
Needs mpmath."""
import mpmath as mp
import numpy as np

mp.mp.dps = 40
ZMAX = (mp.pi / 4 * (1 + mp.mpf(2) ** -20)) ** 2
N = 600
zs = [ZMAX * (1 - mp.cos(mp.pi * (k + 0.5) / N)) / 2 for k in range(N)]


def fit(d, target, weight):
    A = mp.matrix(N, d + 1)
    b = mp.matrix(N, 1)
    for i, z in enumerate(zs):
        w = weight(z)
        for j in range(d + 1):
            A[i, j] = w * z ** j
        b[i] = w * target(z)
    c = mp.lu_solve(A.T * A, A.T * b)
    return [float(c[j]) for j in range(d + 1)]


def poly(cs, z):
    P = mp.mpf(0)
    for cj in reversed(cs):
        P = P * z + mp.mpf(cj)
    return P


# sin: (sin r - r) / (r z); relative error of r + r z S weighted by r z / sin r
S = fit(4, lambda z: (mp.sin(mp.sqrt(z)) - mp.sqrt(z)) / (mp.sqrt(z) * z),
        lambda z: mp.sqrt(z) * z / mp.sin(mp.sqrt(z)))
# cos: (cos r - 1 + z/2) / z^2, weighted by z^2 / cos r
C = fit(4, lambda z: (mp.cos(mp.sqrt(z)) - 1 + z / 2) / z ** 2, lambda z: z ** 2 / mp.cos(mp.sqrt(z)))
ms = mc = 0
for zf in np.linspace(0, float(ZMAX), 20001)[1:]:
    z = mp.mpf(zf)
    r = mp.sqrt(z)
    ms = max(ms, abs((r + r * z * poly(S, z)) / mp.sin(r) - 1))
    mc = max(mc, abs((1 - z / 2 + z * z * poly(C, z)) / mp.cos(r) - 1))
print("sin max rel err 2^%.2f, cos max rel err 2^%.2f" % (float(mp.log(ms, 2)), float(mp.log(mc, 2))))
print("S:", ", ".join(x.hex() for x in S))
print("C:", ", ".join(x.hex() for x in C))
