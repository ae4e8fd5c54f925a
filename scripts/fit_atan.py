"""Weighted least-squares fit of atan(t) = t + t*z*P(z), z = t^2, on [0, 1]
(P of degree 15) for csrc/pll_fast.hpp; prints the max relative error and
the coefficients as hex doubles.  Needs mpmath."""
import mpmath as mp, numpy as np
mp.mp.dps = 40
def target(z):
    t = mp.sqrt(z)
    return (mp.atan(t) - t)/(t*z)
d = 15; N = 600
zs = [ (1 - mp.cos(mp.pi*(k+0.5)/N))/2 for k in range(N)]
A = mp.matrix(N, d+1); b = mp.matrix(N,1)
for i,z in enumerate(zs):
    t = mp.sqrt(z); w = t*z/mp.atan(t)
    for j in range(d+1): A[i,j] = w * z**j
    b[i] = w*target(z)
c = mp.lu_solve(A.T*A, A.T*b)
cs = [float(c[j]) for j in range(d+1)]
m = 0
for z in np.linspace(0,1,20001)[1:]:
    z = mp.mpf(z); t = mp.sqrt(z); P = mp.mpf(0)
    for cj in reversed(cs): P = P*z + mp.mpf(cj)
    m = max(m, abs((t + t*z*P)/mp.atan(t) - 1))
print("max rel err 2^%.2f" % float(mp.log(m,2)))
print(",\n".join(x.hex() for x in cs))
