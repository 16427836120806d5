#!/usr/bin/env python3
"""Chebyshev series for the fused EI partials (csrc/mrbo_device.h ei_phi_Phi):
   g(t) = (1 + 2u) · erfcx(u),  u ≥ 0,  t = (u − K)/(u + K) ∈ [−1, 1),
computed at high precision with mpmath, converted to a power series in t (evaluated by
Horner/Estrin in fp64).  Prints the coefficients and the max relative error of the fp64
evaluation against mpmath over u ∈ [0, 27]."""
import sys
import mpmath as mp
mp.mp.dps = 60
K = mp.mpf(sys.argv[1]) if len(sys.argv) > 1 else mp.mpf(4)
NT = int(sys.argv[2]) if len(sys.argv) > 2 else 30

def g_of_t(t):
    if t >= 1:
        return 2 / mp.sqrt(mp.pi)
    u = K * (1 + t) / (1 - t)
    return (1 + 2 * u) * mp.exp(u * u) * mp.erfc(u)

# Chebyshev coefficients by Gauss-Chebyshev quadrature
M = 200
nodes = [mp.cos(mp.pi * (k + mp.mpf(1) / 2) / M) for k in range(M)]
vals = [g_of_t(x) for x in nodes]
c = []
for n in range(NT):
    s = mp.fsum(vals[k] * mp.cos(mp.pi * n * (k + mp.mpf(1) / 2) / M) for k in range(M))
    c.append(2 * s / M)
c[0] /= 2
# Chebyshev -> power basis (exact in mp)
import itertools
T = [[mp.mpf(1)], [mp.mpf(0), mp.mpf(1)]]
for n in range(2, NT):
    a = [mp.mpf(0)] + [2 * v for v in T[n - 1]]
    b = T[n - 2] + [mp.mpf(0)] * (len(a) - len(T[n - 2]))
    T.append([x - y for x, y in zip(a, b)])
p = [mp.mpf(0)] * NT
for n in range(NT):
    for i, v in enumerate(T[n]):
        p[i] += c[n] * v
print("K", K, "terms", NT, "last cheb coefs", [mp.nstr(abs(x), 3) for x in c[-4:]])
pf = [float(x) for x in p]

def horner(t):
    r = 0.0
    for a in reversed(pf):
        r = r * t + a
    return r

import math
worst = 0.0
for i in range(4000):
    u = 27.0 * (i / 3999.0) ** 2
    t = (u - float(K)) / (u + float(K))
    approx = horner(t) / (1 + 2 * u)
    exact = mp.exp(mp.mpf(u) ** 2) * mp.erfc(mp.mpf(u))
    worst = max(worst, abs((approx - exact) / exact))
print("max rel err (fp64 power-basis Horner)", worst)
if "--emit" in sys.argv:
    for a in pf:
        print(repr(a))
