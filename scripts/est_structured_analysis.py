"""Why the EST 3 window cannot hold on bench.structured_est_probe's RDM, on
the CPU with numpy: d_ab = u_a + u_b + 0.05 noise, u ~ Exp(1)^2, N = 10k, subsets of the
RandomState(42) choice(N, 0.9 N) stream. For each subset (lane) the included-pair count
before A position p is compared with the wave-uniform estimate M'/M p (EST 3) and with
per-lane fits of it: low-degree polynomials and piecewise-linear knots, and a per-segment
wave-uniform centre (the lanes' midpoint). The window holds a lane's ranks only while its
count stays within +-2^14 of the estimate (doubled ranks, 2^16 wide).
Usage: python scripts/est_structured_analysis.py [n] [lanes]   (~2 min, ~6 GB at n = 10k)"""
import sys

import numpy as np

n = int(sys.argv[1]) if len(sys.argv) > 1 else 10000
lanes = int(sys.argv[2]) if len(sys.argv) > 2 else 64
rs = np.random.RandomState(7)
u = rs.exponential(1.0, n) ** 2
iu, ju = np.triu_indices(n, 1)
iu, ju = iu.astype(np.int32), ju.astype(np.int32)
v = (u[iu] + u[ju] + 0.05 * rs.rand(iu.size)).astype(np.float32)
o = np.argsort(v, kind="stable")
ia, ja = iu[o], ju[o]
del o, v, iu, ju
M = ia.size
k = int(0.9 * n)
Mp = k * (k - 1) // 2
r = np.random.RandomState(42)
step = 1 << 8
cps = np.arange(0, M, step)
C = np.empty((lanes, cps.size), np.int64)
for s in range(lanes):
    m = np.zeros(n, bool)
    m[r.choice(n, k, replace=False)] = True
    cs = np.cumsum(m[ia] & m[ja], dtype=np.int64)
    C[s] = np.concatenate([[0], cs])[cps]
dev = C - (Mp / M) * cps[None, :]
print(f"n={n} M={M} lanes={lanes}: window = +-{1 << 14} included pairs around the estimate")
print(f"max |count - wave-uniform linear estimate| = {np.abs(dev).max():.0f}")
print(f"max spread of the lanes' counts at one position = {(C.max(0) - C.min(0)).max()}")
x = 2.0 * cps / M - 1.0
for deg in (1, 3, 5, 8, 12):
    res = max(np.abs(d - np.polynomial.chebyshev.chebval(x, np.polynomial.chebyshev.chebfit(x, d, deg))).max()
              for d in dev)
    print(f"per-lane Chebyshev fit, degree {deg:2d}: max residual {res:.0f}")
for K in (32, 64, 128, 256):
    kn = np.linspace(0, cps.size - 1, K + 1).astype(int)
    res = max(np.abs(d - np.interp(np.arange(cps.size), kn, d[kn])).max() for d in dev)
    print(f"per-lane piecewise-linear, {K:3d} knots: max residual {res:.0f}")
mid = (C.max(0) + C.min(0)) / 2.0
print(f"wave-uniform centre per position (the best any lane-shared window can do): "
      f"max |count - centre| {np.abs(C - mid[None, :]).max():.0f}")
