"""Fit of chord_theta's polynomial (ompl_amd/csrc/knn_fast_impl.h): theta = 2 asin(c / 2) =
c (1 + x R(x)), x = c^2 / 4 in [0, 0.5].  Lawson-reweighted least squares for a minimax fit of
the error on theta; prints the coefficients (low order first) and the largest error in fp64 and
with fp32 Horner evaluation.  Run: python tools/fit_asin.py [degree]"""
import sys

import numpy as np

deg = int(sys.argv[1]) if len(sys.argv) > 1 else 5
cn = 0.25 * (1 - np.cos(np.linspace(0, np.pi, 4000))) + 1e-9
hn = np.sqrt(cn)
Rn = (np.arcsin(hn) / hn - 1) / cn
w = 2 * hn * cn                      # d(theta) = c x dR = 2 h x dR
A = np.vander(cn, deg + 1, increasing=True)
ww = np.ones_like(cn)
for _ in range(60):
    coef, *_ = np.linalg.lstsq(A * (w * np.sqrt(ww))[:, None], Rn * w * np.sqrt(ww), rcond=None)
    e = np.abs((A @ coef - Rn) * w)
    ww = ww * e / e.max() + 1e-12
    ww /= ww.sum()
coef32 = np.float32(coef)
xs = np.linspace(0, 0.5, 400001)
h = np.sqrt(xs)
th = 2 * np.arcsin(h)
print("coefficients (x^0 first):", [float(c) for c in coef32])
print("fp64 |error| on theta:", np.abs(2 * h * (1 + xs * np.polyval(coef[::-1], xs)) - th).max())
c32 = (2 * h).astype(np.float32)
x32 = (np.float32(0.25) * c32 * c32).astype(np.float32)
r = np.full_like(x32, coef32[-1])
for cc in coef32[-2::-1]:
    r = (r.astype(np.float64) * x32 + cc).astype(np.float32)   # fma: one rounding
t32 = (c32.astype(np.float64) * (x32 * r).astype(np.float32) + c32).astype(np.float32)
print("fp32 evaluation |error| on theta:", np.abs(t32 - 2 * np.arcsin(c32.astype(np.float64) / 2)).max())
assert (t32 >= c32).all(), "theta below the chord"
