"""Fit of the branch-free normal CDF used by the GELU / GELU' epilogues and the fused tower MLP (vv_kernels.h
phi_fast):
    h(x) = Phi(-|x|) = 0.5 erfc(|x| / sqrt 2) = 2^(u S(u) - 1),   u = min(|x|, UMAX)
    Phi(x) = x >= 0 ? 1 - h : h ;  GELU(x) = x Phi(x) = x >= 0 ? x - x h : x h
S is a polynomial of degree DEG fitted by iteratively reweighted least squares (towards minimax) on the error of
GELU relative to |x| (weight h u ln 2), then checked in float32 arithmetic (Horner fma chain, one fma for u S - 1,
exp2 rounded to float) against float64 on a dense grid. Prints the float32 coefficients (u^0 .. u^DEG).
Usage: python tools/fit_erf.py [DEG]"""
import sys

import numpy as np
from scipy.special import erfc

DEG = int(sys.argv[1]) if len(sys.argv) > 1 else 8
UMAX = 5.75
u = np.linspace(1e-6, UMAX, 200001)
hh = 0.5 * erfc(u / np.sqrt(2.0))
f = (np.log2(hh) + 1.0) / u                   # S(u)
w = hh * u * np.log(2.0) + 1e-300
x = 2 * u / UMAX - 1
V = np.polynomial.chebyshev.chebvander(x, DEG)
lw = np.ones_like(u)
for it in range(80):
    ww = w * np.sqrt(lw)
    c, *_ = np.linalg.lstsq(V * ww[:, None], f * ww, rcond=None)
    err = np.abs((V @ c - f) * w)
    lw = lw * (err / err.max() + 1e-3)
    lw /= lw.mean()
mono = np.polynomial.chebyshev.Chebyshev(c, domain=[0, UMAX]).convert(kind=np.polynomial.Polynomial).coef
m32 = mono.astype(np.float32)


def h32(xs):
    uu = np.minimum(np.abs(xs), np.float32(UMAX)).astype(np.float32).astype(np.float64)
    q = np.float64(m32[-1])
    for a in m32[-2::-1]:
        q = np.float32(q * uu + np.float64(a)).astype(np.float64)
    e = np.float32(uu * q - 1.0).astype(np.float64)
    return np.exp2(e).astype(np.float32).astype(np.float64)


xs = np.linspace(-9, 9, 3000001).astype(np.float32).astype(np.float64)
h = h32(xs)
phi = np.where(xs >= 0, np.float32(1.0) - h.astype(np.float32), h).astype(np.float64)
phir = 0.5 * erfc(-xs / np.sqrt(2.0))
g = np.where(xs >= 0, (xs - (xs * h).astype(np.float32)).astype(np.float32), (xs * h).astype(np.float32)).astype(np.float64)
gr = xs * phir
print("deg", DEG, "Phi max abs err %.3e" % np.abs(phi - phir).max(),
      "GELU max err / |x| %.3e" % (np.abs(g - gr) / np.maximum(np.abs(xs), 1e-30)).max())
pdf = np.exp(-0.5 * xs * xs) / np.sqrt(2 * np.pi)
pdf32 = np.exp2(np.float32(xs * xs * np.float32(-0.5 / np.log(2.0)) + np.float32(np.log2(1 / np.sqrt(2 * np.pi)))).astype(np.float64))
d = phi + (xs * pdf32).astype(np.float32)
dr = phir + xs * pdf
print("GELU' max abs err %.3e" % np.abs(d - dr).max())
print(", ".join("%.9ef" % v for v in m32))
