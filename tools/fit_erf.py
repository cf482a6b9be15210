"""Fit the branch-free fp32 erf/tanh polynomials used by bcnf_device.h and verify them in emulated fp32
(fma = fp64 product-sum rounded once to fp32). Writes nothing; prints coefficients and max errors."""
import numpy as np
from scipy.special import erf, erfc

f32 = np.float32


def fma(a, b, c):
    return f32(np.float64(a) * np.float64(b) + np.float64(c))


def fit_poly(x, y, deg, w=None):
    # least squares in fp64 on the given nodes (Chebyshev-distributed), returns highest-first coeffs
    V = np.vander(x, deg + 1)
    if w is not None:
        V = V * w[:, None]
        y = y * w
    c, *_ = np.linalg.lstsq(V, y, rcond=None)
    return c


def minimax_refine(x, y, deg, iters=30):
    w = np.ones_like(x)
    for _ in range(iters):
        c = fit_poly(x, y, deg, w)
        err = np.abs(np.polyval(c, x) - y)
        w = w * (1 + 0.5 * err / err.max())
        w /= w.mean()
    return c


# region A: |x| < XA: erf(x) = x * P(s), s = x^2
XA = 0.921875
n = 4000
xs = np.cos(np.pi * (np.arange(n) + 0.5) / n) * XA
xs = xs[xs != 0]
s = xs * xs
ya = erf(xs) / xs
cA = minimax_refine(s, ya, 6)
# region B: XA <= t < 3.9375: erf(t) = 1 - exp(-t * Q(t))   (t * Q(t) = -log(erfc(t)))
XB = 3.9375
tb = XA + (XB - XA) * 0.5 * (1 - np.cos(np.pi * (np.arange(n) + 0.5) / n))
yb = -np.log(erfc(tb)) / tb
cB = minimax_refine(tb, yb, 7)
cA32 = [f32(c) for c in cA]
cB32 = [f32(c) for c in cB]
print("A (s-poly, highest first):", ", ".join(f"{float(c):.9e}f" for c in cA32))
print("B (t-poly, highest first):", ", ".join(f"{float(c):.9e}f" for c in cB32))


def exp32(x):
    return f32(np.exp(np.float64(x)))   # device expf is ~1 ulp; treat as correctly rounded


def erf32(a):
    a = f32(a)
    t = f32(abs(a))
    sq = f32(a * a)
    r = cA32[0]
    for c in cA32[1:]:
        r = fma(r, sq, c)
    rA = fma(r, a, f32(0.0)) if False else f32(np.float64(r) * np.float64(a))
    q = cB32[0]
    for c in cB32[1:]:
        q = fma(q, t, c)
    q = f32(np.float64(q) * np.float64(t))
    rB = f32(1.0) - exp32(-q)
    rB = f32(np.copysign(rB, a))
    if t >= f32(XB):
        rB = f32(np.copysign(1.0, a))
    return rA if t < f32(XA) else rB


grid = np.concatenate([np.linspace(-6, 6, 200001), np.geomspace(1e-8, 6, 20001), -np.geomspace(1e-8, 6, 20001)])
grid = grid.astype(np.float32)
worst_ulp, worst_abs = 0.0, 0.0
for x in grid:
    got = erf32(x)
    ref = erf(np.float64(x))
    ulp = np.spacing(f32(abs(ref))) if ref != 0 else np.float32(1e-45)
    e = abs(np.float64(got) - ref)
    worst_abs = max(worst_abs, e)
    worst_ulp = max(worst_ulp, e / ulp)
print(f"erf: max abs err {worst_abs:.3e}, max ulp {worst_ulp:.2f}")


# tanh: |x| < XT: x + x*s*P(s);  else sign(x) * (1 - 2 / (exp(2|x|) + 1))
XT = 0.625
xt = np.cos(np.pi * (np.arange(n) + 0.5) / n) * XT
xt = xt[np.abs(xt) > 1e-6]
st = xt * xt
yt = (np.tanh(xt) - xt) / (xt * st)
cT = minimax_refine(st, yt, 5)
cT32 = [f32(c) for c in cT]
print("T (s-poly, highest first):", ", ".join(f"{float(c):.9e}f" for c in cT32))


def tanh32(a):
    a = f32(a)
    t = f32(abs(a))
    sq = f32(a * a)
    p = cT32[0]
    for c in cT32[1:]:
        p = fma(p, sq, c)
    rs = fma(f32(np.float64(a) * np.float64(sq)), p, a)
    e = exp32(f32(2.0) * t)
    rl = f32(1.0) - f32(f32(2.0) * f32(1.0 / np.float64(f32(e + f32(1.0)))))
    rl = f32(np.copysign(rl, a))
    return rs if t < f32(XT) else rl


worst_ulp, worst_abs = 0.0, 0.0
for x in grid[::3]:
    got = tanh32(x)
    ref = np.tanh(np.float64(x))
    ulp = np.spacing(f32(abs(ref))) if ref != 0 else np.float32(1e-45)
    e = abs(np.float64(got) - ref)
    worst_abs = max(worst_abs, e)
    worst_ulp = max(worst_ulp, e / ulp)
print(f"tanh: max abs err {worst_abs:.3e}, max ulp {worst_ulp:.2f}")
