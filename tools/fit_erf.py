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


# ---------------------------------------------------------------------------------------------------------------
# gelu_fit (bcnf_device.h gelu_tail, r02x): erfc(z) = t exp(-z^2) Q(t), t = 1 / (1 + p z), Q of degree 6, fitted
# with relative weights on z in [0, 7] (Chebyshev nodes in t), p scanned; then the fp32 evaluation as the kernel
# does it (p / sqrt2 on |x|, the 1/2 folded into Q, exp2 of -x^2 log2(e) / 2) against the fp64 GELU / GELU'.
def gelu_fit(deg=6, zmax=7.0, n=8000):
    from scipy.special import ndtr

    def fit(p):
        tmin = 1 / (1 + p * zmax)
        tt = (np.cos(np.pi * (np.arange(n) + 0.5) / n) * 0.5 + 0.5) * (1 - tmin) + tmin
        z = (1 / tt - 1) / p
        y = erfc(z) * np.exp(z * z) / tt
        w = np.ones_like(tt)
        for _ in range(60):
            c = fit_poly(tt, y, deg, w)
            err = np.abs(np.polyval(c, tt) - y) / y
            w = w * (1 + 0.5 * err / err.max())
            w /= w.mean()
        return c, err.max()

    e, p = min((fit(p)[1], p) for p in np.linspace(0.28, 0.40, 25))
    c, _ = fit(p)
    ps, C = f32(p / np.sqrt(2)), [f32(0.5 * v) for v in c]
    x = np.linspace(-12, 12, 2000001).astype(f32)
    t = f32(1) / fma(ps, np.abs(x), f32(1))
    q = np.full_like(x, C[0])
    for cc in C[1:]:
        q = fma(q, t, cc)
    ez = f32(np.exp2(np.float64(f32(f32(x * x) * f32(-0.5 * np.log2(np.e))))))
    h = f32(f32(t * q) * ez)
    cdf = np.where(x < 0, h, f32(1) - h)
    g, dg = f32(x * cdf), fma(x, f32(ez * f32(1 / np.sqrt(2 * np.pi))), cdf)
    xd = x.astype(np.float64)
    phi = ndtr(xd)
    print(f"gelu_fit: p = {p:.4f}, fit max rel {e:.2e}; fp32 |GELU err| {np.abs(g - xd * phi).max():.2e}, "
          f"|GELU' err| {np.abs(dg - (phi + xd * np.exp(-xd * xd / 2) / np.sqrt(2 * np.pi))).max():.2e}")
    print("  p / sqrt2 =", f"{ps:.9e}", " Q / 2 (highest first):", ", ".join(f"{v:.9e}" for v in C))


def tanh_check():
    """r04 bcnf_device.h tanh_bf: 1 - 2 / (exp(2a) + 1) in emulated fp32 against float64 tanh."""
    a = np.linspace(-12, 12, 2000001).astype(f32)
    e = f32(np.exp2(np.float64(f32(a * f32(2 * np.log2(np.e))))))
    r = f32(1.0 / np.float64(f32(e + f32(1))))
    got = fma(f32(-2), r, f32(1))
    print(f"tanh_check: max abs err {np.abs(got - np.tanh(a.astype(np.float64))).max():.3e}")


def gelu_r04_check():
    """r04 bcnf_device.h gelu_tq / gelu_f / gelu_fg: Q scaled by sqrt(2 pi), phi = exp2(x^2 k + log2(1/sqrt(2 pi))),
    Phi(x) = 1/2 + sign(x) (1/2 - h), GELU = max(x, 0) - |x| h."""
    from scipy.special import ndtr
    C = [f32(v) for v in (-1.828701629e-01, 5.613370996e-01, -2.561027660e-01, 4.147041470e-01, 1.844545274e-01,
                          2.707437625e-01, 2.610471003e-01)]
    x = np.linspace(-12, 12, 2000001).astype(f32)
    t = f32(1) / fma(f32(2.616295218e-01), np.abs(x), f32(1))
    q = np.full_like(x, C[0])
    for cc in C[1:]:
        q = fma(q, t, cc)
    phi = f32(np.exp2(np.float64(fma(f32(x * x), f32(-0.72134752044448170368), f32(-1.32574806473615920)))))
    tq = f32(t * q)
    hm = fma(-tq, phi, f32(0.5))
    cdf = f32(f32(0.5) + f32(np.copysign(hm, x)))
    g, dg = f32(x * cdf), fma(x, phi, cdf)
    g2 = fma(-np.abs(x), f32(tq * phi), np.maximum(x, f32(0)))
    xd = x.astype(np.float64)
    P = ndtr(xd)
    print(f"gelu_r04_check: |GELU err| fg {np.abs(g - xd * P).max():.2e}, f {np.abs(g2 - xd * P).max():.2e}; "
          f"|GELU' err| {np.abs(dg - (P + xd * np.exp(-xd * xd / 2) / np.sqrt(2 * np.pi))).max():.2e}")


def fit_log2h(deg=6, amax=6.5, iters=200):
    """r04 gelu_p2 / gelu_pf (forward-only GELU): log2 h(a), h = erfc(a / sqrt 2) / 2, as ONE polynomial in
    a = min(|x|, amax) (erfc's e^{-a^2/2} decay is quadratic in a, so it sits inside the fit), reweighted toward the
    minimax of the GELU error |a (h_fit - h)|; then the emulated-fp32 GELU error of the rounded coefficients."""
    from scipy.special import erfc
    a = np.linspace(0, amax, 400001)
    h = erfc(a / np.sqrt(2)) / 2
    V = np.vander(a, deg + 1)
    w = np.ones_like(a)
    for _ in range(iters):
        c, *_ = np.linalg.lstsq(V * w[:, None], np.log2(h) * w, rcond=None)
        err = np.abs(a * (np.exp2(V @ c) - h))
        w = w * (1 + 0.5 * err / err.max())
    c32 = c.astype(f32)
    x = np.linspace(-12, 12, 2000001).astype(f32)
    aa = np.minimum(np.abs(x), f32(amax))
    p = np.full_like(x, c32[0])
    for cc in c32[1:]:
        p = fma(p, aa, cc)
    g = fma(-np.abs(x), f32(np.exp2(np.float64(p))), np.maximum(x, f32(0)))
    from scipy.special import ndtr
    xd = x.astype(np.float64)
    print(f"fit_log2h(deg={deg}): exact-arith max |a dh| {err.max():.2e}; fp32 |GELU err| "
          f"{np.abs(g - xd * ndtr(xd)).max():.2e} (x < 0: {np.abs(g - xd * ndtr(xd))[x < 0].max():.2e})")
    print("  coefficients (highest first):", ", ".join(f"{float(v):.9e}" for v in c32))


if __name__ == "__main__":
    gelu_fit()
    tanh_check()
    gelu_r04_check()
    fit_log2h()
