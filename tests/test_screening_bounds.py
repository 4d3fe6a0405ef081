"""A-priori error bounds behind the kernels' screening constants (VERDICT r04 item 8;
land_trendr_amd/csrc/lt_pixel.h kScreen, kZero / kZeroWide, kFitW / fit_width_factor), for the
int16 series the analyze kernel sees from an int16 index raster: m <= 64 points, values of int16
range, year offsets x strictly increasing integers in [0, X], X <= 255 (lt_abi.hip refuses wider
year spans). DESIGN.md § Screening bounds derives them; this file evaluates the derived formulas
and asserts that each bound
  (1) lies below the constant the kernel uses, for every m and X allowed, and
  (2) lies above every error measured on the adversarial segments of tests/test_screening.py (and
      on ill-conditioned segments at offsets up to 255), per segment, from its own x set.

Standard backward-error results (Higham, Accuracy and Stability of Numerical Algorithms, 2nd ed.,
Lemmas 19.2-19.3, Theorems 19.4, 20.3) with gamma(k) = k u / (1 - k u), u = 2^-53, and
gamma~(k) = gamma(C k) for Householder steps, C = 8 (the "small integer constant" of those
results, taken generously). The one hardware constant, the relative error of the kernel's
reciprocal (v_rcp_f64 + one Newton step), is measured on the GPU (tools/rcp_check.hip,
profiles/r05_rcp_check.json).
"""
import json
import math
import os
from fractions import Fraction as F

import numpy as np

from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
U = 2.0 ** -53
C = 8
K_SCREEN = 2.0 ** -30
K_ZERO, K_ZERO_WIDE = 2.0 ** -80, 2.0 ** -74
K_FITW, FIT_WIDE = 2.0 ** -32, 16.0


def gamma(k):
    return k * U / (1 - k * U)


def gt(m):
    return gamma(C * m)


def rcp_newton_err():
    """Relative error of v_rcp_f64 + one Newton step, measured on the box; the bound uses twice
    the worst measured value, and at least 2u."""
    with open(os.path.join(ROOT, 'profiles', 'r05_rcp_check.json')) as f:
        d = json.load(f)
    return max(2.0 * d['rcp_newton_max_rel_err'], 2.0 * U)


def ratio(x):
    """||x|| / ||x - mean(x)||: how far the x column is from the ones column's span."""
    x = np.asarray(x, float)
    return float(np.linalg.norm(x) / np.linalg.norm(x - x.mean()))


def kappa_f(x):
    """||A||_F / sigma_min(A) of A = [1, x]."""
    A = np.stack([np.ones(len(x)), np.asarray(x, float)], 1)
    s = np.linalg.svd(A, compute_uv=False)
    return float(np.linalg.norm(A) / s[-1])


def worst_x(m, X):
    """The worst-conditioned x set of m distinct offsets in [0, X]: consecutive, ending at X."""
    return list(range(X - m + 1, X + 1))


# ---- (A) the closed form of the DP (lt_fast.h price) on int16 data: every sum and t1, D, N1 are
# exact binary64 integers; q = fl(N1^2), n = fl(t1 D - q), r = 1/(mD)(1 + e_r), e = fl(n r):
# |e - E| <= (u + u + e_r + u) E + u N1^2/(mD), and E, N1^2/(mD) <= t1/m <= Syy
def b_closed_form():
    return (4 * U + rcp_newton_err()) * (1 + 2.0 ** -40)


# ---- (B) the emulated dgelsd residual (numpy's lstsq residual = the squared norm of rows 2.. of
# Q^T y, Q from the two Householder reflections of A = [1, x]): the computed reflections are
# those of [1, x + dx], |dx| <= gt(m)|x|, up to gt(m) each; the residual subspace moves by
# sin(theta) <= |dx| / |x - mean(x)|, so |computed residual norm - |r|| <= eta |y| with
# eta = gt(m) (ratio(x) + 2), and the sum of m squares adds gamma(m)
def eta(x):
    return gt(len(x)) * (ratio(x) + 2.0)


def b_lapack(x):
    e = eta(x)
    g = gamma(len(x))
    return (2 * e + e * e + g) * (1 + g)


def b_screen(x):
    return b_lapack(x) + b_closed_form()


# ---- (C) exactly collinear segments: r = 0, so the computed residual is at most (eta |y|)^2
def b_zero(x):
    return eta(x) ** 2 * (1 + gamma(len(x)))


# ---- (D) fitted values at a vertex (a data point of the segment, leverage <= 1), relative to the
# kernel's scale S = 64 |slope| + |icpt| + max|y|: the reference's LS solution is exact for
# (A + dA, y + dy) (|dA e_j| <= gt|A e_j|, |dy| <= gt|y|), so its fitted value moves by at most
# gt sqrt(m) (max|y| + |icpt| + X |slope|) + gt kappa_F |r| (first order) plus the evaluation's
# two roundings; the closed form's slope N1 / D and intercept carry the reciprocal's error
def b_fit(x):
    m, X = len(x), max(x)
    g = gt(m)
    er = rcp_newton_err()
    sx = X / 64.0  # X |slope| <= (X / 64) S
    ref = g * math.sqrt(m) * (2 + sx) + g * kappa_f(x) * math.sqrt(m) + 2 * U * (1 + sx)
    cf = (2 * (er + U) + 2 * U) * sx + (4 * U + er)
    return ref + cf


def test_derived_bounds_lie_below_the_kernel_constants():
    worst = {'screen': 0.0, 'zero63': 0.0, 'zero255': 0.0, 'fit63': 0.0, 'fit255': 0.0}
    for m in range(2, 65):
        for X in range(m - 1, 256):
            x = worst_x(m, X)
            if m >= 3:
                worst['screen'] = max(worst['screen'], b_screen(x))
                worst['zero63' if X <= 63 else 'zero255'] = max(
                    worst['zero63' if X <= 63 else 'zero255'], b_zero(x))
            worst['fit63' if X <= 63 else 'fit255'] = max(worst['fit63' if X <= 63 else 'fit255'],
                                                          b_fit(x))
    print({k: '2^%.1f' % math.log2(v) for k, v in worst.items()})
    assert worst['screen'] <= K_SCREEN
    assert worst['zero63'] <= K_ZERO
    assert worst['zero255'] <= K_ZERO_WIDE
    assert worst['fit63'] <= K_FITW
    assert worst['fit255'] <= K_FITW * FIT_WIDE
    # and the worst case needs the wide constants: X > 63 exceeds the narrow ones
    assert worst['fit255'] > K_FITW or worst['zero255'] > K_ZERO


def _exact_sse(x, y):
    m = len(x)
    Sx, Sxx = sum(F(v) for v in x), sum(F(v) * F(v) for v in x)
    Sy, Syy = sum(F(v) for v in y), sum(F(v) * F(v) for v in y)
    Sxy = sum(F(a) * F(b) for a, b in zip(x, y))
    D, N1 = m * Sxx - Sx * Sx, m * Sxy - Sx * Sy
    return (m * Syy - Sy * Sy - N1 * N1 / D) / m, Syy


def _int16_segments(seed):
    """int16 segments: the test_screening value patterns with integer values, plus short
    ill-conditioned segments at offsets up to 255."""
    rng = np.random.default_rng(seed)
    out = []
    for m in [3, 4, 5, 8, 13, 21, 30, 40, 64]:
        for kind in range(3):
            if kind == 0:
                x = list(range(m))
            elif kind == 1:
                x = [int(v) for v in np.cumsum(rng.integers(1, 4, m)) - 1]
                if max(x) > 255:
                    continue
            else:
                X = int(rng.integers(max(m - 1, 64), 256))
                x = list(range(X - m + 1, X + 1))
            ys = [rng.integers(-32768, 32768, m),
                  np.clip(1200 - 3 * np.arange(m) + np.round(rng.normal(0, 40, m)), -32768, 32767),
                  np.clip(np.round(rng.normal(0, 3, m)) + 20000, -32768, 32767),
                  np.array([100] * (m - 1) + [30000])]
            for y in ys:
                out.append((x, [float(v) for v in y]))
    return out


def test_measured_screening_errors_lie_below_the_derived_bounds():
    n = 0
    tight = 0.0
    for seed in range(6):
        for x, y in _int16_segments(seed):
            rc, slope, icpt, ssr = oracle.lstsq(np.array(x, float), np.array(y, float))
            if rc != 0:
                continue
            exact, syy = _exact_sse(x, y)
            if syy == 0:
                continue
            err = float(abs(F(ssr) - exact) / syy)
            assert err <= b_lapack(x), (x, y, err, b_lapack(x))
            tight = max(tight, err / b_lapack(x))
            n += 1
    assert n > 400
    print('int16 segments %d: measured LAPACK error <= 2^%.1f of the derived bound'
          % (n, math.log2(tight or 2.0 ** -99)))


def test_measured_collinear_residuals_lie_below_the_derived_bound():
    rng = np.random.default_rng(21)
    n = 0
    while n < 3000:
        m = int(rng.choice([3, 3, 4, 5, 8, 20, 64]))
        X = int(rng.integers(m - 1, 256))
        x = np.arange(X - m + 1, X + 1) if rng.integers(0, 2) else np.sort(
            rng.choice(X + 1, m, replace=False))
        b = int(rng.integers(-2000, 2001))
        y = int(rng.integers(-32768, 32768)) + b * (x - x[0])
        if y.min() < -32768 or y.max() > 32767:
            continue
        rc, _, _, ssr = oracle.lstsq(x.astype(float), y.astype(float))
        syy = float((y.astype(float) ** 2).sum())
        if rc != 0 or syy == 0:
            continue
        assert ssr / syy <= b_zero([int(v) for v in x]), (x, y, ssr)
        n += 1


def test_measured_fit_errors_lie_below_the_derived_bound():
    """The reference's fitted value (emulated dgelsd eqn, fl(fl(m x) + b)) against the closed
    form as the kernel computes it, at every point of the segment, relative to the kernel's
    scale: below the derived b_fit of the segment's x set."""
    import test_screening as ts
    n = 0
    for seed in range(6):
        for x, y in _int16_segments(seed):
            rc, slope, icpt, _ = oracle.lstsq(np.array(x, float), np.array(y, float))
            if rc != 0:
                continue
            cm, cb, scale = ts.closed_form_fit(x, y)
            if scale == 0:
                continue
            for xv in x:
                err = abs((slope * xv + icpt) - (cm * xv + cb)) / scale
                assert err <= b_fit(x), (x, y, xv, err, b_fit(x))
            n += 1
    assert n > 400
