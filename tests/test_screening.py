"""Evidence for the DP's screening bound (land_trendr_amd/csrc/lt_pixel.h kScreen = 2^-30).

The analyze kernel prices DP candidates with a closed-form SSE and decides a column without the
emulated LAPACK residual when the candidates' intervals separate; the interval half-width per
segment is kScreen * sum(y^2) (+ rounding terms). That is sound if, for every segment,
    |emulated dgelsd residual (the reference's value) - closed-form residual| <= kScreen * Syy.
This file measures both errors against the EXACT rational SSE (fractions.Fraction) over
adversarial segments — integer and non-integer values, large offsets with small variance,
nearly collinear data, gapped x sets, m up to 64 — and requires a margin of at least 2^10 below
kScreen (the bound the header states: LAPACK within 2^-48 Syy, closed form within 2^-44 Syy).

The closed form is restated exactly as the kernel computes it (lt_fast.h `price`): sums from the
column's end point downwards with fma for Sxy and Syy, t1 = fma(m, Syy, -Sy*Sy),
N1 = fma(m, Sxy, -Sx*Sy), e = fma(t1, D, -N1*N1) * r with r the reciprocal of m*D (the kernel's
v_rcp_f64 + one Newton step is within an ulp of it: counted in the margin). fma is evaluated with
exact rationals and one rounding.
"""
import math
from fractions import Fraction as F

import numpy as np
import pytest

from oracle import oracle

K_SCREEN = 2.0 ** -30
MARGIN = 2.0 ** -10


def fma(a, b, c):
    return float(F(a) * F(b) + F(c))


def exact_sse(x, y):
    m = len(x)
    Sx = sum(F(v) for v in x)
    Sxx = sum(F(v) * F(v) for v in x)
    Sy = sum(F(v) for v in y)
    Sxy = sum(F(a) * F(b) for a, b in zip(x, y))
    Syy = sum(F(v) * F(v) for v in y)
    D = m * Sxx - Sx * Sx
    N1 = m * Sxy - Sx * Sy
    return (m * Syy - Sy * Sy - N1 * N1 / D) / m, Syy


def closed_form(x, y):
    """lt_fast.h price(): starts visited from the column end downwards."""
    Sx = Sxx = 0
    Sy = Sxy = Syy = 0.0
    for xi, yi in zip(reversed(x), reversed(y)):
        Sx += int(xi)
        Sxx += int(xi) * int(xi)
        Sy = Sy + yi
        Sxy = fma(float(xi), yi, Sxy)
        Syy = fma(yi, yi, Syy)
    m = len(x)
    md = float(m)
    D = float(m * Sxx - Sx * Sx)
    t1 = fma(md, Syy, -(Sy * Sy))
    N1 = fma(md, Sxy, -(float(Sx) * Sy))
    den = md * D
    r = float(F(1) / F(den))
    e = fma(t1, D, -(N1 * N1)) * r
    return max(e, 0.0)


def segments(seed=5):
    rng = np.random.default_rng(seed)
    out = []

    def xs(m, gaps):
        if not gaps:
            return list(range(m))
        return [int(v) for v in np.cumsum(rng.integers(1, 4, m)) - 1]

    for m in [3, 4, 5, 8, 13, 21, 30, 40, 48, 64]:
        for gaps in (False, True):
            x = xs(m, gaps)
            if max(x) > 255:
                continue
            # integer index values over the whole int16 range
            out.append((x, [float(v) for v in rng.integers(-32768, 32768, m)]))
            # synthetic-like: base, drop, noise
            out.append((x, [float(v) for v in 1200 - 3 * np.arange(m) +
                            np.round(rng.normal(0, 40, m))]))
            # non-integer binary32 values (the analyze stage's series type)
            out.append((x, [float(np.float32(v)) for v in rng.normal(0.3, 0.2, m)]))
            # non-integer doubles (the resolve stage's binary64 series)
            out.append((x, [float(v) for v in rng.uniform(-1, 1, m)]))
            # large offset, small variance: cancellation in m*Syy - Sy^2
            out.append((x, [1e6 + float(v) for v in rng.integers(-3, 4, m)]))
            out.append((x, [2.0 ** 40 + float(v) for v in rng.integers(-2, 3, m)]))
            out.append((x, [float(v) for v in 1e5 + rng.uniform(0, 1e-3, m)]))
            # nearly collinear: SSE ~ 0 next to a large Syy
            out.append((x, [7.0 + 3.5 * xi + (1e-9 if k == m // 2 else 0.0)
                            for k, xi in enumerate(x)]))
            out.append((x, [1000.0 * xi for xi in x]))
            # one outlier
            y = [100.0] * m
            y[m // 3] = 30000.0
            out.append((x, y))
    return out


def test_screening_bound_holds_with_margin():
    worst_lapack = worst_cf = worst_diff = 0.0
    n = 0
    for x, y in [seg for seed in range(5) for seg in segments(seed)]:
        rc, slope, icpt, ssr = oracle.lstsq(np.array(x, float), np.array(y, float))
        if rc != 0:  # a path the emulation does not cover is flagged, never screened
            continue
        exact, syy = exact_sse(x, y)
        if syy == 0:
            continue
        cf = closed_form(x, y)
        ex = float(exact)
        worst_lapack = max(worst_lapack, float(abs(F(ssr) - exact) / syy))
        worst_cf = max(worst_cf, float(abs(F(cf) - exact) / syy))
        worst_diff = max(worst_diff, abs(ssr - cf) / float(syy))
        n += 1
        assert abs(ssr - cf) <= K_SCREEN * MARGIN * float(syy), (x, y, ssr, cf, ex)
    assert n > 900
    print('segments %d: |lapack-exact|/Syy <= 2^%.1f, |closed-exact|/Syy <= 2^%.1f, '
          '|lapack-closed|/Syy <= 2^%.1f (kScreen 2^-30)' % (
              n, math.log2(worst_lapack or 2.0 ** -99), math.log2(worst_cf or 2.0 ** -99),
              math.log2(worst_diff or 2.0 ** -99)))
    # the header's figures: LAPACK within 2^-48 * Syy of exact, closed form within 2^-44
    assert worst_lapack <= 2.0 ** -44
    assert worst_cf <= 2.0 ** -44


@pytest.mark.parametrize('m', [3, 30, 64])
def test_closed_form_restatement_is_exact_on_small_integers(m):
    """Sanity of the restatement: small integer data, every sum exact, SSE exact up to one
    rounding of the final product."""
    rng = np.random.default_rng(m)
    x = list(range(m))
    y = [float(v) for v in rng.integers(0, 50, m)]
    exact, _ = exact_sse(x, y)
    cf = closed_form(x, y)
    assert abs(F(cf) - exact) <= abs(exact) * F(2) ** -50 + F(2) ** -60


K_ZERO = 2.0 ** -80  # lt_pixel.h kZero


def collinear_segments(seed, count):
    """Exactly collinear integer segments of int16 range: y = a + b*(x - x0) with integer a, b,
    consecutive and gapped x sets, m from 3 to 64."""
    rng = np.random.default_rng(seed)
    out = []
    while len(out) < count:
        m = int(rng.choice([3, 3, 3, 4, 4, 5, 6, 8, 12, 20, 40, 64]))
        if rng.integers(0, 2):
            x0 = int(rng.integers(0, 64 - m + 1))
            x = np.arange(x0, x0 + m)
        else:
            x = np.sort(rng.choice(64, m, replace=False))
        b = int(rng.integers(-2000, 2001)) if rng.integers(0, 2) else int(rng.integers(-3, 4))
        a = int(rng.integers(-32768, 32768))
        y = a + b * (x - x[0])
        if y.min() < -32768 or y.max() > 32767:
            continue
        out.append(([int(v) for v in x], [float(v) for v in y]))
    return out


def test_collinear_residual_bound():
    """kZero: on an exactly collinear segment the reference's residual (the emulated dgelsd,
    bit-exact with numpy's) is pure rounding noise, quadratic in the unit roundoff. The kernel
    treats such a start as worth fl(c + OPT) when kZero * Syy < 2^-54 * c, so kZero must bound it;
    require a 2^10 margin."""
    worst = 0.0
    n = 0
    for x, y in collinear_segments(11, 4000):
        rc, slope, icpt, ssr = oracle.lstsq(np.array(x, float), np.array(y, float))
        assert rc == 0
        syy = sum(v * v for v in y)
        if syy == 0:
            continue
        worst = max(worst, ssr / syy)
        n += 1
        assert ssr <= K_ZERO * MARGIN * syy, (x, y, ssr)
    print('collinear segments %d: residual/Syy <= 2^%.1f (kZero 2^-80)' % (
        n, math.log2(worst or 2.0 ** -200)))


def sse_exact_zero(x, y):
    """lt_pixel.h sse_exact_zero on the closed form's sums as lt_fast.h price() forms them."""
    Sx = Sxx = 0
    Sy = Sxy = Syy = 0.0
    for xi, yi in zip(reversed(x), reversed(y)):
        Sx += xi
        Sxx += xi * xi
        Sy = Sy + yi
        Sxy = fma(float(xi), yi, Sxy)
        Syy = fma(yi, yi, Syy)
    m = len(x)
    md = float(m)
    D = float(m * Sxx - Sx * Sx)
    t1 = fma(md, Syy, -(Sy * Sy))
    N1 = fma(md, Sxy, -(float(Sx) * Sy))
    p, q = t1 * D, N1 * N1
    return p == q and fma(t1, D, -p) == fma(N1, N1, -q)


def test_exact_zero_test_is_exact_on_int16_segments():
    """sse_exact_zero says 'collinear' exactly when the exact rational SSE is 0, for integer
    values of int16 range (where every sum it uses is an exact binary64 integer)."""
    rng = np.random.default_rng(3)
    segs = collinear_segments(12, 600)
    # near misses: one value off by one (the smallest nonzero SSE an integer series can have)
    for x, y in collinear_segments(13, 600):
        k = int(rng.integers(0, len(y)))
        y = list(y)
        y[k] += 1.0 if y[k] < 32767 else -1.0
        segs.append((x, y))
    for x, y in segs:
        exact, _ = exact_sse(x, y)
        assert sse_exact_zero(x, y) == (exact == 0), (x, y, exact)


K_FITW = 2.0 ** -32  # lt_pixel.h kFitW


def closed_form_fit(x, y):
    """lt_fast.h labels-only pass A: the closed-form slope and intercept of a segment (sums from
    its first point on, fma for Sxy; reciprocals of D and m within an ulp: exact roundings here,
    the difference is counted in the margin) and its error scale |slope|*64 + |icpt| + max|y|."""
    Sx = Sxx = 0
    Sy = Sxy = 0.0
    for xi, yi in zip(x, y):
        Sx += int(xi)
        Sxx += int(xi) * int(xi)
        Sy = Sy + yi
        Sxy = fma(float(xi), yi, Sxy)
    m = len(x)
    md = float(m)
    D = float(m * Sxx - Sx * Sx)
    N1 = fma(md, Sxy, -(float(Sx) * Sy))
    sm = N1 * float(F(1) / F(D))
    sb = fma(-sm, float(Sx), Sy) * float(F(1) / F(m))
    scale = fma(abs(sm), 64.0, abs(sb)) + max(abs(v) for v in y)
    return sm, sb, scale


def fit_segments(seed):
    """Segments as the vertex fits see them: 2 to 64 points, x offsets up to 63 (late, short
    segments are the worst conditioned), the value patterns of segments() above."""
    rng = np.random.default_rng(seed)
    out = []
    for m in [2, 2, 2, 3, 3, 4, 4, 5, 8, 13, 30, 64]:
        for gaps in (False, True):
            if gaps and m <= 21:
                x = np.sort(rng.choice(64, m, replace=False))
            else:
                x0 = int(rng.integers(0, 64 - m + 1))
                x = np.arange(x0, x0 + m)
            x = [int(v) for v in x]
            ys = [
                [float(v) for v in rng.integers(-32768, 32768, m)],
                [float(v) for v in 1200 - 3 * np.arange(m) + np.round(rng.normal(0, 40, m))],
                [float(np.float32(v)) for v in rng.normal(0.3, 0.2, m)],
                [1e6 + float(v) for v in rng.integers(-3, 4, m)],
                [float(np.float32(v)) for v in 1e5 + rng.uniform(0, 1e-3, m)],
                [7.0 + 3.5 * xi for xi in x],
                [float(v) for v in rng.integers(-1, 2, m)],
                [0.0] * (m - 1) + [1.0],
            ]
            for y in ys:
                out.append((x, y))
    return out


def test_fit_bound_holds_with_margin():
    """kFitW: the labels-only path prices every vertex fit with the closed form and carries the
    fitted value at a vertex as an interval of half-width kFitW * scale around the reference's;
    the winners are then re-fitted with the emulated dgelsd. Sound if the reference's fitted value
    (emulated dgelsd eqn, evaluated as fl(fl(m*x) + b)) and the closed form's lie within
    kFitW * scale of each other at every x of the segment. Requires a 2^10 margin."""
    worst = worst_ref = 0.0
    n = 0
    for seed in range(40):
        for x, y in fit_segments(seed):
            rc, slope, icpt, _ = oracle.lstsq(np.array(x, float), np.array(y, float))
            assert rc == 0
            cm, cb, scale = closed_form_fit(x, y)
            m = len(x)
            Sx, Sy = sum(F(v) for v in x), sum(F(v) for v in y)
            D = m * sum(F(v) * F(v) for v in x) - Sx * Sx
            se = (m * sum(F(a) * F(b) for a, b in zip(x, y)) - Sx * Sy) / D
            be = (Sy - se * Sx) / m
            for xv in x:
                ref = slope * xv + icpt
                cf = cm * xv + cb
                if scale == 0:  # all-zero values: both fits are 0 (DGELSD's B == 0 shortcut)
                    assert ref == 0 and cf == 0
                    continue
                worst = max(worst, abs(ref - cf) / scale)
                worst_ref = max(worst_ref, float(abs(F(ref) - (se * xv + be)) / F(scale)))
                assert abs(ref - cf) <= K_FITW * MARGIN * scale, (x, y, xv, ref, cf, scale)
            n += 1
    assert n > 3000
    print('segments %d: |reference fit - closed form|/scale <= 2^%.1f, |reference - exact|/scale '
          '<= 2^%.1f (kFitW 2^-32)' % (n, math.log2(worst or 2.0 ** -99),
                                       math.log2(worst_ref or 2.0 ** -99)))
