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
