"""The device LAPACK emulation (land_trendr_amd/csrc/lt_lapack.h), compiled for the HOST by
hipcc (tests/native/lapack_host_check.hip), against the oracle's x87 long-double restatement and
the reference's own lstsq goldens. This runs the kernels' exact arithmetic code without a GPU."""
import ctypes
import os

import numpy as np
import pytest

import golden_io
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOSTCHECK = os.path.join(ROOT, 'tests', 'native', 'build', 'liblt_hostcheck.so')
D = ctypes.POINTER(ctypes.c_double)


@pytest.fixture(scope='module')
def hc():
    if not os.path.exists(HOSTCHECK):
        pytest.fail('host harness not built: run __graft_entry__.build()')
    L = ctypes.CDLL(HOSTCHECK)
    L.ltx_lstsq.argtypes = [ctypes.c_int, D, D, ctypes.c_int, D]
    L.ltx_nrm2.argtypes = [ctypes.c_int, D]
    L.ltx_nrm2.restype = ctypes.c_double
    return L


def _lstsq(hc, x, y, sol=1):
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    o = (ctypes.c_double * 3)()
    rc = hc.ltx_lstsq(len(x), x.ctypes.data_as(D), y.ctypes.data_as(D), sol,
                      ctypes.cast(o, D))
    return rc, o[0], o[1], o[2]


def test_device_lstsq_matches_reference_goldens(hc):
    z = dict(np.load(os.path.join(golden_io.GOLDEN, 'lstsq.npz')))
    bad = 0
    for t in range(len(z['m'])):
        m = int(z['m'][t])
        rc, s, c, r = _lstsq(hc, z['x'][t, :m], z['y'][t, :m])
        assert rc == 0
        want = (z['slope'][t], z['icpt'][t], z['ssr'][t])
        bad += not all(golden_io._bits_equal(a, b) for a, b in zip((s, c, r), want))
    assert bad == 0


def test_device_lstsq_matches_oracle_random(hc):
    rng = np.random.default_rng(2024)
    bad = 0
    for t in range(30000):
        m = int(rng.integers(2, 65))
        x = np.sort(rng.choice(np.arange(0, 70), m, replace=False)).astype(np.float64)
        kind = t % 4
        if kind == 0:
            y = rng.integers(-3000, 3000, m).astype(np.float64)
        elif kind == 1:
            y = rng.normal(0, 1, m) * 10.0 ** rng.integers(-8, 9)
        elif kind == 2:
            y = rng.integers(0, 3, m).astype(np.float64)
        else:
            y = np.round(rng.normal(0, 40, m)) + np.arange(m) * rng.integers(-60, 60)
        got = _lstsq(hc, x, y)
        want = oracle.lstsq(x, y)
        if got != want and not all(golden_io._bits_equal(a, b) for a, b in zip(got, want)):
            bad += 1
        # the DP's residual-only variant must give the same residual
        r2 = _lstsq(hc, x, y, sol=0)[3]
        bad += not golden_io._bits_equal(r2, want[3])
    assert bad == 0


def test_soft_float80_nrm2_matches_x87(hc):
    """dnrm2 over wide-range values: soft-float80 vs the host's x87 long double."""
    rng = np.random.default_rng(5)
    lib = oracle.lib()
    bad = 0
    for t in range(20000):
        n = int(rng.integers(1, 70))
        x = rng.normal(0, 1, n) * 10.0 ** rng.integers(-150, 150, n)
        x = np.ascontiguousarray(x)
        got = hc.ltx_nrm2(n, x.ctypes.data_as(D))
        # oracle: lstsq's H1 uses dnrm2 of x[1:]; compare through the closed form instead
        ld = np.longdouble(0)
        acc = [np.longdouble(0)] * 4
        n8 = n & ~7
        for j in range(n):
            v = np.longdouble(x[j])
            if j < n8:
                acc[j & 3] = acc[j & 3] + v * v
            else:
                acc[0] = acc[0] + v * v
        tt = ((acc[0] + acc[2]) + acc[1]) + acc[3]
        want = abs(x[0]) if n == 1 else float(np.sqrt(tt))
        bad += not golden_io._bits_equal(got, want)
    assert bad == 0


def test_integer_x_fused_variant_matches_oracle(hc):
    """lstsq_xint (fused passes, integer dnrm2 of x) is bit-identical to the oracle."""
    hc.ltx_lstsq_xint.argtypes = [ctypes.c_int, D, D, ctypes.c_int, ctypes.c_int, D]
    rng = np.random.default_rng(77)
    z = dict(np.load(os.path.join(golden_io.GOLDEN, 'lstsq.npz')))
    cases = [(z['x'][t, :int(z['m'][t])], z['y'][t, :int(z['m'][t])]) for t in range(len(z['m']))]
    for t in range(20000):
        m = int(rng.integers(2, 65))
        x = np.sort(rng.choice(np.arange(0, 256), m, replace=False)).astype(np.float64)
        kind = t % 3
        y = (rng.integers(-3000, 3000, m).astype(np.float64) if kind == 0 else
             rng.normal(0, 1, m) * 10.0 ** rng.integers(-8, 9) if kind == 1 else
             rng.integers(0, 3, m).astype(np.float64))
        cases.append((x, y))
    bad = 0
    for x, y in cases:
        x = np.ascontiguousarray(x, np.float64)
        y = np.ascontiguousarray(y, np.float64)
        want = oracle.lstsq(x, y)
        for sol, ssr in ((1, 1), (1, 0), (0, 1)):
            o = (ctypes.c_double * 3)()
            rc = hc.ltx_lstsq_xint(len(x), x.ctypes.data_as(D), y.ctypes.data_as(D), sol, ssr,
                                   ctypes.cast(o, D))
            assert rc == want[0]
            if sol:
                bad += not (golden_io._bits_equal(o[0], want[1]) and
                            golden_io._bits_equal(o[1], want[2]))
            if ssr:
                bad += not golden_io._bits_equal(o[2], want[3])
    assert bad == 0


def test_pair_arithmetic_nrm2_matches_integer_f80(hc):
    """nrm2_dd (binary64 pairs) is bit-identical to the integer soft-float80 nrm2 whenever it does
    not ask for the fallback; adversarial inputs: squares on binade edges (c = 2^k (1 +- eps)),
    exact ties of the 64-bit rounding, zeros, wide exponent spreads."""
    L = hc
    L.ltx_nrm2_dd.argtypes = [ctypes.c_int, D, ctypes.POINTER(ctypes.c_int)]
    L.ltx_nrm2_dd.restype = ctypes.c_double
    rng = np.random.default_rng(99)
    slow = ctypes.c_int(0)
    bad = 0
    nslow = [0] * 6
    for t in range(40000):
        n = int(rng.integers(1, 66))
        kind = t % 6
        if kind == 0:
            x = rng.normal(0, 1, n)
        elif kind == 1:
            x = rng.normal(0, 1, n) * 10.0 ** rng.integers(-12, 12, n)
        elif kind == 2:  # near powers of two: c^2 rounds onto / just below a binade edge
            k = rng.integers(-4, 5, n).astype(np.float64)
            eps = rng.integers(-3, 4, n) * 2.0 ** -52
            x = np.ldexp(1.0 + eps, k.astype(int)) * np.where(rng.random(n) < 0.5, -1, 1)
        elif kind == 3:  # 27-bit significands: squares exact in 54 bits, sums with exact ties
            x = np.ldexp(rng.integers(1 << 26, 1 << 27, n).astype(np.float64),
                         rng.integers(-6, 1, n))
        elif kind == 4:  # zeros and repeated values
            x = rng.choice([0.0, 1.0, -1.0, 3.0, 0.5, 1e-3], n)
        else:  # what the fit sees: c = 1 + sc * x * s1 over increasing integer x
            xs = np.sort(rng.choice(np.arange(0, 70), n, replace=False)).astype(np.float64)
            s1 = 1.0 / (xs[0] - np.sqrt(xs[0] ** 2 + (xs[1:] ** 2).sum() if n > 1 else 1.0))
            x = 1.0 + rng.normal(-1, 0.5) * xs * s1
        x = np.ascontiguousarray(x, np.float64)
        want = hc.ltx_nrm2(n, x.ctypes.data_as(D))
        got = hc.ltx_nrm2_dd(n, x.ctypes.data_as(D), ctypes.byref(slow))
        if slow.value:
            nslow[kind] += 1
            continue
        bad += not golden_io._bits_equal(got, want)
    assert bad == 0
    print('fallbacks per kind (of %d):' % (40000 // 6), nslow)
    assert nslow[0] + nslow[2] + nslow[3] + nslow[4] + nslow[5] < 40000 // 6 * 0.05


def _round64(v):
    """Fraction -> nearest value with a 64-bit significand (ties to even), as a Fraction."""
    from fractions import Fraction
    if v == 0:
        return Fraction(0)
    e = v.numerator.bit_length() - v.denominator.bit_length()
    while Fraction(2) ** e > v:
        e -= 1
    while Fraction(2) ** (e + 1) <= v:
        e += 1
    u = Fraction(2) ** (e - 63)
    q, r = divmod(v, u)
    if r * 2 > u or (r * 2 == u and q % 2 == 1):
        q += 1
    return q * u


def test_pair_sqrt_matches_integer_f80(hc):
    """xdd_sqrt_to_double: x87 double rounding of sqrt (64 then 53 bits) on pairs, against the
    integer soft-float80 path, including values whose root sits next to a 53-bit midpoint."""
    from fractions import Fraction
    hc.ltx_sqrt_pair.argtypes = [ctypes.c_double, ctypes.c_double, D]
    rng = np.random.default_rng(2718)
    out = (ctypes.c_double * 2)()
    bad = nslow = 0
    N = 20000
    for t in range(N):
        kind = t % 3
        if kind == 0:  # random 64-bit significand
            sig = int(rng.integers(1 << 62, 1 << 63)) * 2 + int(rng.integers(0, 2))
            V = Fraction(sig) * Fraction(2) ** int(rng.integers(-80, 80))
        elif kind == 1:  # root next to a 53-bit midpoint: (M + 1/2 + delta)^2, rounded to 64 bits
            M = int(rng.integers(1 << 52, 1 << 53))
            delta = Fraction(int(rng.integers(-64, 65)), 1 << int(rng.integers(10, 40)))
            V = _round64((Fraction(M) + Fraction(1, 2) + delta) ** 2)
            V *= Fraction(2) ** (2 * int(rng.integers(-40, 10)))
        else:  # perfect squares and small integers (the x-norm case)
            V = Fraction(int(rng.integers(1, 1 << 40)))
            if t % 2:
                r = int(rng.integers(1, 1 << 26))
                V = Fraction(r * r)
        hi = float(V)
        lo = float(V - Fraction(hi))
        slow = hc.ltx_sqrt_pair(hi, lo, ctypes.cast(out, D))
        if slow:
            nslow += 1
            continue
        bad += not golden_io._bits_equal(out[0], out[1])
    assert bad == 0
    assert nslow < N * 0.01


def test_xset_table_keys_round_trip(hc):
    """Every slot of the x-set factor table maps back to itself (lt_lapack.h xset_key)."""
    nv = ctypes.c_int(0)
    hc.ltx_xset_roundtrip.argtypes = [ctypes.POINTER(ctypes.c_int)]
    assert hc.ltx_xset_roundtrip(ctypes.byref(nv)) == 0
    assert nv.value > 8000


def test_small_segment_apply_matches_general_bit_for_bit(hc):
    """lsq_apply_small (the vertex fits' straight-line path for 2-4 points) gives lsq_apply's
    solution bits and return code on the same factorisation: integer, non-integer, zero, tiny,
    huge and collinear y over consecutive and gapped x."""
    D = ctypes.POINTER(ctypes.c_double)
    hc.ltx_lsq_small_vs_general.argtypes = [ctypes.c_int, D, D, D]
    rng = np.random.default_rng(77)
    out = (ctypes.c_double * 4)()
    n = 0
    for t in range(30000):
        m = 2 + t % 3
        x = np.cumsum(rng.integers(1, 1 + [1, 3, 9][t % 3], m)).astype(np.float64) + \
            float(rng.integers(0, 40))
        kind = (t // 3) % 6
        if kind == 0:
            y = rng.integers(-32768, 32768, m).astype(np.float64)
        elif kind == 1:
            y = rng.normal(0, 1, m)
        elif kind == 2:
            y = np.zeros(m)
            y[rng.integers(0, m)] = float(rng.integers(-3, 4))
        elif kind == 3:
            y = rng.normal(0, 1, m) * 2.0 ** int(rng.integers(-990, 990))
        elif kind == 4:
            y = 5.0 + 2.5 * x
        else:
            y = np.round(rng.normal(1000, 40, m))
        rc = hc.ltx_lsq_small_vs_general(m, x.ctypes.data_as(D), y.ctypes.data_as(D),
                                         ctypes.cast(out, D))
        a, b = rc // 16 - 8, rc % 16 - 8
        assert a == b, (m, x, y, a, b)
        if b == 0:
            assert golden_io._bits_equal(np.array(out[:2]), np.array(out[2:])).all(), (m, x, y)
            n += 1
    assert n > 20000
