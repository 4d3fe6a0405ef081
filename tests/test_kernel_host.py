"""The kernels' per-pixel pipeline (lt_pixel.h), compiled for the host, against the reference
goldens — the same check as tests/test_gpu_parity.py::test_golden_scene_bit_exact, runnable
without a GPU so kernel changes are parity-checked before they reach the MI355X."""
import ctypes
import os

import numpy as np
import pytest

import golden_io
from land_trendr_amd import _abi
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HOSTCHECK = os.path.join(ROOT, 'tests', 'native', 'build', 'liblt_hostcheck.so')


@pytest.fixture(scope='module')
def hc():
    if not os.path.exists(HOSTCHECK):
        pytest.fail('host harness not built: run __graft_entry__.build()')
    L = ctypes.CDLL(HOSTCHECK)
    L.ltx_analyze_tile.argtypes = [ctypes.POINTER(_abi.LtScene), ctypes.POINTER(_abi.LtParams),
                                   ctypes.POINTER(_abi.LtTileIn), ctypes.POINTER(_abi.LtTileOut)]
    return L


def run_host(hc, scene, params, values, valid):
    values = np.ascontiguousarray(values, np.float64)
    K, P = values.shape
    valid = np.ascontiguousarray(valid, np.uint8) if valid is not None else None
    out = oracle.alloc_outputs(scene.n_years, params.n_rules, P)
    tin = _abi.LtTileIn()
    tin.n_pix, tin.stride = P, P
    tin.obs_val = values.ctypes.data_as(_abi.c_f64p)
    tin.obs_valid = valid.ctypes.data_as(_abi.c_u8p) if valid is not None else None
    sc = scene.to_c()
    o = oracle.out_struct(out, P)
    n_def = hc.ltx_analyze_tile(ctypes.byref(sc), ctypes.byref(params), ctypes.byref(tin),
                                ctypes.byref(o))
    assert 0 <= n_def <= P
    out['_deferred'] = n_def
    return out


@pytest.mark.parametrize('name', golden_io.scene_names())
def test_kernel_code_on_host_matches_reference(hc, name):
    g = golden_io.GoldenScene(name)
    out = run_host(hc, g.scene, g.params, g.values, g.valid)
    bad = golden_io.compare(g, out)
    assert not bad, '\n'.join(bad[:40])


def test_kernel_code_on_host_matches_oracle_synthetic(hc):
    from land_trendr_amd.scene import build_scene, parse_date
    from land_trendr_amd.settings import compile_params
    from land_trendr_amd.synth import make_scene
    for seed, kw, lc in [(11, dict(n_years=30, k_min=1, k_max=3, mask_prob=0.2), 10),
                         (12, dict(n_years=40), 1.0), (13, dict(n_years=20), 0.25)]:
        sc = make_scene(1500, seed=seed, **kw)
        meta = build_scene(sc.dates, parse_date('2014-07-01'))
        params, _ = compile_params(lc, [{'name': 'gd', 'val': 1, 'change_type': 'GD'}])
        vals = sc.values.numpy()
        valid = sc.valid.numpy() if sc.valid is not None else None
        got = run_host(hc, meta, params, vals, valid)
        want = oracle.analyze_tile(meta, params, vals, valid, n_threads=8)
        print('seed %d: %d of %d pixels deferred to the exact-OPT DP' % (seed, got['_deferred'], 1500))
        for f in want:
            a, b = want[f], got[f]
            same = ((a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
                    if a.dtype.kind == 'f' else a == b)
            assert same.all(), (seed, f, int((~same).sum()))


def _vertices(arg, n):
    v, j = {n - 1}, n - 1
    while j >= 0:
        v.add(int(arg[j]))
        j = int(arg[j]) - 1
    return sorted(v)


def _tie_heavy_series(rng, n):
    """Small-integer series built from collinear runs (zero-residual segments of >= 3 points,
    lt_pixel.h kZero), flat stretches and unit noise: the DP's ties and exact-zero starts."""
    kind = rng.integers(0, 4)
    if kind == 0:
        ys = rng.integers(0, 4, n)
    elif kind == 1:  # piecewise-linear integer runs
        ys, v = [], int(rng.integers(-50, 50))
        while len(ys) < n:
            slope, run = int(rng.integers(-5, 6)), int(rng.integers(2, 7))
            for _ in range(run):
                ys.append(v)
                v += slope
        ys = np.array(ys[:n])
    elif kind == 2:  # runs plus occasional unit noise
        ys = np.cumsum(rng.integers(-2, 3, n)) + (rng.random(n) < 0.2) * rng.integers(-1, 2, n)
    else:  # synthetic-like magnitudes
        ys = 1200 + np.round(rng.normal(0, 40, n)) - 10 * np.arange(n)
    xs = np.arange(n) if rng.integers(0, 3) else np.sort(rng.choice(64, n, replace=False))
    return np.ascontiguousarray(xs, np.uint8), np.ascontiguousarray(ys, np.float64)


def test_lazy_dp_with_zero_residual_groups_matches_exact_dp(hc):
    """lt_pixel.h dp_lazy (closed-form intervals, exact-zero starts, same-base tag order) never
    decides a column differently from the exact-OPT DP on the path it reports as decided."""
    u8p = ctypes.POINTER(ctypes.c_uint8)
    f64p = ctypes.POINTER(ctypes.c_double)
    hc.ltx_dp_lazy.argtypes = [ctypes.c_int, u8p, f64p, ctypes.c_double, u8p,
                               ctypes.POINTER(ctypes.c_int)]
    hc.ltx_dp_lazy.restype = ctypes.c_uint64
    hc.ltx_dp_exact.argtypes = [ctypes.c_int, u8p, f64p, ctypes.c_double, u8p]
    rng = np.random.default_rng(21)
    n_dec = n_def = 0
    for _ in range(6000):
        n = int(rng.integers(3, 49))
        xs, ys = _tie_heavy_series(rng, n)
        c = float(rng.choice([1.0, 0.5, 10.0, 3.0, 1e-4, 2.0 / 3.0]))
        a1 = np.zeros(64, np.uint8)
        a2 = np.zeros(64, np.uint8)
        d = ctypes.c_int(0)
        hc.ltx_dp_lazy(n, xs.ctypes.data_as(u8p), ys.ctypes.data_as(f64p), c,
                       a1.ctypes.data_as(u8p), ctypes.byref(d))
        hc.ltx_dp_exact(n, xs.ctypes.data_as(u8p), ys.ctypes.data_as(f64p), c,
                        a2.ctypes.data_as(u8p))
        if d.value:
            n_def += 1
            continue
        n_dec += 1
        assert _vertices(a1, n) == _vertices(a2, n), (list(xs), list(ys), c)
    print('lazy DP decided %d series, deferred %d' % (n_dec, n_def))
    assert n_dec > 4000


def test_rule_candidates_replay_gives_the_full_winner(hc):
    """lt_pixel.h RuleCands (the labels-only certified path): replaying match_rule's exact offers
    over the candidate set alone gives the winner of replaying every disturbance, for FD/GD/LD
    rules with onset/duration/pre_threshold filters, tie-heavy keys, init values straddling the
    threshold, and intervals of zero to large width around the exact values."""
    f64p, i32p = _abi.c_f64p, _abi.c_i32p
    hc.ltx_rule_cands.argtypes = [ctypes.c_int, i32p, i32p, f64p, f64p, f64p, f64p,
                                  ctypes.POINTER(_abi.LtRule), ctypes.c_int,
                                  ctypes.POINTER(ctypes.c_int)]
    rng = np.random.default_rng(17)
    n_cand = ctypes.c_int()
    sizes = []
    for case in range(6000):
        n = int(rng.integers(0, 20))
        on = np.sort(rng.choice(np.arange(1985, 2025), n, replace=False)).astype(np.int32)
        du = rng.integers(1, 4, n).astype(np.int32)
        init = rng.choice([100.0, 100.5, 250.0, 400.0], n) + rng.integers(-2, 3, n) * 0.25
        mag = rng.choice([-50.0, 0.0, 25.0, 25.0 + 2 ** -40, 80.0, 80.0], n)
        scale = [0.0, 2.0 ** -40, 1e-3, 0.3, 30.0][case % 5]
        w_init = rng.uniform(0, 1, n) * scale
        w_mag = rng.uniform(0, 1, n) * scale
        R = _abi.LtRule()
        R.change_type = int(rng.integers(1, 4))
        R.onset_op = int(rng.choice([_abi.LT_Q_UNSET, _abi.LT_Q_EQ, _abi.LT_Q_LE, _abi.LT_Q_GE]))
        R.onset_val = float(rng.integers(1990, 2020))
        R.duration_op = int(rng.choice([_abi.LT_Q_UNSET, _abi.LT_Q_GT, _abi.LT_Q_LT]))
        R.duration_val = float(rng.integers(1, 4))
        R.pre_op = int(rng.choice([_abi.LT_Q_UNSET, _abi.LT_Q_GT, _abi.LT_Q_LT]))
        R.pre_val = float(rng.choice([100.0, 100.5, 250.0]))
        mode = int(rng.choice([_abi.LT_PRE_REFERENCE, _abi.LT_PRE_DOCUMENTED]))
        args = [np.ascontiguousarray(a) for a in (on, du, init, mag, w_init, w_mag)]
        ok = hc.ltx_rule_cands(n, args[0].ctypes.data_as(i32p), args[1].ctypes.data_as(i32p),
                               *[a.ctypes.data_as(f64p) for a in args[2:]], ctypes.byref(R),
                               mode, ctypes.byref(n_cand))
        assert ok == 1, (case, n, R.change_type, R.onset_op, R.duration_op, R.pre_op, mode)
        sizes.append(n_cand.value)
    # exact intervals leave (nearly) one candidate per rule
    assert np.mean(sizes[0::5]) <= 1.5
