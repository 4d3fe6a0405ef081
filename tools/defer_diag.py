"""Why pixels are deferred to the resolve stage (debugging aid, CPU only).

Runs the kernels' per-pixel pipeline compiled for the host (tests/native/lapack_host_check.hip:
lt_pixel.h analyze_pixel, the lazy DP of dp_lazy) over a synthetic scene of a bench config, and
for every pixel the lazy DP defers, classifies each ambiguous column on its backtracked path with
the reference's own binary64 values — each start i worth fl(fl(e + c) + OPT[i]), e the emulated
dgelsd residual (ltx_lstsq), OPT the exact-OPT DP — into:
  exact_tie    two or more starts attain the column minimum bit for bit (the first wins)
  near_tie     a unique minimum, but another start within the interval half-widths
and, for exact ties, what the tied starts are (1-2 point / collinear zero-residual segments, or
general segments, on the same or different OPT values). Prints one JSON object.

    python tools/defer_diag.py --config c2 --pixels 20000
"""
import argparse
import collections
import ctypes
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

from land_trendr_amd import _abi  # noqa: E402

HOSTCHECK = os.path.join(ROOT, 'tests', 'native', 'build', 'liblt_hostcheck.so')


def lib():
    L = ctypes.CDLL(HOSTCHECK)
    L.ltx_analyze_tile.argtypes = [ctypes.POINTER(_abi.LtScene), ctypes.POINTER(_abi.LtParams),
                                   ctypes.POINTER(_abi.LtTileIn), ctypes.POINTER(_abi.LtTileOut)]
    L.ltx_last_series.argtypes = [ctypes.c_void_p, ctypes.c_void_p]
    L.ltx_dp_lazy.restype = ctypes.c_uint64
    L.ltx_dp_lazy.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_double,
                              ctypes.c_void_p, ctypes.POINTER(ctypes.c_int)]
    L.ltx_lstsq.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int,
                            ctypes.c_void_p]
    return L


def ssr(L, xs, ys, i, j):
    """The reference's residual of points i..j: 0.0 for 1-2 points, else the emulated dgelsd's."""
    m = j - i + 1
    if m <= 2:
        return 0.0
    x = np.ascontiguousarray(xs[i:j + 1], np.float64)
    y = np.ascontiguousarray(ys[i:j + 1], np.float64)
    out = np.zeros(3)
    L.ltx_lstsq(m, x.ctypes.data, y.ctypes.data, 1, out.ctypes.data)
    return float(out[2])


def exact_dp(L, xs, ys, c):
    """The reference's DP values: OPT[j+1] = min_i fl(fl(e(i,j) + c) + OPT[i]), first minimum."""
    n = len(xs)
    OPT = [0.0] * (n + 1)
    vals = []
    for j in range(n):
        v = [(ssr(L, xs, ys, i, j) + c) + OPT[i] for i in range(j + 1)]
        b = min(range(j + 1), key=lambda i: (v[i], i))
        OPT[j + 1] = v[b]
        vals.append(v)
    return OPT, vals


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c2')
    ap.add_argument('--pixels', type=int, default=20000)
    ap.add_argument('--seed', type=int, default=0)
    ap.add_argument('--examples', type=int, default=8)
    a = ap.parse_args()
    import bench
    from land_trendr_amd.scene import build_scene, parse_date
    from land_trendr_amd.settings import compile_params
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    c = bench.CONFIGS[a.config]
    sc = make_scene(a.pixels, n_years=c['years'], k_min=c['k'][0], k_max=c['k'][1],
                    mask_prob=c['mask'], seed=a.seed or c['seed'])
    meta = build_scene(sc.dates, parse_date(bench.TARGET))
    params, _ = compile_params(c['line_cost'], c['rules'], c['mode'])
    L = lib()
    vals = np.ascontiguousarray(sc.values.numpy(), np.float64)
    valid = np.ascontiguousarray(sc.valid.numpy(), np.uint8) if sc.valid is not None else None
    K, P = vals.shape
    cost = c['line_cost']
    scn = meta.to_c()
    xs = np.zeros(64, np.uint8)
    ys = np.zeros(64, np.float64)
    arg = np.zeros(64, np.uint8)
    stats = collections.Counter()
    kinds = collections.Counter()
    examples = []
    for p in range(P):
        v1 = np.ascontiguousarray(vals[:, p:p + 1])
        m1 = np.ascontiguousarray(valid[:, p:p + 1]) if valid is not None else None
        out = oracle.alloc_outputs(meta.n_years, params.n_rules, 1)
        tin = _abi.LtTileIn()
        tin.n_pix, tin.stride = 1, 1
        tin.obs_val = v1.ctypes.data_as(_abi.c_f64p)
        tin.obs_valid = m1.ctypes.data_as(_abi.c_u8p) if m1 is not None else None
        o = oracle.out_struct(out, 1)
        L.ltx_analyze_tile(ctypes.byref(scn), ctypes.byref(params), ctypes.byref(tin),
                           ctypes.byref(o))
        n = L.ltx_last_series(xs.ctypes.data, ys.ctypes.data)
        if n < 1:
            stats['no_dp'] += 1
            continue
        d = ctypes.c_int(0)
        amb = L.ltx_dp_lazy(n, xs.ctypes.data, ys.ctypes.data, cost, arg.ctypes.data,
                            ctypes.byref(d))
        stats['pixels'] += 1
        stats['columns'] += n
        stats['amb_columns'] += bin(amb).count('1')
        if not d.value:
            continue
        stats['deferred'] += 1
        x, y = xs[:n].astype(int), ys[:n].copy()
        OPT, V = exact_dp(L, x, y, cost)
        # the backtracked path of the reference
        path, j = [], n - 1
        while j >= 0:
            v = V[j]
            b = min(range(j + 1), key=lambda i: (v[i], i))
            path.append((j, b))
            j = b - 1
        for j, b in path:
            if not (amb >> j) & 1:
                continue
            v = V[j]
            best = v[b]
            tied = [i for i in range(j + 1) if v[i] == best]
            if len(tied) > 1:
                def kind(i):
                    m = j - i + 1
                    if m <= 2:
                        return 'pt%d' % m
                    return 'zero' if ssr(L, x, y, i, j) == 0.0 else 'gen'
                ks = tuple(sorted(kind(i) for i in tied))
                same_opt = len({OPT[i] for i in tied}) == 1
                kinds['tie:' + '+'.join(ks) + (':sameOPT' if same_opt else ':diffOPT')] += 1
                stats['exact_tie_columns'] += 1
                if len(examples) < a.examples:
                    examples.append({'pixel': p, 'n': n, 'x': x.tolist(), 'y': y.tolist(),
                                     'column': j, 'tied_starts': tied,
                                     'tied_m': [j - i + 1 for i in tied],
                                     'opt_of_tied': [OPT[i] for i in tied], 'value': best,
                                     'ssr_of_tied': [ssr(L, x, y, i, j) for i in tied]})
            else:
                gap = min(v[i] - best for i in range(j + 1) if i != b) if j > 0 else float('inf')
                kinds['near_tie'] += 1
                stats['near_tie_columns'] += 1
                stats['near_tie_rel_gap_log2_sum'] += float(np.log2(gap / abs(best))) if gap > 0 else -60
    res = {'config': a.config, 'pixels': P, 'stats': dict(stats),
           'deferred_frac': stats['deferred'] / max(1, stats['pixels']),
           'ambiguous_columns_on_deferred_paths': dict(kinds), 'examples': examples}
    print(json.dumps(res, indent=1))


if __name__ == '__main__':
    main()
