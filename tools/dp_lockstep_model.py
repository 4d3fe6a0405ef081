"""The lazy DP's exit test in lockstep, modelled on the host (CPU only).

For every pixel of a synthetic scene of a bench config, the despiked compacted series comes from
the kernels' per-pixel pipeline compiled for the host (tests/native liblt_hostcheck.so, as
tools/defer_diag.py gets it); then each DP column is walked as the analyze kernel walks it —
starts j, j-1 (residual 0), then j-2, j-3, ... each priced with the closed-form SSE and followed by
the early-exit test (lt_pixel.h dp_start_bound with its screening slack, on exact OPT values) —
and the starts of >= 3 points priced before the exit are counted per lane and column. A wave of
64 consecutive pixels prices, per column, the largest count of its lanes. Prints the per-column
averages (lane mean vs wave maximum), the distributions, and what deferring every pixel that
needs more than B starts in some column would leave.

    python tools/dp_lockstep_model.py --config c2 --pixels 6400
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
sys.path.insert(0, os.path.join(ROOT, 'tools'))
sys.path.insert(0, os.path.join(ROOT, 'tests'))

K_SCREEN = 2.0 ** -30


def series_of(cfg, P):
    import bench
    import defer_diag as dd
    from land_trendr_amd import _abi
    from land_trendr_amd.scene import build_scene, parse_date
    from land_trendr_amd.settings import compile_params
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    c = bench.CONFIGS[cfg]
    sc = make_scene(P, n_years=c['years'], k_min=c['k'][0], k_max=c['k'][1],
                    mask_prob=c['mask'], seed=c['seed'])
    meta = build_scene(sc.dates, parse_date(bench.TARGET))
    params, _ = compile_params(c['line_cost'], c['rules'], c['mode'])
    L = dd.lib()
    vals = np.ascontiguousarray(sc.values.numpy(), np.float64)
    valid = np.ascontiguousarray(sc.valid.numpy(), np.uint8) if sc.valid is not None else None
    scn = meta.to_c()
    xs = np.zeros(64, np.uint8)
    ys = np.zeros(64, np.float64)
    out = []
    for p in range(P):
        v1 = np.ascontiguousarray(vals[:, p:p + 1])
        m1 = np.ascontiguousarray(valid[:, p:p + 1]) if valid is not None else None
        o = oracle.out_struct(oracle.alloc_outputs(meta.n_years, params.n_rules, 1), 1)
        tin = _abi.LtTileIn()
        tin.n_pix, tin.stride = 1, 1
        tin.obs_val = v1.ctypes.data_as(_abi.c_f64p)
        tin.obs_valid = m1.ctypes.data_as(_abi.c_u8p) if m1 is not None else None
        L.ltx_analyze_tile(ctypes.byref(scn), ctypes.byref(params), ctypes.byref(tin),
                           ctypes.byref(o))
        n = max(0, L.ltx_last_series(xs.ctypes.data, ys.ctypes.data))
        out.append((xs[:n].astype(np.int64).copy(), ys[:n].copy()))
    return out, c['line_cost']


def starts_per_column(x, y, cost):
    """Starts of >= 3 points the exit test lets through, per column (exact OPT)."""
    n = len(x)
    OPT = np.zeros(n + 1)
    K = np.zeros(n, int)
    syy_all = 0.0
    for j in range(n):
        syy_all += y[j] * y[j]
        slack = 4 * K_SCREEN * syy_all * (1 + 2 ** -49)
        sx = sxx = 0
        sy = sxy = syy = 0.0
        H = best = np.inf
        for i in range(j, -1, -1):
            sx += x[i]
            sxx += x[i] * x[i]
            sy += y[i]
            sxy += x[i] * y[i]
            syy += y[i] * y[i]
            m = j - i + 1
            e = 0.0
            if m >= 3:
                D = m * sxx - sx * sx
                e = max((m * syy - sy * sy) * D - (m * sxy - sx * sy) ** 2, 0.0) / (m * D)
            v = (e + cost) + OPT[i]
            w = (K_SCREEN * syy if m >= 3 else 0.0) + 2 ** -50 * abs(v)
            H = min(H, v + w)
            best = min(best, v)
            if m >= 3:
                K[j] += 1
                if (e + max(OPT[i], cost)) * (1 - 2 ** -49) - slack > H:
                    break
        OPT[j + 1] = best
    return K


def lockstep(Ks):
    tot_w = tot_l = cols = 0
    hist = collections.Counter()
    for w0 in range(0, len(Ks), 64):
        grp = Ks[w0:w0 + 64]
        nmax = max((len(k) for k in grp), default=0)
        for j in range(nmax):
            ks = [int(k[j]) for k in grp if j < len(k)]
            if not ks:
                continue
            tot_w += max(ks)
            tot_l += sum(ks) / len(ks)
            cols += 1
            hist[max(ks)] += 1
    return tot_w / max(cols, 1), tot_l / max(cols, 1), cols, hist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c2')
    ap.add_argument('--pixels', type=int, default=6400)
    a = ap.parse_args()
    series, cost = series_of(a.config, a.pixels)
    Ks = [starts_per_column(x, y, cost) for x, y in series]
    wave, lane, cols, hist = lockstep(Ks)
    allk = np.concatenate([k for k in Ks if len(k)])
    res = {'config': a.config, 'pixels': a.pixels, 'columns': cols,
           'wave_starts_per_column': round(wave, 3), 'lane_mean_starts_per_column': round(lane, 3),
           'wave_max_hist': {str(k): v for k, v in sorted(hist.items())},
           'lane_starts_hist': {str(k): int(v) for k, v in
                                sorted(collections.Counter(allk.tolist()).items())},
           'budget': {}}
    for B in (1, 2, 3, 4):
        keep = [k for k in Ks if len(k) == 0 or k.max() <= B]
        w, _, _, _ = lockstep(keep)
        res['budget'][str(B)] = {'deferred_frac': round(1 - len(keep) / len(Ks), 4),
                                 'wave_starts_per_column': round(w, 3)}
    # pixels regrouped into waves by a per-pixel key within blocks of G consecutive pixels (a
    # workgroup that sorts its pixels in LDS before the DP): the key 'total' is the lane's own
    # starts over all columns (known only after the DP: the bound of any such regrouping), the
    # others computable before it
    def rough(i):
        y = np.asarray(series[i][1], float)
        return float(np.sum((y[2:] - 2 * y[1:-1] + y[:-2]) ** 2)) if len(y) >= 3 else 0.0
    keys = {'total': lambda i: float(Ks[i].sum()) if len(Ks[i]) else 0.0,
            'roughness': rough, 'points': lambda i: float(len(series[i][1]))}
    res['sorted_blocks'] = {}
    for name, key in keys.items():
        for G in (256, 1024):
            order = []
            for g0 in range(0, len(Ks), G):
                order += sorted(range(g0, min(len(Ks), g0 + G)), key=key)
            res['sorted_blocks']['%s_G%d' % (name, G)] = round(
                lockstep([Ks[i] for i in order])[0], 3)
    print(json.dumps(res))


if __name__ == '__main__':
    main()
