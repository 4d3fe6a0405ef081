"""Generate the golden vectors under tests/golden/ by running the REFERENCE itself.

Survey container only (needs /root/reference; see ref_shim.py). Outputs are plain arrays
(np.savez_compressed, no pickles) + JSON, committed as fixtures; the GPU box only reads them.

Sets:
  lstsq.npz           12k segments -> reference least_squares (utils.py:584-598): slope, icpt, ssr
  scene_<name>.npz    synthetic / hand-built scenes -> reference analyze (utils.py:735) +
                      change_labeling (utils.py:795) per pixel, including the exception type for
                      pixels the reference rejects
  mr_output.json      Trendline.mr_label_output (classes.py:135-154) for a few pixels (key format)

Run: python tests/golden/make_golden.py   (≈2-3 min on 8 cores)
"""
import datetime as dt
import json
import multiprocessing as mp
import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
sys.path.insert(0, os.path.dirname(os.path.dirname(HERE)))

NAN = float('nan')


# ------------------------------------------------------------------------------------------------
# scene description helpers
# ------------------------------------------------------------------------------------------------
def scene_from_synth(name, n_pix, seed, line_cost, rules, target='2014-07-01', mode='reference',
                     **kw):
    from land_trendr_amd.synth import make_scene
    sc = make_scene(n_pix, seed=seed, **kw)
    valid = sc.valid.numpy() if sc.valid is not None else np.ones(sc.values.shape, np.uint8)
    return dict(name=name, dates=[d.isoformat() for d in sc.dates], values=sc.values.numpy(),
                valid=valid, line_cost=line_cost, rules=rules, target=target, mode=mode)


def scene_from_lists(name, pixels, line_cost, rules, target='2014-07-01', mode='reference'):
    """pixels: list of pix_datas lists [{'date','val'}] → union scene. An obs is keyed by
    (date, n-th occurrence of that date in the pixel); obs order = order of first appearance,
    pixel by pixel. Each pixel is valid only on its own obs. pick_winners' tie-break depends only
    on the input order inside a calendar year, which is checked to survive the union."""
    dates, key_index, P = [], {}, len(pixels)
    rows = []
    for p, pd_list in enumerate(pixels):
        seen = {}
        for d in pd_list:
            occ = seen.get(d['date'], 0)
            seen[d['date']] = occ + 1
            key = (d['date'], occ)
            if key not in key_index:
                key_index[key] = len(dates)
                dates.append(d['date'])
            rows.append((key_index[key], p, float(d['val'])))
    K = len(dates)
    values = np.zeros((K, P), np.float64)
    valid = np.zeros((K, P), np.uint8)
    last = {}
    for k, p, val in rows:
        yk = (p, dates[k][:4])
        assert last.get(yk, -1) < k, 'input order inside a year not representable'
        last[yk] = k
        values[k, p] = val
        valid[k, p] = 1
    return dict(name=name, dates=dates, values=values, valid=valid, line_cost=line_cost,
                rules=rules, target=target, mode=mode)


# ------------------------------------------------------------------------------------------------
# reference evaluation (worker processes)
# ------------------------------------------------------------------------------------------------
_REF = None


def _ref():
    global _REF
    if _REF is None:
        import ref_shim
        _REF = ref_shim.load_reference()
    return _REF


def _eval_pixel(args):
    """Run reference analyze + change_labeling on one pixel; return a plain dict."""
    pix_datas, line_cost, target, rules, mode = args
    utils, classes = _ref()
    out = {'err': '', 'points': [], 'labels': {}}
    try:
        tl = utils.analyze(pix_datas, line_cost, utils.parse_date(target))
    except Exception as e:  # the reference rejects this pixel
        out['err'] = type(e).__name__
        return out
    for p in tl.points:
        out['points'].append(dict(
            date=p.index_date, day=int(p.index_day), val_raw=float(p.val_raw),
            val_fit=float(p.val_fit), fit=(float(p.eqn_fit[0]), float(p.eqn_fit[1])),
            right=(float(p.eqn_right[0]), float(p.eqn_right[1])), spike=bool(p.spike),
            vertex=bool(p.vertex)))
    try:
        lrs = [classes.LabelRule(r) for r in rules]
        if mode == 'documented':
            for lr in lrs:  # instance patch, no source change
                lr.threshold = lr.pre_threshold
        labels = utils.change_labeling(tl, lrs)
        out['labels'] = {k: dict(class_val=v['class_val'], onset_year=int(v['onset_year']),
                                 magnitude=float(v['magnitude']), duration=int(v['duration']))
                         for k, v in labels.items()}
    except Exception as e:
        out['err'] = 'label:' + type(e).__name__
    return out


def evaluate_scene(sc, pool):
    dates = sc['dates']
    K, P = sc['values'].shape
    jobs = []
    for p in range(P):
        pdl = [{'date': dates[k], 'val': float(sc['values'][k, p])} for k in range(K)
               if sc['valid'][k, p]]
        jobs.append((pdl, sc['line_cost'], sc['target'], sc['rules'], sc['mode']))
    res = pool.map(_eval_pixel, jobs, chunksize=4)
    years = sorted({int(d[:4]) for d in dates})
    Y, R = len(years), len(sc['rules'])
    yidx = {y: i for i, y in enumerate(years)}
    f = lambda: np.full((Y, P), NAN)
    o = dict(winner=np.full((Y, P), -1, np.int16), index_day=np.full((Y, P), -1, np.int16),
             val_raw=f(), val_fit=f(), fit_m=f(), fit_b=f(), right_m=f(), right_b=f(),
             spike=np.zeros((Y, P), np.uint8), vertex=np.zeros((Y, P), np.uint8),
             matched=np.zeros((R, P), np.uint8), onset_year=np.full((R, P), -99, np.int32),
             duration=np.full((R, P), -99, np.int32), magnitude=np.full((R, P), -99.0),
             class_val=np.full((R, P), -99, np.int32))
    errs = []
    for p, r in enumerate(res):
        errs.append(r['err'])
        for pt in r['points']:
            y = yidx[int(pt['date'][:4])]
            # winner obs id: first valid obs of this pixel with that date and value (input order)
            w = next(k for k in range(K) if sc['valid'][k, p] and dates[k] == pt['date']
                     and float(sc['values'][k, p]) == pt['val_raw'])
            o['winner'][y, p] = w
            o['index_day'][y, p] = pt['day']
            o['val_raw'][y, p] = pt['val_raw']
            o['val_fit'][y, p] = pt['val_fit']
            o['fit_m'][y, p], o['fit_b'][y, p] = pt['fit']
            o['right_m'][y, p], o['right_b'][y, p] = pt['right']
            o['spike'][y, p] = pt['spike']
            o['vertex'][y, p] = pt['vertex']
        for ri, rule in enumerate(sc['rules']):
            lab = r['labels'].get(rule['name'])
            if lab:
                o['matched'][ri, p] = 1
                o['class_val'][ri, p] = lab['class_val']
                o['onset_year'][ri, p] = lab['onset_year']
                o['duration'][ri, p] = lab['duration']
                o['magnitude'][ri, p] = lab['magnitude']
    meta = dict(name=sc['name'], dates=dates, years=years, line_cost=sc['line_cost'],
                rules=sc['rules'], target=sc['target'], mode=sc['mode'])
    np.savez_compressed(os.path.join(HERE, 'scene_%s.npz' % sc['name']),
                        meta=np.array(json.dumps(meta)), values=sc['values'], valid=sc['valid'],
                        err=np.array(errs), **o)
    n_err = sum(1 for e in errs if e)
    print('scene %-12s P=%5d K=%3d Y=%2d errors=%d' % (sc['name'], P, K, Y, n_err), flush=True)
    return res


# ------------------------------------------------------------------------------------------------
# lstsq vectors
# ------------------------------------------------------------------------------------------------
def _lstsq_case(args):
    x, y = args
    import pandas as pd
    utils, _ = _ref()
    (m, c), ssr = utils.least_squares(pd.Series(y, index=x))
    return float(m), float(c), float(ssr)


def make_lstsq(pool, n=12000, seed=11):
    rng = np.random.default_rng(seed)
    M = 40
    xs = np.zeros((n, M), np.float64)
    ys = np.zeros((n, M), np.float64)
    ms = np.zeros(n, np.int32)
    jobs = []
    for t in range(n):
        m = int(rng.integers(2, M + 1))
        x = np.sort(rng.choice(np.arange(0, 45), m, replace=False)).astype(np.float64)
        kind = t % 4
        if kind == 0:
            y = rng.integers(-500, 1500, m).astype(np.float64)
        elif kind == 1:
            y = rng.normal(500, 300, m)
        elif kind == 2:
            y = np.round(rng.normal(0, 40, m)) + np.arange(m) * rng.integers(-50, 50)
        else:  # small integers: many exact rational ties in the DP
            y = rng.integers(0, 4, m).astype(np.float64) * 100
        xs[t, :m], ys[t, :m], ms[t] = x, y, m
        jobs.append((x.astype(np.int64), y))
    out = np.array(pool.map(_lstsq_case, jobs, chunksize=64))
    np.savez_compressed(os.path.join(HERE, 'lstsq.npz'), m=ms, x=xs, y=ys, slope=out[:, 0],
                        icpt=out[:, 1], ssr=out[:, 2])
    print('lstsq cases', n, flush=True)


# ------------------------------------------------------------------------------------------------
# hand-built edge / known-answer scenes
# ------------------------------------------------------------------------------------------------
def yearly(vals, y0=2010, md='12-31'):
    return [{'date': '%d-%s' % (y0 + i, md), 'val': float(v)} for i, v in enumerate(vals)]


def edge_pixels():
    px = []
    # reference known-answer tests (tests/utils_test.py:161-189, classes_test.py:35-62)
    px.append(yearly([10, 10, 10, 5, 5, 5, 7, 9, 10, 10]))          # TrendLineTestCase.test_match
    px.append(yearly([1, 1, 1, 5, 1, 1, 1]))                          # test_despike #1
    px.append(yearly([1, 3, 1, 5, 1, 1, 1]))                          # test_despike #2
    px.append(yearly([0, 0, 0, 1, 2, 3]))                             # test_segmented_least_squares
    px.append(yearly([0, 0, 0, 1, 1, 1, 3, 3]))
    px.append(yearly([1, 2, 3, 4, 5, 7, 9, 11, 13, 15]))              # test_analyze_simple data
    px.append(yearly([1, 2, 3, 4, 1000, 7, 9, 11, 13, 15]))           # test_analyze_simple_spike
    # sizes
    px.append(yearly([100, 50]))                                      # T = 2
    px.append(yearly([100, 50, 75]))                                  # T = 3
    px.append(yearly([5]))                                            # T = 1 -> ValueError
    px.append([])                                                     # empty -> IndexError
    px.append(yearly([7] * 12))                                       # constant
    px.append(yearly([-300, -250, -900, -100, -120, -500, 40, 0]))    # negative / zero values
    px.append(yearly([1e6, 2e6, 1.5e6, 3e6, 2.5e6, 1e6]))             # large values
    px.append(yearly([0.125, 0.5, 0.25, 0.75, 0.5]))                  # fractional values
    # gap years: x offsets non-contiguous
    px.append([{'date': '%d-07-01' % y, 'val': float(v)} for y, v in
               zip([1990, 1991, 1995, 1996, 1997, 2003, 2004, 2010],
                   [500, 520, 300, 340, 380, 600, 610, 200])])
    # pick_winners ties: input order decides among equidistant obs (target 07-01)
    px.append([{'date': '2001-07-02', 'val': 10.0}, {'date': '2001-06-30', 'val': 20.0},
               {'date': '2002-06-30', 'val': 30.0}, {'date': '2002-07-02', 'val': 40.0},
               {'date': '2003-07-01', 'val': 50.0}, {'date': '2003-07-01', 'val': 60.0},
               {'date': '2004-05-01', 'val': 70.0}, {'date': '2004-09-01', 'val': 80.0}])
    # obs in descending date order (the reference sorts winners by date)
    px.append([{'date': '%d-08-01' % y, 'val': float(v)} for y, v in
               zip(range(2012, 2000, -1), [5, 9, 3, 8, 8, 1, 0, 4, 7, 7, 2, 6])])
    # year-boundary distances (Dec 31 vs Jan 1 around the target month/day)
    px.append([{'date': '2005-01-01', 'val': 1.0}, {'date': '2005-12-31', 'val': 2.0},
               {'date': '2006-12-31', 'val': 3.0}, {'date': '2006-01-01', 'val': 4.0},
               {'date': '2007-06-15', 'val': 5.0}])
    return px


def tie_pixels(n, seed):
    """Small-integer series: exact rational SSE ties decided by LAPACK rounding."""
    rng = np.random.default_rng(seed)
    px = []
    for _ in range(n):
        T = int(rng.integers(8, 31))
        kind = rng.integers(0, 3)
        if kind == 0:
            v = rng.integers(0, 4, T) * 100
        elif kind == 1:
            v = np.cumsum(rng.integers(-1, 2, T)) * 50 + 500
        else:
            v = (np.arange(T) % int(rng.integers(2, 5))) * 100
        px.append(yearly(v.tolist(), y0=1990, md='07-01'))
    return px


GD = [{'name': 'gd', 'val': 1, 'change_type': 'GD'}]
C3_RULES = [
    {'name': 'fd', 'val': 2, 'change_type': 'FD', 'onset_year': ['>=', 1995],
     'duration': ['<', 4]},
    {'name': 'gd', 'val': 3, 'change_type': 'GD', 'pre_threshold': ['>', 500]},
    {'name': 'ld', 'val': 4, 'change_type': 'LD', 'duration': ['>', 2]},
]
EDGE_RULES = [
    {'name': 'gd', 'val': 1, 'change_type': 'GD'},
    {'name': 'fd', 'val': 2, 'change_type': 'FD', 'onset_year': ['<=', 2012]},
    {'name': 'ld', 'val': 3, 'change_type': 'LD', 'duration': ['>', 1]},
    {'name': 'any', 'val': 4, 'change_type': None, 'onset_year': ['=', 2013]},
    {'name': 'odd', 'val': 5, 'change_type': 'GD', 'onset_year': ['>', 2000],
     'duration': ['>=', 2]},   # qualifiers match_rule ignores: never filter
]


def main():
    n = max(1, min(8, os.cpu_count() or 1))
    with mp.Pool(n) as pool:
        make_lstsq(pool)
        scenes = [
            scene_from_synth('c1', 1000, 1, 10, GD, n_years=30),
            scene_from_synth('c3', 600, 3, 10, C3_RULES, mode='documented', n_years=30,
                             k_min=1, k_max=4, mask_prob=0.2),
            scene_from_synth('c3ref', 40, 3, 10, C3_RULES, mode='reference', n_years=30,
                             k_min=1, k_max=4, mask_prob=0.2),
            scene_from_synth('c5', 200, 5, 1.0, GD, n_years=40),
            scene_from_synth('lc05', 200, 6, 0.5, EDGE_RULES[:3], n_years=25),
            scene_from_synth('lc1000', 200, 7, 1000, GD, n_years=25),
            scene_from_lists('ties2', tie_pixels(300, 21), 2, EDGE_RULES[:3]),
            scene_from_lists('ties10', tie_pixels(300, 22), 10, GD),
            scene_from_lists('edge', edge_pixels(), 2, EDGE_RULES),
            scene_from_lists('edge_lc0', edge_pixels(), 0, EDGE_RULES),
            scene_from_lists('feb29', [
                [{'date': '%d-02-20' % y, 'val': float(v)} for y, v in
                 zip([1988, 1992, 1996, 2000, 2004], [5, 4, 9, 2, 2])],          # leap years only
                [{'date': '%d-03-01' % y, 'val': float(v)} for y, v in
                 zip([1996, 1997, 1998], [1, 2, 3])],                            # has non-leap
            ], 2, GD, target='2012-02-29'),
        ]
        res_c1 = None
        for sc in scenes:
            r = evaluate_scene(sc, pool)
            if sc['name'] == 'c1':
                res_c1 = (sc, r)
    # mr_label_output key format for a few pixels (classes.py:84-154)
    utils, classes = _ref()
    sc, _ = res_c1
    outs = []
    for p in range(3):
        pdl = [{'date': sc['dates'][k], 'val': float(sc['values'][k, p])}
               for k in range(sc['values'].shape[0])]
        tl = utils.analyze(pdl, 10, utils.parse_date('2014-07-01'))
        outs.append({k: float(v) for k, v in tl.mr_label_output().items()})
    with open(os.path.join(HERE, 'mr_output.json'), 'w') as fh:
        json.dump(dict(scene='c1', pixels=[0, 1, 2], outputs=outs), fh, indent=0, sort_keys=True)
    print('done')


if __name__ == '__main__':
    main()
