"""Drop-in counterparts of the reference's hot-path functions (/root/reference/utils.py).

    analyze(pix_datas, line_cost, target_date) -> Trendline        utils.py:735-789
    change_labeling(trendline, label_rules) -> dict                utils.py:795-820
    analysis_reducer(point_wkt, pix_datas, settings) -> generator  mr_land_trendr_job.py:83-126
    analysis_reducer_batch(tile, settings) -> dense rasters        (the batched form of the above)

Same names, arguments, results and exception types as the reference; every number comes from
the HIP kernels of liblt_hip.so (one pixel per lane). The per-pixel functions exist for
drop-in compatibility; throughput comes from the batched tile path (analyze_tile).
"""
import datetime as _dt

import numpy as np
import torch

from . import _abi
from .classes import Disturbance, LabelRule, Trendline, TrendlinePoint
from .engine import ALL_FIELDS, LABELS, get_engine, label_tile
from .scene import build_scene, parse_date
from .settings import compile_params, load_settings

__all__ = ['parse_date', 'analyze', 'change_labeling', 'analysis_reducer',
           'analysis_reducer_batch', 'analyze_tile', 'index_tile', 'match_rules_gpu']


def _raise_for_status(status, n_obs_valid):
    """Raise what the reference raises for a pixel (classes.py:207)."""
    if status & _abi.LT_ST_FEB29:
        raise ValueError('day is out of range for month')
    if status & _abi.LT_ST_EMPTY:
        raise IndexError('index 0 is out of bounds for axis 0 with size 0')
    if status & _abi.LT_ST_SINGLE_YEAR:
        raise ValueError('Length of values (2) does not match length of index (1)')
    if status & _abi.LT_ST_NUMERIC:
        raise FloatingPointError('least-squares path outside the emulated LAPACK range')


def analyze_tile(scene, params, values, valid=None, fields=ALL_FIELDS, out=None, device=None):
    """Batched analyze + label of a pixel tile on the GPU (see Engine.analyze_tile)."""
    return get_engine(device).analyze_tile(scene, params, values, valid, fields, out)


def analyze(pix_datas, line_cost, target_date):
    """utils.analyze: [{'date': 'YYYY-MM-DD', 'val': v}, ...] -> Trendline."""
    pix_datas = list(pix_datas)
    dates = [parse_date(d['date']) for d in pix_datas]
    vals = [float(d['val']) for d in pix_datas]
    if not vals:  # pick_winners -> [] then despike indexes an empty series (utils.py:569)
        raise IndexError('index 0 is out of bounds for axis 0 with size 0')
    scene = build_scene(dates, target_date)
    eng = get_engine()
    v = torch.tensor(vals, dtype=torch.float64).reshape(len(vals), 1).to(eng.device)
    params, _ = compile_params(line_cost)
    fields = ('winner', 'val_raw', 'val_fit', 'fit_m', 'fit_b', 'right_m', 'right_b', 'spike',
              'vertex', 'status', 'n_years')
    out = eng.analyze_tile(scene, params, v, None, fields)
    host = {k: t.cpu().numpy() for k, t in out.items()}
    _raise_for_status(int(host['status'][0]), len(vals))
    points = []
    y0 = None
    for y in range(scene.n_years):
        w = int(host['winner'][y, 0])
        if w < 0:
            continue
        yr = int(scene.years[y])
        if y0 is None:
            y0 = yr
        points.append(TrendlinePoint(
            val_raw=float(host['val_raw'][y, 0]), val_fit=float(host['val_fit'][y, 0]),
            eqn_fit=(float(host['fit_m'][y, 0]), float(host['fit_b'][y, 0])),
            eqn_right=(float(host['right_m'][y, 0]), float(host['right_b'][y, 0])),
            index_date=dates[w].strftime('%Y-%m-%d'), index_day=yr - y0,
            spike=bool(host['spike'][y, 0]), vertex=bool(host['vertex'][y, 0])))
    return Trendline(points)


def match_rules_gpu(trendline, rules, pre_threshold_mode='reference'):
    """Trendline.match_rule for each rule, on the GPU label stage. -> [Disturbance | None]."""
    rules = [r if isinstance(r, LabelRule) else LabelRule(r) for r in rules]
    params, _ = compile_params(0.0, rules, pre_threshold_mode)
    pts = trendline.points
    eng = get_engine()
    if not pts:
        return [None] * len(rules)
    years = [parse_date(p.index_date).year for p in pts]
    vf = torch.tensor([[float(p.val_fit)] for p in pts], dtype=torch.float64).to(eng.device)
    vx = torch.tensor([[1 if p.vertex else 0] for p in pts], dtype=torch.uint8).to(eng.device)
    out = label_tile(eng, years, params, vf, vx)
    host = {k: t.cpu().numpy() for k, t in out.items()}
    if int(host['status'][0]) & _abi.LT_ST_PRE_THRESHOLD_ATTR:
        raise AttributeError("LabelRule instance has no attribute 'threshold'")
    res = []
    for r in range(len(rules)):
        if not host['matched'][r, 0]:
            res.append(None)
            continue
        res.append(Disturbance(int(host['onset_year'][r, 0]), float(host['initial_val'][r, 0]),
                               float(host['magnitude'][r, 0]), int(host['duration'][r, 0])))
    return res


def change_labeling(pix_trendline, label_rules, pre_threshold_mode='reference'):
    """utils.change_labeling: {rule.name: {class_val, onset_year, magnitude, duration}} for the
    rules the trendline matches."""
    label_rules = list(label_rules)
    matches = match_rules_gpu(pix_trendline, label_rules, pre_threshold_mode)
    labels = {}
    for rule, match in zip(label_rules, matches):
        if match:
            labels[rule.name] = {'class_val': rule.val, 'onset_year': match.onset_year,
                                 'magnitude': match.magnitude, 'duration': match.duration}
    return labels


def analysis_reducer(point_wkt, pix_datas, settings, pre_threshold_mode='reference'):
    """MRLandTrendrJob.analysis_reducer (mr_land_trendr_job.py:83-126) for one grid point:
    yields ('trendline/<date>-<attr>', {...}) for every point, then ('<label>_<field>', {...})."""
    settings = load_settings(settings)
    pix_trendline = analyze(list(pix_datas), settings['line_cost'],
                            parse_date(settings['target_date']))
    for label, val in pix_trendline.mr_label_output().items():
        yield 'trendline/%s' % label, {'pix_ctr_wkt': point_wkt, 'value': val}
    label_rules = [LabelRule(lr) for lr in settings['label_rules']]
    change_labels = change_labeling(pix_trendline, label_rules, pre_threshold_mode)
    for label_name, data in change_labels.items():
        for key in ['class_val', 'onset_year', 'magnitude', 'duration']:
            yield '%s_%s' % (label_name, key), {'pix_ctr_wkt': point_wkt, 'value': data[key]}


def analysis_reducer_batch(dates, values, valid, settings, fields=LABELS + ('status',),
                           pre_threshold_mode='reference', device=None, bands=None,
                           band_numbers=None):
    """Batched analysis_reducer: a co-registered tile (obs `dates`, values [K, P] — float64 or
    an index raster in its stored type — valid [K, P] uint8 or None, on the GPU) -> dict of dense
    output planes (GPU tensors): the label rasters the reference emits per grid point as
    '<label>_<field>' values, and, when requested, the trendline planes
    ('trendline/<date>-<attr>' values, per year slot).

    bands: instead of values, the raw band planes [K, n_bands, P] (their dtype is the raster's);
    settings['index_eqn'] is then evaluated on the GPU first (parse_mapper's rast_algebra,
    mr_land_trendr_job.py:67-68). band_numbers: the reference band number of each plane (default
    1..n_bands)."""
    settings = load_settings(settings)
    scene = build_scene(dates, parse_date(settings['target_date']))
    params, rules = compile_params(settings['line_cost'], settings.get('label_rules', ()),
                                   pre_threshold_mode)
    if bands is not None:
        values = index_tile(settings['index_eqn'], bands, band_numbers, device=device)
    out = analyze_tile(scene, params, values, valid, fields, device=device)
    out['_scene'] = scene
    out['_rules'] = rules
    return out


def index_tile(index_eqn, bands, band_numbers=None, device=None):
    """rast_algebra (utils.py:447-484) on the GPU: bands [K, n_bands, P] (the raster's dtype) ->
    the index raster [K, P] in the same dtype (array2raster's template type, utils.py:396-397)."""
    from .index_eqn import IndexProgram
    eng = get_engine(device)
    nb = bands.shape[1]
    numbers = list(band_numbers) if band_numbers is not None else list(range(1, nb + 1))
    prog = IndexProgram(index_eqn, band_dtype=np.dtype(str(bands.dtype).replace('torch.', '')),
                        raster_count=max(numbers))
    slots = [numbers.index(b) for b in prog.bands]  # the planes the equation reads, in order
    sel = bands[:, slots, :] if slots != list(range(nb)) else bands
    return eng.index_tile(eng.compile_index(prog), sel.contiguous() if sel.stride(2) != 1 else sel)
