"""GPU parity: the HIP kernels (through the C ABI) against the reference goldens and the oracle.

Bar: bit-exact for every integer and floating output; the north_star's 1e-9
relative tolerance for fitted values / magnitude is not needed because the emulated LAPACK
arithmetic reproduces the reference bits.
"""
import json
import os

import numpy as np
import pytest
import torch

import golden_io
from land_trendr_amd import _abi
from land_trendr_amd.scene import build_scene, parse_date
from land_trendr_amd.settings import compile_params

pytestmark = pytest.mark.gpu


@pytest.fixture(scope='module')
def engine():
    from land_trendr_amd.engine import get_engine
    return get_engine(0)


def _run(engine, g_scene, params, values, valid):
    dev = engine.device
    v = torch.from_numpy(np.ascontiguousarray(values)).to(dev)
    m = torch.from_numpy(np.ascontiguousarray(valid)).to(dev) if valid is not None else None
    out = engine.analyze_tile(g_scene, params, v, m)
    torch.cuda.synchronize()
    return {k: t.cpu().numpy() for k, t in out.items()}


@pytest.mark.parametrize('name', golden_io.scene_names())
def test_golden_scene_bit_exact(engine, name):
    g = golden_io.GoldenScene(name)
    out = _run(engine, g.scene, g.params, g.values, g.valid)
    bad = golden_io.compare(g, out)
    assert not bad, '\n'.join(bad[:40])


def _synthetic_vs_oracle(engine, n_pix, seed, line_cost, rules, mode, **kw):
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    sc = make_scene(n_pix, seed=seed, **kw)
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    params, _ = compile_params(line_cost, rules, mode)
    vals = sc.values.numpy()
    valid = sc.valid.numpy() if sc.valid is not None else None
    got = _run(engine, meta, params, vals, valid)
    want = oracle.analyze_tile(meta, params, vals, valid, n_threads=os.cpu_count() or 1)
    for f in want:
        a, b = want[f], got[f]
        if a.dtype.kind == 'f':
            same = (a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
        else:
            same = a == b
        assert same.all(), '%s: %d of %d differ' % (f, (~same).sum(), same.size)
    return got


def test_synthetic_c3_masks_vs_oracle(engine):
    rules = [{'name': 'fd', 'val': 2, 'change_type': 'FD', 'onset_year': ['>=', 1995],
              'duration': ['<', 4]},
             {'name': 'gd', 'val': 3, 'change_type': 'GD', 'pre_threshold': ['>', 500]},
             {'name': 'ld', 'val': 4, 'change_type': 'LD', 'duration': ['>', 2]}]
    got = _synthetic_vs_oracle(engine, 20000, 103, 10, rules, 'documented', n_years=30,
                               k_min=1, k_max=4, mask_prob=0.2)
    assert (got['status'] == 0).mean() > 0.99


def test_synthetic_c5_t40_low_cost_vs_oracle(engine):
    _synthetic_vs_oracle(engine, 8000, 105, 1.0, [{'name': 'gd', 'val': 1, 'change_type': 'GD'}],
                         'reference', n_years=40)


@pytest.mark.parametrize('kind', ['eighths', 'offset1e6', 'offset2e7', 'f32_noise', 'f64'])
def test_non_integer_and_large_offset_series_vs_oracle(engine, kind):
    """Values the integer generator never makes, through every path of the analyze stage:
    binary32-exact non-integers (k/8) and large offsets below 2^24 stay on the lazy binary32
    path; offsets above 2^24 with odd values and arbitrary doubles take the binary64 resolve
    (kDeferWide); small-variance noise on a large offset stresses the screening bound
    (tests/test_screening.py). Every output field bit-exact against the oracle."""
    import datetime as dt
    from oracle import oracle
    rng = np.random.default_rng(['eighths', 'offset1e6', 'offset2e7', 'f32_noise', 'f64'].index(
        kind) + 300)
    P, T = 4096, 30
    dates = [dt.date(1985 + t, 6, 15) for t in range(T)]
    base = np.round(rng.normal(0, 40, (T, P)))
    trend = np.where(np.arange(T)[:, None] > rng.integers(3, 25, P)[None, :], -300.0, 0.0)
    if kind == 'eighths':
        vals = (1000 + base + trend) + rng.integers(0, 8, (T, P)) / 8.0
    elif kind == 'offset1e6':
        vals = 1e6 + base + trend
    elif kind == 'offset2e7':
        vals = 2e7 + 1 + 2 * (base + trend)
    elif kind == 'f32_noise':
        vals = (5e5 + rng.normal(0, 1e-2, (T, P)) + trend).astype(np.float32).astype(np.float64)
    else:
        vals = rng.uniform(-1, 1, (T, P)) + trend / 300.0
    meta = build_scene(dates, parse_date('2014-07-01'))
    for lc in (10.0, 0.5):
        params, _ = compile_params(lc, [{'name': 'gd', 'val': 1, 'change_type': 'GD'},
                                        {'name': 'fd', 'val': 2, 'change_type': 'FD'}])
        got = _run(engine, meta, params, vals, None)
        want = oracle.analyze_tile(meta, params, vals, None, n_threads=os.cpu_count() or 1)
        for f in want:
            a, b = want[f], got[f]
            same = ((a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
                    if a.dtype.kind == 'f' else a == b)
            assert same.all(), (kind, lc, f, int((~same).sum()))


def test_two_scenes_on_two_streams_back_to_back(engine):
    """The context keeps one device copy of the scene metadata: a call with a new scene on
    another stream must not overwrite it while the previous call's kernels still read it."""
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    dev = engine.device
    scenes = []
    for seed, years in ((31, 30), (32, 24)):
        sc = make_scene(1 << 18, n_years=years, k_min=1, k_max=3, mask_prob=0.1, seed=seed)
        meta = build_scene(sc.dates, parse_date('2014-07-01'))
        scenes.append((sc, meta))
    params, _ = compile_params(10, [{'name': 'gd', 'val': 1, 'change_type': 'GD'}])
    streams = [torch.cuda.Stream(dev), torch.cuda.Stream(dev)]
    ins = [(sc.values.to(dev), sc.valid.to(dev)) for sc, _ in scenes]
    torch.cuda.synchronize()
    outs = []
    for (sc, meta), (v, m), st in zip(scenes, ins, streams):
        outs.append(engine.analyze_tile(meta, params, v, m, stream=st))  # no sync in between
    torch.cuda.synchronize()
    for (sc, meta), out in zip(scenes, outs):
        want = oracle.analyze_tile(meta, params, sc.values.numpy(), sc.valid.numpy(),
                                   n_threads=os.cpu_count() or 1)
        for f in ('status', 'matched', 'magnitude', 'val_fit', 'vertex', 'winner'):
            a, b = want[f], out[f].cpu().numpy()
            same = ((a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
                    if a.dtype.kind == 'f' else a == b)
            assert same.all(), (meta.n_years, f, int((~same).sum()))


def test_tie_heavy_small_integers_tiny_line_cost_vs_oracle(engine):
    """Small-integer series at line_cost 1e-4 (the reference tests' value) and 0.5: exact
    rational ties everywhere, singles/pairs on top of inexact OPT bases (provenance chains)."""
    from land_trendr_amd.synth import Scene
    from oracle import oracle
    import datetime as dt
    rng = np.random.default_rng(4242)
    P, T = 6000, 30
    dates = [dt.date(1990 + t, 7, 1) for t in range(T)]
    kind = rng.integers(0, 3, P)
    vals = np.where(kind[None, :] == 0, rng.integers(0, 4, (T, P)) * 100,
                    np.where(kind[None, :] == 1, np.cumsum(rng.integers(-1, 2, (T, P)), 0),
                             (np.arange(T)[:, None] % rng.integers(2, 5, P)[None, :]) * 7))
    vals = vals.astype(np.float64)
    meta = build_scene(dates, parse_date('2014-07-01'))
    for lc in (1e-4, 0.5):
        params, _ = compile_params(lc, [{'name': 'gd', 'val': 1, 'change_type': 'GD'},
                                        {'name': 'ld', 'val': 2, 'change_type': 'LD'}])
        got = _run(engine, meta, params, vals, None)
        want = oracle.analyze_tile(meta, params, vals, None, n_threads=os.cpu_count() or 1)
        for f in want:
            a, b = want[f], got[f]
            same = ((a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
                    if a.dtype.kind == 'f' else a == b)
            assert same.all(), (lc, f, int((~same).sum()))


@pytest.mark.parametrize('cfg', ['c2', 'c3', 'c5'])
def test_full_size_scene_sampled_vs_oracle(engine, cfg):
    """BASELINE.json sizes: a 7000x7000-pixel scene per config analysed on the GPU in 16.8 Mpx
    tiles (bench.py's default); 200,000 random pixels re-analysed by the oracle must agree bit
    for bit, every pixel's status must be 0 (no unemulated path), and the label rasters must be
    internally consistent (matched <=> class_val/onset/duration/magnitude set)."""
    import bench
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    c = bench.CONFIGS[cfg]
    P = c['pixels']
    sc = make_scene(P, n_years=c['years'], k_min=c['k'][0], k_max=c['k'][1],
                    mask_prob=c['mask'], seed=2024, device=engine.device)
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    params, _ = compile_params(c['line_cost'], c['rules'], c['mode'])
    fields = ('status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude',
              'val_fit', 'vertex')
    out = engine.alloc_outputs(meta.n_years, params.n_rules, P, fields)
    tile = 1 << 24
    spans = [(p0, min(P, p0 + tile)) for p0 in range(0, P, tile)]
    # one batched call, as bench.py makes it (tile t's resolve beside tile t+1's analyze)
    engine.analyze_tiles(meta, params,
                         [(sc.values[:, p0:p1], sc.valid[:, p0:p1] if sc.valid is not None
                           else None) for p0, p1 in spans], fields,
                         outs=[{f: t[..., p0:p1] for f, t in out.items()} for p0, p1 in spans])
    torch.cuda.synchronize()
    assert int((out['status'] != 0).sum()) == 0
    m = out['matched'].bool()
    assert bool(((out['class_val'] != -99) == m).all())
    assert bool(((out['duration'] > 0) | ~m).all())
    idx = torch.from_numpy(np.random.default_rng(7).choice(P, 200000, replace=False)).to(
        engine.device)
    vals = sc.values[:, idx].cpu().numpy()
    valid = sc.valid[:, idx].cpu().numpy() if sc.valid is not None else None
    want = oracle.analyze_tile(meta, params, vals, valid, n_threads=os.cpu_count() or 1)
    for f in fields:
        a, b = want[f], out[f][..., idx].cpu().numpy()
        same = ((a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
                if a.dtype.kind == 'f' else a == b)
        assert same.all(), (cfg, f, int((~same).sum()))
    del sc, out
    torch.cuda.empty_cache()


def test_strided_tile_and_subset_outputs(engine):
    """Tiles carved from a larger stack (stride > n_pix) and NULL outputs."""
    g = golden_io.GoldenScene('c1')
    dev = engine.device
    K, P = g.values.shape
    big = torch.zeros((K, P + 77), dtype=torch.float64, device=dev)
    big[:, :P] = torch.from_numpy(g.values).to(dev)
    view = big[:, :P]
    out = engine.analyze_tile(g.scene, g.params, view, None,
                              fields=('status', 'matched', 'magnitude'))
    torch.cuda.synchronize()
    mag = out['magnitude'].cpu().numpy()
    assert golden_io._bits_equal(mag, g.ref['magnitude']).all()
    assert (out['matched'].cpu().numpy() == g.ref['matched']).all()


# ---- drop-in API (land_trendr_amd.utils mirrors /root/reference/utils.py) ----

def test_reference_trendline_match_known_answer(engine):
    """classes_test.py:35-62 (TrendLineTestCase.test_match) through the drop-in API."""
    from land_trendr_amd import utils
    from land_trendr_amd.classes import LabelRule
    values = [{'date': '%d-12-31' % y, 'val': v} for y, v in
              zip(range(2010, 2020), [10, 10, 10, 5, 5, 5, 7, 9, 10, 10])]
    rule = LabelRule({'name': 'fast_dist', 'val': 2, 'change_type': 'GD',
                      'duration': ['<', 4]})
    tl = utils.analyze(values, 2, utils.parse_date('2014-07-01'))
    match = tl.match_rule(rule)
    assert match is not None
    assert match.onset_year == 2010
    assert round(match.initial_val - 10.999999999, 7) == 0
    assert round(match.magnitude - 6.3999999999999, 7) == 0
    assert match.duration == 3


def test_reference_despike_and_segments_known_answers(engine):
    """utils_test.py:161-189: despike flags and segmented-least-squares vertex lists."""
    from land_trendr_amd import utils
    t = utils.parse_date('2014-07-01')
    yearly = lambda vals: [{'date': '%d-12-31' % (2010 + i), 'val': v}
                           for i, v in enumerate(vals)]
    tl = utils.analyze(yearly([1, 1, 1, 5, 1, 1, 1]), 1e-4, t)
    assert [p.spike for p in tl.points] == [False, False, False, True, False, False, False]
    tl = utils.analyze(yearly([1, 3, 1, 5, 1, 1, 1]), 1e-4, t)
    assert [p.spike for p in tl.points] == [False, True, False, True, False, False, False]
    tl = utils.analyze(yearly([0, 0, 0, 1, 2, 3]), 0.0001, t)
    assert [p.index_day for p in tl.points if p.vertex] == [0, 2, 5]
    tl = utils.analyze(yearly([0, 0, 0, 1, 1, 1, 3, 3]), 0.0001, t)
    assert [p.index_day for p in tl.points if p.vertex] == [0, 3, 6, 7]


def test_mr_label_output_matches_reference(engine):
    from land_trendr_amd import utils
    with open(os.path.join(golden_io.GOLDEN, 'mr_output.json')) as fh:
        gold = json.load(fh)
    g = golden_io.GoldenScene(gold['scene'])
    for p, want in zip(gold['pixels'], gold['outputs']):
        pdl = [{'date': g.meta['dates'][k], 'val': float(g.values[k, p])}
               for k in range(g.values.shape[0])]
        tl = utils.analyze(pdl, 10, utils.parse_date('2014-07-01'))
        got = tl.mr_label_output()
        assert sorted(got) == sorted(want)
        for k in want:
            assert golden_io._bits_equal(float(got[k]), want[k]), k


def test_reference_error_types(engine):
    from land_trendr_amd import utils
    from land_trendr_amd.classes import LabelRule
    t = utils.parse_date('2014-07-01')
    with pytest.raises(IndexError):
        utils.analyze([], 10, t)
    with pytest.raises(ValueError):
        utils.analyze([{'date': '2001-07-01', 'val': 3.0}], 10, t)
    with pytest.raises(ValueError):
        utils.analyze([{'date': '2001-07-01', 'val': 3.0}, {'date': '2002-07-01', 'val': 3.0}],
                      10, utils.parse_date('2012-02-29'))
    with pytest.raises(ValueError):
        utils.analyze([{'date': '2001/07/01', 'val': 3.0}], 10, t)
    tl = utils.analyze([{'date': '%d-07-01' % y, 'val': float(y % 7)} for y in range(2000, 2010)],
                       10, t)
    rule = LabelRule({'name': 'x', 'val': 1, 'change_type': 'GD', 'pre_threshold': ['>', 5]})
    with pytest.raises(AttributeError):
        utils.change_labeling(tl, [rule])
    got = utils.change_labeling(tl, [rule], pre_threshold_mode='documented')
    assert isinstance(got, dict)


def test_analysis_reducer_key_format(engine):
    from land_trendr_amd import utils
    settings = {'line_cost': 10, 'target_date': '2014-07-01',
                'label_rules': [{'name': 'gd', 'val': 1, 'change_type': 'GD'}]}
    pdl = [{'date': '%d-07-01' % y, 'val': float(v)} for y, v in
           zip(range(2000, 2012), [500, 510, 505, 520, 300, 330, 360, 390, 420, 800, 450, 470])]
    out = list(utils.analysis_reducer('POINT(1 2)', pdl, settings))
    keys = [k for k, _ in out]
    assert keys[0] == 'trendline/2000-07-01-val_raw'
    assert len([k for k in keys if k.startswith('trendline/')]) == 12 * 8
    assert keys[-4:] == ['gd_class_val', 'gd_onset_year', 'gd_magnitude', 'gd_duration']
    assert all(v['pix_ctr_wkt'] == 'POINT(1 2)' for _, v in out)
    d = dict(out)
    assert d['gd_onset_year']['value'] == 2002 and d['gd_duration']['value'] == 2


def test_label_tile_matches_fused_labels(engine):
    """lt_label_tile on the fused kernel's own trendline planes gives the same labels."""
    from land_trendr_amd.engine import label_tile
    g = golden_io.GoldenScene('lc05')
    dev = engine.device
    out = engine.analyze_tile(g.scene, g.params, torch.from_numpy(g.values).to(dev),
                              torch.from_numpy(g.valid).to(dev))
    present = (out['winner'] >= 0).to(torch.uint8).contiguous()
    lab = label_tile(engine, g.scene.years, g.params, out['val_fit'], out['vertex'], present)
    torch.cuda.synchronize()
    for f in ('matched', 'onset_year', 'duration'):
        assert torch.equal(lab[f], out[f]), f
    a, b = lab['magnitude'].cpu().numpy(), out['magnitude'].cpu().numpy()
    assert golden_io._bits_equal(a, b).all()


def test_mixed_series_lengths_in_one_wave_vs_oracle(engine):
    """Every wave mixes pixels with 0..30 present years (heavy, varying cloud masks): numpy's
    pairwise-sum branches (n < 8 / n >= 8 with different n % 8), the despike scan and the
    compaction all run with per-lane lengths against the oracle."""
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    sc = make_scene(4096, seed=31, n_years=30, k_min=1, k_max=1, mask_prob=0.0)
    rng = np.random.default_rng(31)
    K, P = sc.values.shape
    keep_frac = rng.uniform(0.0, 1.0, P)  # per pixel: fraction of years kept
    valid = (rng.uniform(0.0, 1.0, (K, P)) < keep_frac[None, :]).astype(np.uint8)
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    params, _ = compile_params(10.0, [{'name': 'gd', 'val': 1, 'change_type': 'GD'}])
    vals = sc.values.numpy()
    got = _run(engine, meta, params, vals, valid)
    want = oracle.analyze_tile(meta, params, vals, valid, n_threads=os.cpu_count() or 1)
    ny = valid.sum(axis=0)
    assert len(np.unique(ny)) > 25  # lengths really mixed
    for f in want:
        a, b = want[f], got[f]
        same = ((a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
                if a.dtype.kind == 'f' else a == b)
        assert same.all(), '%s: %d of %d differ' % (f, (~same).sum(), same.size)


def test_analyze_tiles_batch_equals_single_tiles_and_oracle(engine):
    """lt_analyze_tiles (resolve of tile t on the side stream beside tile t+1's analyze, two
    deferred-list sets in turn) gives the single-tile results bit for bit, for uneven and empty
    tiles and more tiles than list sets, and agrees with the oracle."""
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    sc = make_scene(20000, n_years=30, k_min=1, k_max=2, mask_prob=0.1, seed=99,
                    device=engine.device)
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    params, _ = compile_params(1.0, [{'name': 'gd', 'val': 1, 'change_type': 'GD'},
                                     {'name': 'fd', 'val': 2, 'change_type': 'FD'}])
    cuts = [0, 7000, 7000, 7001, 13000, 20000]  # an empty tile and a one-pixel tile
    spans = list(zip(cuts[:-1], cuts[1:]))
    batch = engine.analyze_tiles(meta, params,
                                 [(sc.values[:, a:b], sc.valid[:, a:b]) for a, b in spans])
    single = [engine.analyze_tile(meta, params, sc.values[:, a:b], sc.valid[:, a:b])
              for a, b in spans]
    torch.cuda.synchronize()
    want = oracle.analyze_tile(meta, params, sc.values.cpu().numpy(), sc.valid.cpu().numpy(),
                               n_threads=os.cpu_count() or 1)
    for (a, b), ob, os_ in zip(spans, batch, single):
        for f in ob:
            x, y = ob[f].cpu().numpy(), os_[f].cpu().numpy()
            assert x.view(np.uint8).tobytes() == y.view(np.uint8).tobytes(), (a, b, f)
            if f in ('class_val', 'onset_year', 'duration', 'magnitude', 'initial_val'):
                continue  # unmatched slots hold no defined value
            w = want[f][..., a:b]
            same = ((w.view(np.int64) == x.view(np.int64)) | (np.isnan(w) & np.isnan(x))
                    if w.dtype.kind == 'f' else w == x)
            assert same.all(), (a, b, f, int((~same).sum()))


def _label_datasets():
    """(name, dates, values [K, P] float64, rules, mode) for the labels-only test below."""
    import datetime as dt
    rng = np.random.default_rng(777)
    T, P = 30, 4096
    dates = [dt.date(1990 + t, 7, 1) for t in range(T)]
    sets = []
    # small-integer plateaus: 2-point segments whose fitted values sit ON the pre_threshold
    # values and equal-magnitude disturbances (exact ties the closed form cannot order)
    kind = rng.integers(0, 3, P)
    v = np.where(kind[None, :] == 0, rng.integers(0, 4, (T, P)) * 100,
                 np.where(kind[None, :] == 1, np.cumsum(rng.integers(-1, 2, (T, P)), 0) * 50,
                          (np.arange(T)[:, None] % rng.integers(2, 5, P)[None, :]) * 100))
    rules = [{'name': 'gd', 'val': 1, 'change_type': 'GD', 'pre_threshold': ['>', 100]},
             {'name': 'fd', 'val': 2, 'change_type': 'FD', 'pre_threshold': ['<', 200]},
             {'name': 'ld', 'val': 3, 'change_type': 'LD', 'duration': ['<', 3],
              'pre_threshold': ['>', 0]},
             {'name': 'gd2', 'val': 4, 'change_type': 'GD', 'onset_year': ['>=', 2000]}]
    for lc in (1e-4, 0.5, 10.0):
        sets.append(('plateaus-lc%g' % lc, dates, v.astype(np.float64), lc, rules, 'documented'))
    sets.append(('plateaus-reference-mode', dates, v.astype(np.float64), 0.5, rules, 'reference'))
    # the synthetic generator's series (c2 shape) with three rules
    from land_trendr_amd.synth import make_scene
    sc = make_scene(P, n_years=T, seed=778)
    sets.append(('synthetic', sc.dates, sc.values.numpy(), 10.0, rules[:3], 'documented'))
    # non-integer and large-offset values (closed-form error scale)
    base = np.round(rng.normal(0, 40, (T, P)))
    trend = np.where(np.arange(T)[:, None] > rng.integers(3, 25, P)[None, :], -300.0, 0.0)
    sets.append(('eighths', dates, (1000 + base + trend) + rng.integers(0, 8, (T, P)) / 8.0, 0.5,
                 rules[:1], 'documented'))
    sets.append(('offset1e6', dates, 1e6 + base + trend, 10.0, rules[:1], 'documented'))
    return sets


@pytest.mark.parametrize('ds', range(7))
def test_labels_only_launch_matches_oracle_and_full_launch(engine, ds):
    """Labels-only launches take the certified path (closed-form vertex fits as intervals, the
    emulated fits only around the rules' candidates, lt_fast.h): their rule rasters and status must
    equal, bit for bit, the oracle's and those of a launch that also writes the trendline planes
    (every vertex fit emulated). Datasets aim at the certified path's decisions: equal-magnitude
    disturbances, fitted values equal to the pre_threshold values, FD/GD/LD rules with filters."""
    from oracle import oracle
    name, dates, vals, lc, rules, mode = _label_datasets()[ds]
    meta = build_scene(dates, parse_date('2014-07-01'))
    params, _ = compile_params(lc, rules, mode)
    fields = ('status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude',
              'initial_val')
    dev = engine.device
    v = torch.from_numpy(np.ascontiguousarray(vals)).to(dev)
    lab = engine.analyze_tile(meta, params, v, None, fields)
    full = engine.analyze_tile(meta, params, v, None)
    torch.cuda.synchronize()
    want = oracle.analyze_tile(meta, params, vals, None, n_threads=os.cpu_count() or 1)
    for f in fields:
        a, b, c = want[f], lab[f].cpu().numpy(), full[f].cpu().numpy()
        for got, what in ((b, 'labels-only vs oracle'), (c, 'full vs oracle')):
            same = ((a.view(np.int64) == got.view(np.int64)) | (np.isnan(a) & np.isnan(got))
                    if a.dtype.kind == 'f' else a == got)
            assert same.all(), (name, what, f, int((~same).sum()))


@pytest.mark.parametrize('name', golden_io.scene_names())
def test_golden_scene_as_float32_index_raster(engine, name):
    """Binary64 values take the binary64 analyze instance; a float32 index raster keeps the
    binary32 one. Every golden scene whose values binary32 holds exactly, fed as float32, must give
    the golden outputs too."""
    g = golden_io.GoldenScene(name)
    v32 = np.asarray(g.values, np.float64).astype(np.float32)
    if not np.array_equal(v32.astype(np.float64), np.asarray(g.values, np.float64),
                          equal_nan=True):
        pytest.skip('values not exact in binary32')
    out = _run(engine, g.scene, g.params, v32, g.valid)
    bad = golden_io.compare(g, out)
    assert not bad, '\n'.join(bad[:40])
