"""The compact trendline (lt_fast.h tl_split + lt_abi.hip trendline_expand_kernel, VERDICT r04
item 2): every per-year plane written from per-pixel vertex / spike / left-eqn words and segment
eqns by a separate store-only kernel must equal, bit for bit, what the year-major loop writes
(LT_TL_SPLIT=0) and what the oracle computes (eqns2fitted_points and the TrendlinePoint fields,
/root/reference/utils.py:646-722, classes.py:67-116): both series paths (binary64 observations on
the precompiled kernels, int16 bands with the program JIT-inlined), cloud masks, absent years,
spikes, pixels the reference raises for, tie-heavy line costs (deferred pixels: the resolve stage
writes their records) and a ragged last wave."""
import os

import numpy as np
import pytest
import torch

from land_trendr_amd import index_eqn
from land_trendr_amd.engine import ALL_FIELDS, Engine, valid_bytes
from land_trendr_amd.scene import build_scene, parse_date
from land_trendr_amd.settings import compile_params
from land_trendr_amd.synth import make_scene

pytestmark = pytest.mark.gpu


def _bits_equal(a, b):
    if a.dtype.kind == 'f':
        return (a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
    return a == b


@pytest.fixture(scope='module')
def engines():
    old = os.environ.get('LT_TL_SPLIT')
    os.environ['LT_TL_SPLIT'] = '0'
    ref = Engine(0)  # the year-major loop
    os.environ['LT_TL_SPLIT'] = '1'
    split = Engine(0)
    if old is None:
        del os.environ['LT_TL_SPLIT']
    else:
        os.environ['LT_TL_SPLIT'] = old
    yield ref, split
    ref.close()
    split.close()


CASES = [  # (years, k_min, k_max, mask_prob, line_cost, pixels, seed)
    (40, 1, 1, 0.0, 1.0, 20000 + 37, 5),      # c5's shape
    (30, 1, 4, 0.3, 10.0, 12000 + 5, 6),      # c3's shape: masks, absent years
    (30, 1, 2, 0.6, 1e-4, 8000 + 1, 7),       # ties (deferred pixels), T = 0 / 1 pixels
    (64, 1, 1, 0.1, 0.5, 4000 + 63, 8),       # 64 year slots
]


@pytest.mark.parametrize('case', CASES)
def test_compact_trendline_matches_year_major_and_oracle(engines, case):
    from oracle import oracle
    ref, split = engines
    Y, kmin, kmax, mp, lc, P, seed = case
    sc = make_scene(P, n_years=Y, k_min=kmin, k_max=kmax, mask_prob=mp, seed=seed)
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    params, _ = compile_params(lc, [{'name': 'gd', 'val': 1, 'change_type': 'GD'},
                                    {'name': 'fd', 'val': 2, 'change_type': 'FD'}])
    vals = sc.values.to(ref.device)
    valid = sc.valid.to(ref.device) if sc.valid is not None else None
    a = ref.analyze_tile(meta, params, vals, valid, ALL_FIELDS)
    b = split.analyze_tile(meta, params, vals, valid, ALL_FIELDS)
    torch.cuda.synchronize()
    for f in ALL_FIELDS:
        same = _bits_equal(a[f].cpu().numpy(), b[f].cpu().numpy())
        assert same.all(), (case, f, int((~same).sum()))
    rng = np.random.default_rng(seed)
    idx = np.sort(rng.choice(P, min(P, 3000), replace=False))
    want = oracle.analyze_tile(meta, params, sc.values[:, idx].numpy(),
                               None if sc.valid is None else sc.valid[:, idx].numpy(),
                               n_threads=min(os.cpu_count() or 1, 16))
    for f in ALL_FIELDS:
        g = b[f][..., idx].cpu().numpy()
        w = want[f][:g.shape[0]] if g.ndim == 2 else want[f]
        if f in ('class_val', 'onset_year', 'duration', 'magnitude', 'initial_val'):
            mt = want['matched'].astype(bool)[:g.shape[0]]
            g, w = np.where(mt, g, 0), np.where(mt, w, 0)
        assert _bits_equal(w, g).all(), (case, f)


def test_compact_trendline_jit_bands_matches_year_major(engines):
    """The JIT-fused path (int16 bands, 'B1 - B2' inlined, the module specialised with
    LT_SPEC_TL_SPLIT) in two tiles of one call, against the year-major loop."""
    from land_trendr_amd.engine import pack_valid_bits
    ref, split = engines
    outs = []
    for eng in (ref, split):
        sc = make_scene(2 * 9000 + 11, n_years=40, k_min=1, k_max=2, mask_prob=0.15, seed=9,
                        with_bands=True, band_layout='pixel')
        meta = build_scene(sc.dates, parse_date('2014-07-01'))
        params, _ = compile_params(1.0, [{'name': 'gd', 'val': 1, 'change_type': 'GD'}])
        fn = eng.compile_index(index_eqn.IndexProgram('B1 - B2', band_dtype='int16'))
        bands = sc.bands.to(eng.device)
        valid = pack_valid_bits(sc.valid.to(eng.device))
        h = bands.shape[-1] // 2
        tiles = [(bands[..., :h], valid[:, :h].contiguous()), (bands[..., h:], valid[:, h:].contiguous())]
        outs.append(eng.analyze_tiles(meta, params, tiles, ALL_FIELDS, index=fn))
    torch.cuda.synchronize()
    assert split.jit_stats()['jit_tiles'] >= 2
    for ta, tb in zip(*outs):
        for f in ALL_FIELDS:
            same = _bits_equal(ta[f].cpu().numpy(), tb[f].cpu().numpy())
            assert same.all(), (f, int((~same).sum()))
