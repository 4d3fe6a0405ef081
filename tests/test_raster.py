"""Output raster assembly (output_reducer / data2raster / array2raster) on the
CPU: the dense planes (from the oracle here; the GPU writes the same planes bit for bit, see
test_gpu_parity.py) assembled into the reference's per-key rasters, against a literal restatement
of data2raster's per-point loop; GeoTIFF write/read round trip on the reference's fixture."""
import os

import numpy as np

from land_trendr_amd import raster
from land_trendr_amd.classes import LabelRule
from land_trendr_amd.geotiff import GeoTiff
from land_trendr_amd.scene import build_scene, parse_date
from land_trendr_amd.settings import compile_params
from land_trendr_amd.synth import make_scene
from oracle import oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TIF = os.path.join(ROOT, 'tests', 'golden', 'files', 'dummy_single_band.tif')
RULES = [{'name': 'fd', 'val': 2, 'change_type': 'FD', 'onset_year': ['>=', 1995]},
         {'name': 'gd', 'val': 3, 'change_type': 'GD'}]


def _tile(rows=12, cols=17, seed=3):
    sc = make_scene(rows * cols, seed=seed, n_years=20, k_min=1, k_max=2, mask_prob=0.1)
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    params, rules = compile_params(10.0, RULES)
    out = oracle.analyze_tile(meta, params, sc.values.numpy(), sc.valid.numpy(), n_threads=8)
    return sc, meta, rules, out


# numpy 1.x value-based promotion of `template_array * -99` (the reference pins numpy 1.7.1,
# requirements.txt:7): -99 is an int8 scalar, so an unsigned template widens to the next signed type
_LEGACY_TIMES_NODATA = {np.dtype(np.int16): np.int16, np.dtype(np.float32): np.float32,
                        np.dtype(np.uint8): np.int16, np.dtype(np.uint16): np.int32,
                        np.dtype(np.int8): np.int8, np.dtype(np.uint32): np.int64}


def _data2raster_literal(points, shape, template_dtype):
    """utils.py:414-440 as written: holder = ones_like(template) * NODATA, holder[y, x] = float(v)
    (numpy's own assignment cast), then array2raster with data_type=compress=True: GDT_Byte."""
    holder = np.ones(shape, _LEGACY_TIMES_NODATA[np.dtype(template_dtype)]) * raster.NODATA
    for (y, x), v in points:
        holder[y, x] = float(v)
    return raster.gdal_to_byte(holder)


def test_label_rasters_reference_mode_matches_literal_data2raster():
    sc, meta, rules, out = _tile()
    rows, cols = 12, 17
    for tdt in (np.int16, np.float32, np.uint8, np.uint16):
        got = raster.label_rasters(out, rules, (rows, cols), template_dtype=tdt)
        for r, rule in enumerate(rules):
            for key in raster.LABEL_KEYS:
                # the reducer's emissions: only matched pixels yield '<rule>_<key>' values
                pts = []
                for p in range(rows * cols):
                    if out['matched'][r, p]:
                        v = rule.val if key == 'class_val' else out[key][r, p]
                        pts.append(((p // cols, p % cols), v))
                want = _data2raster_literal(pts, (rows, cols), tdt)
                assert np.array_equal(got['%s_%s' % (rule.name, key)], want), (tdt, key)


def test_holder_dtype_follows_numpy1_promotion():
    for tdt, want in _LEGACY_TIMES_NODATA.items():
        assert raster.holder_dtype(tdt) == np.dtype(want), tdt
    # an unsigned template keeps NODATA at -99, which GDAL's Byte conversion writes as 0
    out = raster.label_rasters({'matched': np.zeros((1, 4), np.uint8),
                                'class_val': np.zeros((1, 4), np.int32),
                                'onset_year': np.zeros((1, 4), np.int32),
                                'duration': np.zeros((1, 4), np.int32),
                                'magnitude': np.zeros((1, 4))},
                               [LabelRule({'name': 'gd', 'val': 1, 'change_type': 'GD'})],
                               (2, 2), template_dtype=np.uint16)
    assert (out['gd_onset_year'] == 0).all()


def test_label_rasters_typed_mode():
    sc, meta, rules, out = _tile()
    got = raster.label_rasters(out, rules, (12, 17), mode='typed')
    m = out['matched'][1].reshape(12, 17).astype(bool)
    assert got['gd_onset_year'].dtype == np.int32
    assert (got['gd_onset_year'][~m] == raster.NODATA).all()
    assert (got['gd_onset_year'][m] == out['onset_year'][1].reshape(12, 17)[m]).all()
    assert (got['gd_magnitude'][m] == out['magnitude'][1].reshape(12, 17)[m]).all()


def test_trendline_rasters_keys_follow_mr_label_output():
    sc, meta, rules, out = _tile(rows=4, cols=5)
    got = raster.trendline_rasters(out, meta, sc.dates, (4, 5), mode='typed')
    # every pixel contributes one key per winning date (classes.py:100-116)
    for p in range(20):
        for y in range(meta.n_years):
            w = out['winner'][y, p]
            if w < 0:
                continue
            d = sc.dates[w].strftime('%Y-%m-%d')
            v = got['trendline/%s-val_fit' % d][p // 5, p % 5]
            assert v == out['val_fit'][y, p] or (np.isnan(v) and np.isnan(out['val_fit'][y, p]))


def test_geotiff_write_read_round_trip_with_template_georeferencing(tmp_path):
    tmpl = GeoTiff(TIF)
    for dt in (np.uint8, np.int16, np.int32, np.float32, np.float64):
        a = (np.arange(45 * 54).reshape(45, 54) % 251).astype(dt)
        f = str(tmp_path / ('o_%s.tif' % np.dtype(dt).name))
        raster.write_geotiff(f, a, template=tmpl)
        g = GeoTiff(f)
        assert np.array_equal(g.read()[0], a) and g.read().dtype == dt
        assert g.pixel_scale == tmpl.pixel_scale and g.tiepoint == tmpl.tiepoint
        assert g.geokeys == tmpl.geokeys and g.nodata == raster.NODATA


def test_output_reducer_writes_every_key(tmp_path):
    sc, meta, rules, out = _tile(rows=45, cols=54)
    rasters = raster.label_rasters(out, rules, (45, 54))
    got = dict(raster.output_reducer(rasters, TIF, str(tmp_path), job='j1'))
    assert set(got) == set(rasters)
    for key, (path,) in got.items():
        assert path.endswith('j1/output/rasters/%s.tif' % key)
        assert np.array_equal(GeoTiff(path).read()[0], rasters[key])
