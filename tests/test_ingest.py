"""Ingest and job orchestration on the CPU: the reference's own known-answer
tests for its string/grid/decompress helpers (tests/utils_test.py:14-41, :65-135) on its fixtures,
and the batched ingest against a literal per-point restatement of parse_mapper + apply_grid."""
import os
import shutil

import numpy as np
import pytest

from land_trendr_amd import ingest
from land_trendr_amd.geotiff import GeoTiff
from land_trendr_amd.job import LocalJob
from land_trendr_amd.raster import write_geotiff

from jobfixture import GT, make_job

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
FILES = os.path.join(ROOT, 'tests', 'golden', 'files')
TIF = os.path.join(FILES, 'dummy_single_band.tif')


# ---- utils_test.py known answers ----
def test_filename2date():
    assert ingest.filename2date('/tmp/4529_2012_222_ledaps.tif') == '2012-08-09'
    assert ingest.filename2date('LE7045029_1999_211_20120124_104859_cloudmask.tif.tar.gz') == \
        '1999-07-30'


def test_decompress(tmp_path):
    with pytest.raises(ValueError):
        ingest.decompress(os.path.join(FILES, 'dummy.csv'), str(tmp_path / 'invalid'))
    assert not os.path.exists(tmp_path / 'invalid')  # the partial dir is removed
    for name in ('dummy.tar.gz', 'dummy.zip'):
        d = str(tmp_path / name.replace('.', '_'))
        assert ingest.decompress(os.path.join(FILES, name), d) == [os.path.join(d, 'dummy.csv')]
        # an existing out_dir is returned as is (no second extraction)
        assert ingest.decompress(os.path.join(FILES, name), d) == [os.path.join(d, 'dummy.csv')]


def test_serialize_rast():
    assert next(ingest.serialize_rast(TIF)) == ('POINT(-2097378.06273 2642045.53514)',
                                                {'val': 16000.0})
    assert next(ingest.serialize_rast(TIF, {'date': '2013-01-30'})) == (
        'POINT(-2097378.06273 2642045.53514)', {'date': '2013-01-30', 'val': 16000.0})
    with pytest.raises(ValueError):  # the reference raises from GDAL for a non-raster
        next(ingest.serialize_rast(os.path.join(FILES, 'dummy.csv')))


def test_rast2grid_and_apply_grid(tmp_path):
    out = str(tmp_path / 'grid.csv')
    assert ingest.rast2grid(TIF, out) == out
    import pandas as pd
    wkts = pd.read_csv(out)['pix_ctr_wkt']
    assert len(wkts) == 2430
    assert wkts[0] == 'POINT(-2097378.06273 2642045.53514)'
    # the vectorised WKT column equals serialize_rast's per-pixel text
    assert list(wkts) == [w for w, _ in ingest.serialize_rast(TIF)]
    pix = list(ingest.apply_grid(TIF, out, {'x': 'y'}))
    assert len(pix) == 2430
    assert pix[0] == ('POINT(-2097378.06273 2642045.53514)', {'val': 16000.0, 'x': 'y'})


def test_py2_float_str():
    cases = {16000.0: '16000.0', -2097378.06273: '-2097378.06273', 0.1: '0.1', 1e20: '1e+20',
             123456789012345.0: '1.23456789012e+14', -0.0: '-0.0', 2642045.535140001: '2642045.53514',
             1e-5: '1e-05', 3.0: '3.0'}
    for v, s in cases.items():
        assert ingest.py2_float_str(v) == s, (v, ingest.py2_float_str(v), s)


def test_geotransform_roundtrip(tmp_path):
    g = GeoTiff(TIF)
    assert g.geotransform() == (-2097393.06273, 30.0, 0.0, 2642060.53514, 0.0, -30.0)
    a = np.arange(2 * 3 * 5, dtype=np.int16).reshape(2, 3, 5)
    fn = str(tmp_path / 'x.tif')
    write_geotiff(fn, a, geotransform=GT)
    h = GeoTiff(fn)
    assert h.geotransform() == GT
    assert np.array_equal(h.read(), a)


def test_pt2val_wraps_and_raises():
    arr = np.arange(12).reshape(3, 4)
    gt = (0.0, 1.0, 0.0, 0.0, 0.0, -1.0)
    assert ingest.pt2val(gt, 'POINT(-0.5 -0.5)', arr) == arr[0, 0]
    # int() truncates toward zero: x = -1.5 -> -1, which numpy wraps to the last column
    assert ingest.pt2val(gt, 'POINT(-1.5 -0.5)', arr) == arr[0, -1]
    with pytest.raises(IndexError):
        ingest.pt2val(gt, 'POINT(4.5 -0.5)', arr)
    lng = np.array([-0.5, -1.5, 4.5, -4.5, -5.5, 0.5])
    lat = np.array([-0.5, -0.5, -0.5, -2.5, -0.5, 3.5])
    idx, ok = ingest.grid_offsets(gt, arr.shape, lng, lat)
    for k in range(len(lng)):
        try:
            v = ingest.pt2val(gt, ingest.point_wkt(lng[k], lat[k]), arr)
            assert ok[k] and arr.reshape(-1)[idx[k]] == v
        except IndexError:
            assert not ok[k]


def _literal_parse(job, rast_fns, mask_fns, grid_fn):
    """parse_mapper per raster + the reducer's grouping, point by point (mr_land_trendr_job.py:
    47-81, utils.py:328-359, 447-484 with index_eqn 'B1 - B2' on int16 bands)."""
    per_point = {}
    for fn, mfn in zip(rast_fns, mask_fns):
        g = GeoTiff(fn)
        a = g.read()
        index = (a[0] - a[1]).astype(np.int16)  # Py2 numpy int16 arithmetic (wraps)
        tmp = fn + '.index.tif'
        write_geotiff(tmp, index, template=g)
        date = ingest.filename2date(fn)
        for wkt, d in ingest.apply_grid(tmp, grid_fn, {'date': date}, mask_fn=mfn):
            per_point.setdefault(wkt, []).append(d)
        os.remove(tmp)
    return per_point


def test_ingest_stack_matches_per_point_parse(tmp_path):
    root = str(tmp_path)
    make_job(root)
    j = LocalJob(root, 'synth')
    j.setup()
    assert any(m is not None for m in j.mask_fns) and any(m is None for m in j.mask_fns)
    st = j.parse()
    wkts = j.grid_wkts()  # the job's pixel order (raster order for a co-registered grid)
    literal = _literal_parse(j, j.rast_fns, j.mask_fns, j.grid_fn)
    idx = (st['bands'][:, 0, :].astype(np.int32) - st['bands'][:, 1, :]).astype(np.int16)
    n_dropped = 0
    for p, w in enumerate(wkts):
        got = [{'val': float(idx[k, p]), 'date': st['dates'][k]}
               for k in range(len(st['dates'])) if st['valid'][k, p]]
        assert got == literal.get(w, []), w
        n_dropped += len(st['dates']) - len(got)
    assert n_dropped > 0
    # the shifted raster drops some grid points and wraps others
    assert not st['valid'][3].all()


def test_grid_coords_equal_parsing_the_written_grid(tmp_path):
    """grid_coords (each distinct coordinate text parsed once) equals grid_points of the CSV
    rast2grid writes, bit for bit, on the reference's fixture and on a job raster."""
    out = str(tmp_path / 'grid.csv')
    ingest.rast2grid(TIF, out)
    for a, b in zip(ingest.grid_coords(TIF), ingest.grid_points(out)):
        assert a.dtype == b.dtype and np.array_equal(a.view(np.int64), b.view(np.int64))
    root = str(tmp_path / 'job')
    make_job(root)
    j = LocalJob(root, 'synth')
    j.setup()
    order = j.order if j.order is not None else slice(None)
    for a, b in zip(j.grid_xy, ingest.grid_points(j.grid_fn)):
        assert np.array_equal(a.view(np.int64), b[order].view(np.int64))
    assert j.order is not None  # the fixture's grid is its template's pixels: raster order
    # the threaded ingest from coordinates equals a serial one from the CSV
    st = ingest.ingest_stack(j.rast_fns, j.grid_xy, j.mask_fns, bands=[1, 2])
    st1 = ingest.ingest_stack(j.rast_fns, j.grid_fn, j.mask_fns, bands=[1, 2], threads=1)
    assert st['dates'] == st1['dates']
    assert np.array_equal(st['bands'], st1['bands'][..., order])
    assert np.array_equal(st['valid'], st1['valid'][..., order])
    # a rank's share (pixel ranges): exactly those columns, back to back; stack_range finds them
    P = st['n_pix']
    spans = [(0, 7), (P // 2, P // 2 + 13), (P - 5, P)]
    sub = ingest.ingest_stack(j.rast_fns, j.grid_xy, j.mask_fns, bands=[1, 2], pixels=spans)
    assert sub['n_pix'] == P and sub['bands'].shape[-1] == 25 == sub['valid'].shape[-1]
    assert [r[:2] for r in sub['ranges']] == spans
    for p0, p1 in spans + [(P // 2 + 3, P // 2 + 9)]:
        b, v = ingest.stack_range(sub, p0, p1)
        assert np.array_equal(b, st['bands'][:, :, p0:p1]) and np.array_equal(v, st['valid'][:, p0:p1])
    with pytest.raises(KeyError):
        ingest.stack_range(sub, 6, 9)  # straddles a range end
    empty = ingest.ingest_stack(j.rast_fns, j.grid_xy, j.mask_fns, bands=[1, 2], pixels=[])
    assert empty['bands'].shape[-1] == 0 and empty['dates'] == st['dates']


def test_job_setup_errors(tmp_path):
    os.makedirs(tmp_path / 'j' / 'input' / 'rasters')
    with pytest.raises(Exception, match='No analysis rasters'):
        LocalJob(str(tmp_path), 'j').setup()
    shutil.rmtree(tmp_path / 'j')


def test_grid_csv_writer_thread_reraises(tmp_path, monkeypatch):
    """A one-rank setup() writes the grid CSV on a thread beside parse(); a failure there reaches
    the caller at the first grid_fn access (and at output()), not silently."""
    import land_trendr_amd.job as jobmod
    root = str(tmp_path / 'job')
    make_job(root)

    def broken(*a, **k):
        raise OSError('disk full')
    monkeypatch.setattr(jobmod, 'rast2grid', broken)
    j = LocalJob(root, 'synth')
    j.setup()  # returns: the grid is still being written
    with pytest.raises(OSError, match='disk full'):
        j.grid_fn
    assert os.path.basename(j.grid_fn)  # joined once: the path itself afterwards
