"""The whole local job on the GPU: setup -> parse -> analysis -> output on a
synthetic job directory (tests/jobfixture.py: tar.gz-compressed and plain int16 'ledaps' rasters,
cloudmasks, a shifted raster), against the oracle fed by a literal per-point parse_mapper, and
output rasters against a literal data2raster over the reducer's per-point emissions."""
import os

import numpy as np
import pytest

from land_trendr_amd import _abi, ingest, raster
from land_trendr_amd.geotiff import GeoTiff
from land_trendr_amd.job import LocalJob
from land_trendr_amd.scene import build_scene, parse_date
from land_trendr_amd.settings import compile_params
from oracle import oracle

from golden_io import _bits_equal
from jobfixture import SETTINGS, check_job_outputs, make_job

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('tile', [1 << 22, 50])
def test_local_job_end_to_end(tmp_path, tile):
    root = str(tmp_path)
    make_job(root)
    j = LocalJob(root, 'synth', device=0, tile_pixels=tile, on_error='skip')
    files = j.run()
    st = j.stack
    # oracle on the same observations: index 'B1 - B2' in int16 (the template type)
    idx = (st['bands'][:, 0, :].astype(np.int32) - st['bands'][:, 1, :]).astype(np.int16)
    meta = build_scene(st['dates'], parse_date(SETTINGS['target_date']))
    params, rules = compile_params(SETTINGS['line_cost'], SETTINGS['label_rules'])
    exp = oracle.analyze_tile(meta, params, idx.astype(np.float64), st['valid'], n_threads=8)
    bad = np.flatnonzero(exp['status'] & ~_abi.LT_ST_EMPTY)  # on_error='skip': nothing emitted
    exp['matched'][:, bad] = 0
    exp['winner'][:, bad] = -1
    for k, a in j.planes.items():
        e = exp[k][:a.shape[0]] if a.ndim == 2 else exp[k]
        if k in ('onset_year', 'duration', 'class_val', 'magnitude', 'initial_val'):
            m = exp['matched'][:a.shape[0]].astype(bool)
            a, e = np.where(m, a, 0), np.where(m, e, 0)
        if a.dtype.kind == 'f':
            assert _bits_equal(a, e).all(), k
        else:
            assert np.array_equal(a, e), k
    # label rasters: the literal data2raster over the '<rule>_<key>' emissions of every grid point
    tmpl = GeoTiff(j.rast_fns[0])
    gt = tmpl.geotransform()
    wkts = ingest.read_grid(j.grid_fn)
    ok_status = (exp['status'] & ~_abi.LT_ST_EMPTY) == 0
    for r, rule in enumerate(rules):
        for key in raster.LABEL_KEYS:
            holder = (np.ones((tmpl.height, tmpl.width), tmpl.dtype) * raster.NODATA).astype(
                tmpl.dtype.newbyteorder('='))
            for p, w in enumerate(wkts):
                if not (exp['matched'][r, p] and ok_status[p]):
                    continue
                val = rule.val if key == 'class_val' else exp[key][r, p]
                lng, lat = ingest.parse_point_wkt(w)
                x, y = ingest.get_pix_offsets_for_point(gt, lng, lat)
                holder[y, x] = float(val)
            name = '%s_%s' % (rule.name, key)
            got = GeoTiff(files[name][0]).read()[0]
            assert np.array_equal(got, raster.gdal_to_byte(holder)), name
    assert any(k.startswith('trendline/') for k in files)


@pytest.mark.parametrize('dtype', [np.int16, np.uint16])
def test_local_job_output_rasters_match_literal_data2raster(tmp_path, dtype):
    """Every output raster the GPU assembles (lt_raster_assemble), trendline/<date>-<attr> keys
    included, against a literal data2raster over the reducer's per-point emissions
    (jobfixture.literal_output_rasters; mr_land_trendr_job.py:108-152, utils.py:414-440), for an
    int16 and a uint16 template; tiles of 40 px so several tiles stream their trendline rows."""
    root = str(tmp_path)
    make_job(root, dtype=dtype)
    j = LocalJob(root, 'synth', device=0, tile_pixels=40, on_error='skip')
    files = j.run()
    assert GeoTiff(j.rast_fns[0]).dtype == np.dtype(dtype)
    check_job_outputs(j, files)


def test_local_job_raises_like_the_reference(tmp_path):
    """A pre_threshold rule in reference mode fails the job with AttributeError, as the
    reference's reducer does for the first pixel whose trendline has a disturbance."""
    root = str(tmp_path)
    s = dict(SETTINGS, label_rules=[{'name': 'gd', 'val': 3, 'change_type': 'GD',
                                     'pre_threshold': ['>', 500]}])
    make_job(root, settings=s)
    with pytest.raises(AttributeError):
        LocalJob(root, 'synth', device=0).run()
