"""A synthetic job directory laid out like the reference's S3 job (settings.py:19-25), for the
ingest / job tests: int16 two-band 'ledaps' rasters (B1 = B2 + index, synth.make_scene), some
tar.gz-compressed as the reference stores them, cloudmask rasters for some dates, and one raster
with a shifted geotransform so that grid points fall off it (and wrap, pt2val's numpy indexing)."""
import io
import json
import os
import tarfile

import numpy as np

from land_trendr_amd.raster import write_geotiff
from land_trendr_amd.synth import make_scene

GT = (500000.0, 30.0, 0.0, 4200000.0, 0.0, -30.0)
SETTINGS = {'index_eqn': 'B1 - B2', 'line_cost': 10, 'target_date': '2014-07-01',
            'label_rules': [{'name': 'fd', 'val': 2, 'change_type': 'FD',
                             'onset_year': ['>=', 1990]},
                            {'name': 'gd', 'val': 3, 'change_type': 'GD'},
                            {'name': 'ld', 'val': 4, 'change_type': 'LD',
                             'duration': ['>', 2]}]}


def make_job(root, job='synth', rows=9, cols=13, n_years=12, seed=5, settings=SETTINGS,
             dtype=np.int16):
    """dtype: the rasters' sample type (int16, or uint16: the int16 bands' bits, so negative B1
    values wrap, and so does the index 'B1 - B2' computed in uint16)."""
    sc = make_scene(rows * cols, n_years=n_years, k_min=1, k_max=2, mask_prob=0.2, seed=seed,
                    with_bands=True)
    rdir = os.path.join(root, job, 'input', 'rasters')
    os.makedirs(rdir, exist_ok=True)
    with open(os.path.join(root, job, 'input', 'settings.json'), 'w') as f:
        json.dump(settings, f)
    bands = sc.bands.numpy().astype(dtype)
    valid = sc.valid.numpy()
    names = []
    for k, d in enumerate(sc.dates):
        stem = 'LT5045029_%d_%03d_20120124_104859' % (d.year, d.timetuple().tm_yday)
        gt = GT
        if k == 3:  # shifted: the last 3 grid columns are off the raster (IndexError, skipped),
            # rows above it get negative offsets (numpy wraps them)
            gt = (GT[0] - 3 * GT[1], GT[1], 0.0, GT[3] + 2 * GT[5], 0.0, GT[5])
        # stored [bands, rows, cols]; grid point p = xoff * rows + yoff (rast2grid's order)
        img = bands[k].reshape(2, cols, rows).transpose(0, 2, 1)
        fn = os.path.join(rdir, stem + '_ledaps.tif')
        write_geotiff(fn, np.ascontiguousarray(img), geotransform=gt, nodata=None)
        if k % 3 == 1:  # compressed like the reference's S3 objects
            with tarfile.open(fn + '.tar.gz', 'w:gz') as tf:
                tf.add(fn, arcname=os.path.basename(fn))
            os.remove(fn)
            fn += '.tar.gz'
        if k % 2 == 0:
            m = valid[k].reshape(cols, rows).T.astype(np.uint8)
            write_geotiff(os.path.join(rdir, stem + '_cloudmask.tif'), np.ascontiguousarray(m),
                          geotransform=GT, nodata=None)
        names.append(os.path.basename(fn))
    return sc, names


def expected_index(stack):
    """rast_algebra's 'B1 - B2' in the rasters' own type (numpy integer arithmetic wraps), as the
    stack's band samples give it."""
    b = stack['bands']
    return (b[:, 0, :] - b[:, 1, :]).astype(b.dtype)


def literal_output_rasters(exp, rules, dates, wkts, tmpl, ok_status):
    """The reference's step-3 output for the emissions of analysis_reducer
    (mr_land_trendr_job.py:108-126) over the oracle's planes `exp`, reduced per key by a literal
    data2raster (utils.py:414-440): a holder of NODATA in the template's type as numpy 1.x
    promotes it (np.ones_like(template) * -99), float(value) assigned at each grid point's
    (y_off, x_off) in grid order (the last point wins), then GDAL's Byte conversion — restated by
    raster.gdal_to_byte, GDAL being absent here (parity unpinned). Keys: '<rule>_<field>' for
    matched rules and 'trendline/<winner date>-<attr>' (classes.py:84-116) for every present
    year of every pixel the reducer does not raise for."""
    from land_trendr_amd import ingest, raster
    gt = tmpl.geotransform()
    hdt = raster.holder_dtype(tmpl.dtype.newbyteorder('='))
    offs = []
    for w in wkts:
        lng, lat = ingest.parse_point_wkt(w)
        offs.append(ingest.get_pix_offsets_for_point(gt, lng, lat))
    holders = {}

    def emit(key, p, value):
        h = holders.get(key)
        if h is None:
            h = holders[key] = np.full((tmpl.height, tmpl.width), raster.NODATA, hdt)
        x, y = offs[p]
        h[y, x] = float(value)

    plane = {'val_raw': 'val_raw', 'val_fit': 'val_fit', 'eqn_fit_slope': 'fit_m',
             'eqn_fit_intercept': 'fit_b', 'eqn_right_slope': 'right_m',
             'eqn_right_intercept': 'right_b', 'spike': 'spike', 'vertex': 'vertex'}
    for p in range(len(wkts)):
        if not ok_status[p]:
            continue
        for yslot in range(exp['winner'].shape[0]):
            o = int(exp['winner'][yslot, p])
            if o < 0:
                continue
            d = dates[o].strftime('%Y-%m-%d')
            for attr, f in plane.items():
                v = exp[f][yslot, p]
                if attr in ('spike', 'vertex'):
                    v = 1 if v else 0
                emit('trendline/%s-%s' % (d, attr), p, v)
        for r, rule in enumerate(rules):
            if exp['matched'][r, p]:
                for key in raster.LABEL_KEYS:
                    emit('%s_%s' % (rule.name, key), p,
                         rule.val if key == 'class_val' else exp[key][r, p])
    return {k: raster.gdal_to_byte(h) for k, h in holders.items()}


def check_job_outputs(j, files):
    """Every output file of the finished job `j` against literal_output_rasters over the
    oracle's analysis of the job's stack; returns the oracle's planes."""
    from land_trendr_amd import _abi, ingest
    from land_trendr_amd.geotiff import GeoTiff
    from land_trendr_amd.scene import build_scene, parse_date
    from land_trendr_amd.settings import compile_params
    from oracle import oracle
    st = j.stack
    meta = build_scene(st['dates'], parse_date(SETTINGS['target_date']))
    params, rules = compile_params(SETTINGS['line_cost'], SETTINGS['label_rules'])
    exp = oracle.analyze_tile(meta, params, expected_index(st).astype(np.float64), st['valid'])
    ok_status = (exp['status'] & ~_abi.LT_ST_EMPTY) == 0
    tmpl = GeoTiff(j.rast_fns[0])
    want = literal_output_rasters(exp, rules, meta.dates, j.grid_wkts(), tmpl,
                                  ok_status)
    assert sorted(files) == sorted(want)
    for k, w in want.items():
        assert np.array_equal(GeoTiff(files[k][0]).read()[0], w), k
    # some acquisition date wins in some of the pixels but not all (two obs in its year)
    present = {}
    for p in np.flatnonzero(ok_status):
        for y in range(exp['winner'].shape[0]):
            o = exp['winner'][y, p]
            if o >= 0:
                present.setdefault(y, set()).add(int(o))
    assert any(len(v) > 1 for v in present.values())
    return exp
