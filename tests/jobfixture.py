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


def make_job(root, job='synth', rows=9, cols=13, n_years=12, seed=5, settings=SETTINGS):
    sc = make_scene(rows * cols, n_years=n_years, k_min=1, k_max=2, mask_prob=0.2, seed=seed,
                    with_bands=True)
    rdir = os.path.join(root, job, 'input', 'rasters')
    os.makedirs(rdir, exist_ok=True)
    with open(os.path.join(root, job, 'input', 'settings.json'), 'w') as f:
        json.dump(settings, f)
    bands = sc.bands.numpy()
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
