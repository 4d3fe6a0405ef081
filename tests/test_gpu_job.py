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
    wkts = j.grid_wkts()  # the planes' pixel order
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


def _gpu_job_worker(rank, world, port, root, result_path):
    """One rank of a multi-rank GPU job (every rank on cuda:0; gloo carries the label tiles)."""
    import torch
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    torch.cuda.set_device(0)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    j = LocalJob(root, 'synth', device=0, tile_pixels=10, on_error='skip')
    files = j.run()
    if rank == 0:
        arrs = {'raster:' + k: GeoTiff(v[0]).read() for k, v in files.items()}
        arrs.update({'plane:' + k: a for k, a in j.planes.items()})
        np.savez(result_path, **arrs)
    else:
        assert files is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_multi_rank_gpu_job_matches_single_rank(tmp_path):
    """The default GPU job path over 2 ranks on one GPU (gloo for the label exchange): fused
    'B1 - B2' load stage, mask bit planes, per-rank ingest, trendline rows streamed by
    TrendlineStream from a ring of three tiles' buffers into the ranks' shared host maps (tiles of
    10 px: six tiles per rank, nonzero offsets, every ring buffer reused). Every output raster and
    plane equals the single-rank GPU job's (the multi-rank job had CPU-only tests)."""
    import socket
    import torch.multiprocessing as mp
    multi, single = str(tmp_path / 'multi'), str(tmp_path / 'single')
    make_job(multi)
    make_job(single)
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    path = str(tmp_path / 'job.npz')
    mp.spawn(_gpu_job_worker, args=(2, port, multi, path), nprocs=2, join=True)
    got = dict(np.load(path))
    j = LocalJob(single, 'synth', device=0, tile_pixels=1 << 20, on_error='skip')
    files = j.run()
    assert sorted('raster:' + k for k in files) == sorted(k for k in got if k.startswith('raster:'))
    assert any(k.startswith('trendline/') for k in files)
    for k, v in files.items():
        assert np.array_equal(GeoTiff(v[0]).read(), got['raster:' + k]), k
    m = j.planes['matched'].astype(bool)
    for k, a in j.planes.items():
        b = got['plane:' + k]
        if k in ('onset_year', 'duration', 'class_val', 'magnitude', 'initial_val'):
            a, b = np.where(m[:a.shape[0]], a, 0), np.where(m[:a.shape[0]], b, 0)
        assert (_bits_equal(a, b).all() if a.dtype.kind == 'f' else np.array_equal(a, b)), k
