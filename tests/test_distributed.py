"""Multi-process (gloo, CPU) checks of the mosaic path bench.py and the job runner use:
distributed.Mosaic tiling, runner.MosaicRunner's per-rank pipeline and distributed.LabelExchange's
point-to-point sends to the writer, and the multi-rank local job (job.LocalJob: rank-0 setup, label
exchange, trendline rows through the shared host maps). The per-tile compute is the CPU oracle (test
infrastructure) behind a stand-in for the HIP engine (tests/engine_double.py); on a GPU job it is
liblt_hip.so."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from land_trendr_amd import distributed as ltd

from engine_double import OracleEngine

RULES = [{'name': 'gd', 'val': 1, 'change_type': 'GD'},
         {'name': 'fd', 'val': 2, 'change_type': 'FD', 'duration': ['<', 5]}]
FIELDS = ('status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude')


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(world, rank, scene_px, tile, assign, seed0, dist=None, dst=0, steps=1, overlap=False):
    from land_trendr_amd.engine import IndexFn
    from land_trendr_amd.index_eqn import IndexProgram
    from land_trendr_amd.runner import MosaicRunner
    from land_trendr_amd.settings import compile_params
    from land_trendr_amd.synth import mosaic_inputs
    m = ltd.Mosaic(scene_px, tile, world, rank, assign)
    items = mosaic_inputs(m, 20, 1, 2, 0.1, seed0, 'cpu')
    params, _ = compile_params(10, RULES)
    fn = IndexFn(None, IndexProgram('B1 - B2', band_dtype='int16'))
    r = MosaicRunner(OracleEngine(), m, params, items, FIELDS, fn, dist, dst=dst)
    for _ in range(steps):
        r.step(overlap=overlap)
    r.finish()
    return r


def _worker(rank, world, port, scene_px, tile, assign, result_path, dst=0, steps=1,
            overlap=False):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    r = _run(world, rank, scene_px, tile, assign, 7, dist, dst, steps, overlap)
    # the label planes travel narrowed (runner.label_wire_types) and arrive widened, exactly
    assert all(r.exchange.wire[f] == torch.int16 for f in ('class_val', 'onset_year', 'duration'))
    if overlap:  # the steps ran pipelined: some sends stayed in flight past their step
        assert r._overlap
    # bench.py's exchange check: the owners' per-tile checksums, all-reduced, equal the writer's
    tot = r.exchange.checksums(r.m.mine)
    dist.all_reduce(tot)
    if rank == dst:
        assert torch.equal(r.exchange.checksums(r.m.tiles), tot)
        np.savez(result_path, **{f: r.exchange.raster(f).numpy()
                                 for f in ltd.LABEL_GATHER_FIELDS})
    dist.barrier()
    dist.destroy_process_group()


def _want(scene_px, seed0):
    """Every scene of the mosaic analysed whole by the oracle, scenes back to back."""
    from land_trendr_amd.scene import build_scene, parse_date
    from land_trendr_amd.settings import compile_params
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    params, _ = compile_params(10, RULES)
    parts = []
    for s, n in enumerate(scene_px):
        sc = make_scene(n, n_years=20, k_min=1, k_max=2, mask_prob=0.1, seed=seed0 + s)
        meta = build_scene(sc.dates, parse_date('2014-07-01'))
        parts.append(oracle.analyze_tile(meta, params, sc.values.numpy(), sc.valid.numpy()))
    return {f: np.concatenate([p[f] for p in parts], axis=-1) for f in ltd.LABEL_GATHER_FIELDS}


def _same(a, b):
    if a.dtype.kind == 'f':
        return (a.view(np.int64) == b.view(np.int64)).all()
    return (a == b).all()


def test_label_wire_types_follow_the_rules_values():
    """onset_year / duration always travel as int16; class_val only when every rule's value
    (and LT_NODATA) fits, else in its API type; magnitude never narrows."""
    from land_trendr_amd.runner import label_wire_types
    from land_trendr_amd.settings import compile_params
    p, _ = compile_params(10, RULES)
    w = label_wire_types(p, ltd.LABEL_GATHER_FIELDS)
    assert w == {'class_val': torch.int16, 'onset_year': torch.int16, 'duration': torch.int16}
    big = [dict(RULES[0], val=40000)] + RULES[1:]
    p2, _ = compile_params(10, big)
    assert 'class_val' not in label_wire_types(p2, ltd.LABEL_GATHER_FIELDS)
    assert label_wire_types(p, ('magnitude',)) == {}


def test_tile_assignment_covers_mosaic_once():
    for px, tile, world, assign in [([1000], 64, 2, 'round_robin'), ([1000], 1000, 4,
                                    'round_robin'), ([7], 3, 8, 'round_robin'),
                                    ([12345, 999], 1024, 8, 'round_robin'),
                                    ([500, 500, 300], 128, 3, 'by_scene')]:
        seen = np.zeros(sum(px), int)
        for r in range(world):
            m = ltd.Mosaic(px, tile, world, r, assign)
            for t in m.mine:
                assert m.owner(t) == r
                seen[t.g0:t.g0 + t.n] += 1
        assert (seen == 1).all()
    m = ltd.Mosaic([100, 50], 40, 2, 0, 'by_scene')
    assert [t.scene for t in m.mine] == [0, 0, 0] and m.rounds == 3
    assert ltd.my_tiles(10, 4, 2, 1) == [(4, 8)]


def test_single_process_runner_matches_oracle():
    px = [700, 300]
    r = _run(1, 0, px, 256, 'round_robin', 7)
    want = _want(px, 7)
    for f in ltd.LABEL_GATHER_FIELDS:
        got = r.exchange.raster(f).numpy()
        assert _same(want[f][:2], got), f


@pytest.mark.parametrize('world,px,tile,assign,dst', [
    (2, [700, 300], 256, 'round_robin', 0),  # the c4 shape: one mosaic, tiles round-robin
    (2, [600, 600], 256, 'by_scene', 0),     # the c2 shape: one scene per rank
    (3, [300], 256, 'round_robin', 0),       # more ranks than tiles: rank 2 owns nothing
    # the writer owns fewer tiles than a peer: it must still post the peer's later rounds
    (2, [300, 900], 256, 'by_scene', 0),     # unequal scenes (writer 2 tiles, peer 4)
    (2, [700, 300], 256, 'round_robin', 1),  # writer rank 1 (2 tiles) under round-robin (3)
    (3, [300, 200, 900], 256, 'by_scene', 2),  # writer 4 tiles, peers 2 and 1
    (2, [1300], 256, 'round_robin', 0),      # bench --strong: ONE scene's tiles round-robin
])
@pytest.mark.timeout(180)  # an unmatched send hangs: fail instead
def test_multi_rank_exchange_matches_single_process(tmp_path, world, px, tile, assign, dst):
    path = str(tmp_path / 'r.npz')
    mp.spawn(_worker, args=(world, _free_port(), px, tile, assign, path, dst), nprocs=world,
             join=True)
    got = np.load(path)
    want = _want(px, 7)
    for f in ltd.LABEL_GATHER_FIELDS:
        assert _same(want[f][:2], got[f]), f


@pytest.mark.parametrize('world,px,tile,assign,dst', [
    (2, [600, 600], 256, 'by_scene', 0),     # the c2 shape
    (2, [700, 300], 256, 'round_robin', 0),  # the c4 shape
    (3, [300, 200, 900], 256, 'by_scene', 2),  # unequal scenes, writer rank 2
    (2, [1300], 256, 'round_robin', 0),        # bench --strong
])
@pytest.mark.timeout(180)
def test_pipelined_exchange_over_steps_matches_single_process(tmp_path, world, px, tile, assign,
                                                              dst):
    """bench.py's timed loop at N > 1: three steps with overlap=True (each step's sends stay in
    flight into the next; a sender's kernels for tile k first wait for the previous send of
    tile k's slab), then finish(): the writer holds exactly the single-process result."""
    path = str(tmp_path / 'r.npz')
    mp.spawn(_worker, args=(world, _free_port(), px, tile, assign, path, dst, 3, True),
             nprocs=world, join=True)
    got = np.load(path)
    want = _want(px, 7)
    for f in ltd.LABEL_GATHER_FIELDS:
        assert _same(want[f][:2], got[f]), f


def _job_worker(rank, world, port, root, result_path):
    import torch.distributed as dist
    from land_trendr_amd.geotiff import GeoTiff
    from land_trendr_amd.job import LocalJob
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    j = LocalJob(root, 'synth', tile_pixels=20, on_error='skip', engine=OracleEngine())
    files = j.run()
    # this rank's parse gathered only the grid points of its own tiles
    st = j.stack
    np.savez('%s.rank%d.npz' % (result_path, rank), bands=st['bands'], valid=st['valid'],
             ranges=np.array(st['ranges'], np.int64).reshape(-1, 3),
             mine=np.array([(t.p0, t.p1) for t in j.mosaic.mine], np.int64).reshape(-1, 2),
             n_pix=st['n_pix'])
    if rank == 0:
        arrs = {'raster:' + k: GeoTiff(v[0]).read() for k, v in files.items()}
        arrs.update({'plane:' + k: a for k, a in j.planes.items()})
        np.savez(result_path, **arrs)
    else:
        assert files is None
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.timeout(300)
def test_multi_rank_job_matches_single_rank_and_oracle(tmp_path):
    """job.LocalJob over 2 gloo ranks (tar.gz inputs extracted by rank 0 alone, tiles
    round-robin, labels exchanged to rank 0, trendline rows through the shared host maps): every
    output raster equals the single-rank job's, and the planes equal the oracle's."""
    from jobfixture import SETTINGS, make_job
    from land_trendr_amd import _abi
    from land_trendr_amd.geotiff import GeoTiff
    from land_trendr_amd.job import LocalJob
    from land_trendr_amd.scene import build_scene, parse_date
    from land_trendr_amd.settings import compile_params
    from oracle import oracle
    multi, single = str(tmp_path / 'multi'), str(tmp_path / 'single')
    make_job(multi)
    make_job(single)
    path = str(tmp_path / 'job.npz')
    mp.spawn(_job_worker, args=(2, _free_port(), multi, path), nprocs=2, join=True)
    got = dict(np.load(path))
    j = LocalJob(single, 'synth', tile_pixels=1 << 20, on_error='skip', engine=OracleEngine())
    files = j.run()
    assert sorted('raster:' + k for k in files) == sorted(k for k in got if k.startswith('raster:'))
    assert any(k.startswith('trendline/') for k in files)
    for k, v in files.items():
        assert np.array_equal(GeoTiff(v[0]).read(), got['raster:' + k]), k
    st = j.stack
    # per-rank ingest: each rank's stack holds its own tiles' grid points only (about half of
    # them here), and they are the single-rank stack's columns of those points
    held = 0
    for rank in range(2):
        r = np.load('%s.rank%d.npz' % (path, rank))
        assert int(r['n_pix']) == st['n_pix']
        assert [tuple(x[:2]) for x in r['ranges']] == [tuple(x) for x in r['mine']]
        n = int((r['mine'][:, 1] - r['mine'][:, 0]).sum())
        assert r['bands'].shape[-1] == n == r['valid'].shape[-1] < st['n_pix']
        for p0, p1, q0 in r['ranges']:
            assert np.array_equal(r['bands'][:, :, q0:q0 + p1 - p0], st['bands'][:, :, p0:p1])
            assert np.array_equal(r['valid'][:, q0:q0 + p1 - p0], st['valid'][:, p0:p1])
        held += n
    assert held == st['n_pix']
    idx = (st['bands'][:, 0, :].astype(np.int32) - st['bands'][:, 1, :]).astype(np.int16)
    meta = build_scene(st['dates'], parse_date(SETTINGS['target_date']))
    params, _ = compile_params(SETTINGS['line_cost'], SETTINGS['label_rules'])
    exp = oracle.analyze_tile(meta, params, idx.astype(np.float64), st['valid'])
    bad = np.flatnonzero(exp['status'] & ~_abi.LT_ST_EMPTY)  # on_error='skip'
    exp['matched'][:, bad] = 0
    exp['winner'][:, bad] = -1
    for k in [k for k in got if k.startswith('plane:')]:
        a, e = got[k], exp[k[6:]]
        e = e[:a.shape[0]] if a.ndim == 2 else e
        if k[6:] in ('onset_year', 'duration', 'class_val', 'magnitude', 'initial_val'):
            m = exp['matched'][:a.shape[0]].astype(bool)
            a, e = np.where(m, a, 0), np.where(m, e, 0)
        assert _same(a, e) or (a.dtype.kind == 'f' and _same_nan(a, e)), k


def _same_nan(a, b):
    return ((a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))).all()


def _own_worker(rank, world, port, scene_px, tile, assign, result_path):
    """bench.py's end-to-end 'own' label mode: no exchange, each rank keeps (copies to its host)
    its own tiles' label planes; saved per tile with the tile's mosaic position."""
    import torch.distributed as dist
    from land_trendr_amd.engine import IndexFn
    from land_trendr_amd.index_eqn import IndexProgram
    from land_trendr_amd.runner import MosaicRunner
    from land_trendr_amd.settings import compile_params
    from land_trendr_amd.synth import mosaic_inputs
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    m = ltd.Mosaic(scene_px, tile, world, rank, assign)
    items = mosaic_inputs(m, 20, 1, 2, 0.1, 7, 'cpu')
    params, _ = compile_params(10, RULES)
    fn = IndexFn(None, IndexProgram('B1 - B2', band_dtype='int16'))
    r = MosaicRunner(OracleEngine(), m, params, items, FIELDS, fn, dist, exchange_fields=())
    r.step()
    r.finish()
    assert r.exchange.full is None or not r.exchange.fields  # nothing gathered
    out = {}
    for k, it in enumerate(items):
        for f in ltd.LABEL_GATHER_FIELDS:
            out['%s:%d:%d' % (f, it.tile.g0, it.tile.n)] = r.outs[k][f][..., :it.tile.n].numpy()
    np.savez('%s.rank%d.npz' % (result_path, rank), **out)
    dist.barrier()
    dist.destroy_process_group()


@pytest.mark.parametrize('world,px,tile,assign', [
    (2, [600, 600], 256, 'by_scene'),  # the c2 shape
    (2, [1300], 256, 'round_robin'),   # bench --strong
])
@pytest.mark.timeout(180)
def test_own_label_planes_per_rank_match_single_process(tmp_path, world, px, tile, assign):
    """The end-to-end 'own' label mode at N > 1 (bench.py --e2e-labels own): no
    rank sends anything; the ranks' per-tile label planes, laid side by side by mosaic position,
    are the single-process rasters."""
    path = str(tmp_path / 'own')
    mp.spawn(_own_worker, args=(world, _free_port(), px, tile, assign, path), nprocs=world,
             join=True)
    want = _want(px, 7)
    got = {f: np.full(want[f][:2].shape, 7, want[f].dtype) for f in ltd.LABEL_GATHER_FIELDS}
    seen = np.zeros(sum(px), int)
    for rank in range(world):
        for key, a in np.load('%s.rank%d.npz' % (path, rank)).items():
            f, g0, n = key.split(':')
            g0, n = int(g0), int(n)
            got[f][..., g0:g0 + n] = a
            if f == 'magnitude':
                seen[g0:g0 + n] += 1
    assert (seen == 1).all()
    for f in ltd.LABEL_GATHER_FIELDS:
        assert _same(want[f][:2], got[f]), f
