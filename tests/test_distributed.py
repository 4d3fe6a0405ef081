"""Multi-process (gloo, CPU) checks of the mosaic path bench.py and the job runner use:
distributed.Mosaic tiling, runner.MosaicRunner's per-rank pipeline and distributed.LabelExchange's
point-to-point sends to the writer. The per-tile compute is the CPU oracle (test infrastructure)
behind a stand-in for the HIP engine (OracleEngine); on a GPU job it is liblt_hip.so."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from land_trendr_amd import distributed as ltd

RULES = [{'name': 'gd', 'val': 1, 'change_type': 'GD'},
         {'name': 'fd', 'val': 2, 'change_type': 'FD', 'duration': ['<', 5]}]
FIELDS = ('status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude')


class OracleEngine:
    """Engine stand-in on the CPU: index_tile evaluates the IndexProgram with numpy
    (oracle/index_oracle.py), analyze_tiles runs oracle/lt_oracle.c into the given outputs."""
    device = torch.device('cpu')

    def index_tile(self, fn, bands, out=None, stream=None):
        from oracle import index_oracle
        b = bands.numpy()
        v = index_oracle.evaluate(fn.program, np.moveaxis(b, 1, 0))
        out.copy_(torch.from_numpy(np.ascontiguousarray(v)))
        return out

    def analyze_tiles(self, scene, params, tiles, fields, outs=None, ready=None):
        from oracle import oracle
        for (vals, valid), o in zip(tiles, outs):
            want = oracle.analyze_tile(scene, params, vals.numpy().astype(np.float64),
                                       None if valid is None else valid.numpy())
            for f in fields:
                o[f].copy_(torch.from_numpy(want[f][..., :o[f].shape[-1]]))
        return outs


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _run(world, rank, scene_px, tile, assign, seed0, dist=None):
    from land_trendr_amd.engine import IndexFn
    from land_trendr_amd.index_eqn import IndexProgram
    from land_trendr_amd.runner import MosaicRunner
    from land_trendr_amd.settings import compile_params
    from land_trendr_amd.synth import mosaic_inputs
    m = ltd.Mosaic(scene_px, tile, world, rank, assign)
    items = mosaic_inputs(m, 20, 1, 2, 0.1, seed0, 'cpu')
    params, _ = compile_params(10, RULES)
    fn = IndexFn(None, IndexProgram('B1 - B2', band_dtype='int16'))
    r = MosaicRunner(OracleEngine(), m, params, items, FIELDS, fn, dist)
    r.step()
    return r


def _worker(rank, world, port, scene_px, tile, assign, result_path):
    import torch.distributed as dist
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    r = _run(world, rank, scene_px, tile, assign, 7, dist)
    if rank == 0:
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


@pytest.mark.parametrize('world,px,tile,assign', [
    (2, [700, 300], 256, 'round_robin'),   # the c4 shape: one mosaic, tiles round-robin
    (2, [600, 600], 256, 'by_scene'),      # the c2 shape: one scene per rank
    (3, [300], 256, 'round_robin'),        # more ranks than tiles: rank 2 owns nothing
])
def test_multi_rank_exchange_matches_single_process(tmp_path, world, px, tile, assign):
    path = str(tmp_path / 'r.npz')
    mp.spawn(_worker, args=(world, _free_port(), px, tile, assign, path), nprocs=world,
             join=True)
    got = np.load(path)
    want = _want(px, 7)
    for f in ltd.LABEL_GATHER_FIELDS:
        assert _same(want[f][:2], got[f]), f
