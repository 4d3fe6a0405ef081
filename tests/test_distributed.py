"""Multi-process (gloo, world_size 2, CPU) check of the sharding + label gather of
land_trendr_amd/distributed.py. The per-tile compute here is the CPU oracle (test
infrastructure), injected as analyze_tile_fn; on a GPU job it is the HIP engine."""
import os
import socket

import numpy as np
import pytest
import torch
import torch.multiprocessing as mp

from land_trendr_amd import distributed as ltd


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _worker(rank, world, port, n_pix, tile, result_path):
    import torch.distributed as dist
    from land_trendr_amd.scene import build_scene, parse_date
    from land_trendr_amd.settings import compile_params
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    os.environ['MASTER_ADDR'] = '127.0.0.1'
    os.environ['MASTER_PORT'] = str(port)
    dist.init_process_group('gloo', rank=rank, world_size=world)
    sc = make_scene(n_pix, n_years=20, k_min=1, k_max=2, mask_prob=0.1, seed=5)  # same on all
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    rules = [{'name': 'gd', 'val': 1, 'change_type': 'GD'},
             {'name': 'fd', 'val': 2, 'change_type': 'FD', 'duration': ['<', 5]}]
    params, _ = compile_params(10, rules)
    vals, valid = sc.values.numpy(), sc.valid.numpy()

    def fn(p0, p1):
        o = oracle.analyze_tile(meta, params, vals[:, p0:p1], valid[:, p0:p1])
        return {k: torch.from_numpy(v) for k, v in o.items()}

    shard = ltd.analyze_shard(n_pix, tile, world, rank, fn)
    full = ltd.gather_labels(shard, n_pix, tile, params.n_rules, world, rank, dist)
    if rank == 0:
        np.savez(result_path, **{k: v.numpy() for k, v in full.items()})
    dist.barrier()
    dist.destroy_process_group()


def test_tile_assignment_covers_scene_once():
    for n_pix, tile, world in [(1000, 64, 2), (1000, 1000, 4), (7, 3, 8), (12345, 1024, 8)]:
        seen = np.zeros(n_pix, int)
        for r in range(world):
            for p0, p1 in ltd.my_tiles(n_pix, tile, world, r):
                seen[p0:p1] += 1
        assert (seen == 1).all()


def test_two_rank_gather_matches_single_process(tmp_path):
    from land_trendr_amd.scene import build_scene, parse_date
    from land_trendr_amd.settings import compile_params
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    n_pix, tile = 1500, 256
    path = str(tmp_path / 'r.npz')
    mp.spawn(_worker, args=(2, _free_port(), n_pix, tile, path), nprocs=2, join=True)
    got = np.load(path)
    sc = make_scene(n_pix, n_years=20, k_min=1, k_max=2, mask_prob=0.1, seed=5)
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    params, _ = compile_params(10, [{'name': 'gd', 'val': 1, 'change_type': 'GD'},
                                    {'name': 'fd', 'val': 2, 'change_type': 'FD',
                                     'duration': ['<', 5]}])
    want = oracle.analyze_tile(meta, params, sc.values.numpy(), sc.valid.numpy())
    for f in ltd.LABEL_GATHER_FIELDS:
        a, b = want[f][:2], got[f]
        if a.dtype.kind == 'f':
            assert (a.view(np.int64) == b.view(np.int64)).all(), f
        else:
            assert (a == b).all(), f
