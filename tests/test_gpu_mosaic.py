"""The bench / job code path on the GPU at BASELINE.json sizes: synthetic int16 band stacks
(synth.mosaic_inputs, bench.py's seeds and tiling) -> index_eqn 'B1 - B2' (fused into the analyze
kernel: a linear form) -> lt_analyze_tiles -> label exchange (runner.MosaicRunner), checked
against the CPU oracle on 200,000 sampled pixels per config (fed the index raster the load kernel
writes from the same bands, as the reference's apply_grid feeds float(val) of the rast_algebra
raster), plus whole-raster invariants. c4 is the
4-scene, 196 Mpx mosaic of configs[3], dealt round-robin in 6.1 Mpx tiles as bench.py deals it
(one rank here: every tile of the mosaic on this GPU)."""
import os

import numpy as np
import pytest
import torch

import bench
from land_trendr_amd.distributed import Mosaic, TrendlineStream
from land_trendr_amd.engine import get_engine, valid_bytes
from land_trendr_amd.index_eqn import IndexProgram
from land_trendr_amd.runner import MosaicRunner
from land_trendr_amd.settings import compile_params
from land_trendr_amd.synth import mosaic_inputs

pytestmark = pytest.mark.gpu
SAMPLE = 200_000


def _threads():
    try:
        return min(len(os.sched_getaffinity(0)), 64)
    except AttributeError:
        return 8


def _same(a, b):
    if a.dtype.kind == 'f':
        return (a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
    return a == b


def _bench_runner(cfg_name, fields, pixels=0, whole=False):
    """whole: the scene as ONE tile (one lt_analyze_tiles launch of 49 Mpx), as bench.py runs a
    labels-only config on one GPU (bench.py main: `whole`); else 16.8 Mpx tiles."""
    c = bench.CONFIGS[cfg_name]
    P = pixels or c['pixels']
    if 'scenes' in c:
        tile = ((P + 7) // 8 + 63) // 64 * 64
        m = Mosaic([P] * c['scenes'], tile, 1, 0, 'round_robin')
    else:
        m = Mosaic([P], P if whole else 1 << 24, 1, 0, 'by_scene')
    eng = get_engine(0)
    items = mosaic_inputs(m, c['years'], c['k'][0], c['k'][1], c['mask'], c['seed'],
                          eng.device, bench.TARGET)
    params, _ = compile_params(c['line_cost'], c['rules'], c['mode'])
    fn = eng.compile_index(IndexProgram('B1 - B2', band_dtype='int16'))
    return MosaicRunner(eng, m, params, items, fields, fn), params


@pytest.mark.parametrize('cfg', ['c2', 'c3', 'c4', 'c5', 'c2-bench', 'c3-bench',
                                 'c2-bench-whole', 'c3-bench-whole'])
def test_bench_path_full_size_sampled_vs_oracle(cfg):
    """'c2' / 'c3' add the val_fit / vertex planes (the emulated-fit, year-major output path);
    'c2-bench' / 'c3-bench' request exactly bench.py's fields (labels only), so the kernel
    instance bench.py times runs: the certified labels path (lt_fast.h LT_CERT_RULES) over an
    int16 series with the fused 'B1 - B2' load stage, 1 rule (c2) or 3 rules with onset / duration
    / pre_threshold filters over mask bit planes (c3), on one full 16.8 Mpx tile each.
    '-bench-whole': the exact launch bench.py times on one GPU — the whole 49 Mpx scene as one
    tile, so one analyze launch of 765,625 waves, one deferred list sized for 49 Mpx and one
    resolve launch (bench.py main, `whole`)."""
    from oracle import oracle
    bench_fields = '-bench' in cfg
    whole = cfg.endswith('-whole')
    cfg = cfg.split('-')[0]
    c = bench.CONFIGS[cfg]
    fields = ['status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude']
    if cfg == 'c5':
        fields += bench.TRENDLINE_FIELDS
    elif cfg != 'c4' and not bench_fields:
        fields += ['val_fit', 'vertex']
    runner, params = _bench_runner(cfg, fields, whole=whole)
    if whole:  # the geometry bench.py times: one tile, one launch
        assert len(runner.items) == 1 and runner.items[0].tile.n == bench.CONFIGS[cfg]['pixels']
        assert runner.jit is not None  # the JIT kernels specialised for this launch
    runner.step()
    torch.cuda.synchronize()
    m = runner.m
    rng = np.random.default_rng(11)
    n_checked = 0
    for s in range(len(m.scene_pixels)):  # per scene: invariants, then a sample vs the oracle
        items = [(k, it) for k, it in enumerate(runner.items) if it.tile.scene == s]
        for k, it in items:
            o = {f: t[..., :it.tile.n] for f, t in runner.outs[k].items()}
            assert int((o['status'] != 0).sum()) == 0, (cfg, it.tile)
            mt = o['matched'].bool()
            assert bool(((o['class_val'] != -99) == mt).all())
            assert bool(((o['duration'] > 0) | ~mt).all())
            # the load stage: the index raster is B1 - B2 of the tile's int16 bands (the fused
            # steps never write it: the load kernel materialises it for the oracle)
            assert runner.fused
            runner.materialise_index(k)
            b = it.bands
            assert torch.equal(it.values, (b[:, 0, :].int() - b[:, 1, :].int()).short())
        n = SAMPLE // len(m.scene_pixels)
        for k, it in items:
            share = max(1, n * it.tile.n // m.scene_pixels[s])
            idx = torch.from_numpy(np.sort(rng.choice(it.tile.n, share, replace=False))).to(
                it.values.device)
            vals = it.values[:, idx].double().cpu().numpy()
            valid = (valid_bytes(it.valid[:, idx], it.scene.n_obs).cpu().numpy()
                     if it.valid is not None else None)
            want = oracle.analyze_tile(it.scene, params, vals, valid, n_threads=_threads())
            for f in fields:
                a = want[f]
                g = runner.outs[k][f][..., idx].cpu().numpy()
                same = _same(a[:g.shape[0]] if a.ndim == 2 else a, g)
                assert same.all(), (cfg, f, it.tile, int((~same).sum()))
            n_checked += share
    assert n_checked >= SAMPLE // 2
    del runner
    torch.cuda.empty_cache()


def test_stage_in_and_trendline_stream_match_resident_path():
    """bench.py's end-to-end pipeline (bands H2D from pinned memory into a two-slab ring, every
    trendline plane D2H through TrendlineStream) writes what the device-resident step writes."""
    fields = ['status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude'] + \
        bench.TRENDLINE_FIELDS
    c = bench.CONFIGS['c5']
    m = Mosaic([3 * (1 << 20) + 4321], 1 << 20, 1, 0, 'by_scene')
    eng = get_engine(0)
    items = mosaic_inputs(m, c['years'], 1, 1, 0.0, 77, eng.device, bench.TARGET)
    params, _ = compile_params(c['line_cost'], c['rules'], c['mode'])
    fn = eng.compile_index(IndexProgram('B1 - B2', band_dtype='int16'))
    runner = MosaicRunner(eng, m, params, items, fields, fn)
    runner.step()
    torch.cuda.synchronize()
    ref = [{f: t.clone() for f, t in o.items()} for o in runner.outs]
    for o in runner.outs:
        for t in o.values():
            t.fill_(0)
    got = {}

    def sink(f, row, host, key):
        got.setdefault(f, []).append((row, host.clone(), key))

    stage = bench._PinnedBands(items, eng.device)
    d2h = TrendlineStream(m.tile * 8, eng.device, depth=4, sink=sink)
    pushed = []

    def after(k):
        if k > 0:
            d2h.push({f: runner.outs[k - 1][f] for f in bench.TRENDLINE_FIELDS},
                     items[k - 1].tile.n, key=k - 1)
            pushed.append(k - 1)

    runner.step(after_tile=after, stage_in=stage)
    d2h.push({f: runner.outs[-1][f] for f in bench.TRENDLINE_FIELDS}, items[-1].tile.n,
             key=len(items) - 1)
    pushed.append(len(items) - 1)
    torch.cuda.synchronize()
    d2h.drain()
    for k, (o, r) in enumerate(zip(runner.outs, ref)):
        n = items[k].tile.n
        for f in fields:
            assert torch.equal(o[f][..., :n], r[f][..., :n]), (k, f)
    # the host copies: tile by tile, field by field, row by row, in push order
    for f in bench.TRENDLINE_FIELDS:
        rows = got[f]
        Y = ref[0][f].shape[0]
        assert len(rows) == Y * len(pushed)
        for j, k in enumerate(pushed):
            n = items[k].tile.n
            for y in range(Y):
                row, host, key = rows[j * Y + y]
                assert row == y and key == k
                want = ref[k][f][y, :n].cpu().contiguous().view(torch.uint8)
                assert torch.equal(host, want), (f, k, y)


@pytest.mark.parametrize('cfg', ['c3', 'c5'])
def test_pipelined_steps_match_joined_step(cfg):
    """bench.py's timed loop on one GPU: runner.step(overlap=True) leaves each tile's last stages
    (resolve; with trendline planes the expand kernel) in flight past the step, so a step's last
    resolve runs beside the next step's first analyze. After finish() every output equals what a
    joined step writes (c3: cloud-mask bit planes and 3 rules; c5: all 15 fields)."""
    fields = ['status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude']
    if cfg == 'c5':
        fields += bench.TRENDLINE_FIELDS
    c = bench.CONFIGS[cfg]
    m = Mosaic([3 * (1 << 20) + 4321], 1 << 20, 1, 0, 'by_scene')
    eng = get_engine(0)
    items = mosaic_inputs(m, c['years'], c['k'][0], c['k'][1], c['mask'], c['seed'], eng.device,
                          bench.TARGET)
    params, _ = compile_params(c['line_cost'], c['rules'], c['mode'])
    fn = eng.compile_index(IndexProgram('B1 - B2', band_dtype='int16'))
    runner = MosaicRunner(eng, m, params, items, fields, fn)
    runner.step()
    torch.cuda.synchronize()
    assert eng.last_deferred() > 0  # the resolve stage has work in every step
    ref = [{f: t.clone() for f, t in o.items()} for o in runner.outs]
    for o in runner.outs:
        for t in o.values():
            t.fill_(7)
    for _ in range(3):
        runner.step(overlap=True)
    assert len(runner._pending) == 3 * len(items)  # no step joined its tiles' last stages
    runner.finish()
    torch.cuda.synchronize()
    for k, (o, r) in enumerate(zip(runner.outs, ref)):
        n = items[k].tile.n
        for f in fields:
            a, b = o[f][..., :n], r[f][..., :n]
            same = (a == b) | (torch.isnan(a) & torch.isnan(b)) if a.is_floating_point() else a == b
            assert bool(same.all()), (cfg, k, f)
    del runner
    torch.cuda.empty_cache()


@pytest.mark.parametrize('tiles', [1, 3])
def test_pipelined_steps_with_changing_inputs_match_joined_steps(tiles):
    """a pipelined step (overlap=True) whose inputs differ from the previous step's.
    The caller rewrites every tile's bands between two pipelined steps (after waiting for the
    tile's tile_done event, the contract of runner.step); the outputs after finish() must equal
    a joined step over the new inputs in every plane — also for pixels the first step deferred
    and the second did not, whose stale resolve result would otherwise survive. tiles=1: the
    one-launch geometry bench.py times (two output banks); tiles=3: per-tile waits."""
    fields = ['status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude']
    c = bench.CONFIGS['c3']
    P = 3 * (1 << 20) + 4321
    m = Mosaic([P], P if tiles == 1 else 1 << 20, 1, 0, 'by_scene')
    eng = get_engine(0)
    params, _ = compile_params(c['line_cost'], c['rules'], c['mode'])
    fn = eng.compile_index(IndexProgram('B1 - B2', band_dtype='int16'))

    def inputs():
        return mosaic_inputs(m, c['years'], c['k'][0], c['k'][1], c['mask'], c['seed'],
                             eng.device, bench.TARGET)

    g = torch.Generator(device='cpu').manual_seed(99)
    deltas = [torch.randint(-300, 301, (it.bands.shape[0], it.bands.shape[2]), generator=g,
                            dtype=torch.int16).to(eng.device) for it in inputs()]
    a_items = inputs()
    a = MosaicRunner(eng, m, params, a_items, fields, fn)
    a.step()
    torch.cuda.synchronize()
    a.step(overlap=True)  # scene X, left in flight
    cur = torch.cuda.current_stream(eng.device)
    for k, it in enumerate(a_items):  # scene Y: the caller's rewrite, after tile_done(k)
        ev = a.tile_done(k)
        assert ev is not None
        cur.wait_event(ev)
        it.bands[:, 0, :] += deltas[k]
    a.step(overlap=True)
    assert len(a._pending) > 0
    a.finish()
    torch.cuda.synchronize()
    b_items = inputs()
    for k, it in enumerate(b_items):
        it.bands[:, 0, :] += deltas[k]
    b = MosaicRunner(eng, m, params, b_items, fields, fn)
    b.step()
    torch.cuda.synchronize()
    assert eng.last_deferred() > 0  # pixels go through the resolve stage in these steps
    for k in range(len(a_items)):
        n = a_items[k].tile.n
        for f in fields:
            x, y = a.outs[k][f][..., :n], b.outs[k][f][..., :n]
            same = (x == y) | (torch.isnan(x) & torch.isnan(y)) if x.is_floating_point() else x == y
            assert bool(same.all()), (tiles, k, f, int((~same).sum()))
    # the writer's label rasters (at world 1 a one-tile runner alternates two sets of them)
    assert a.exchange.fields
    for f in a.exchange.fields:
        x, y = a.exchange.raster(f), b.exchange.raster(f)
        assert bool((x == y).all()), (tiles, 'raster', f)
    if tiles == 1:
        assert a.exchange.full is a._fulls[a._bank]
        assert a.outs[0]['class_val'].data_ptr() == a.exchange.full['class_val'][0].data_ptr()
    del a, b, a_items, b_items
    torch.cuda.empty_cache()
