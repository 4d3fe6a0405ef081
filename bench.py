"""Benchmark: full LandTrendr analyze + label of a Landsat-scene-sized stack per GPU.

Metric (BASELINE.json): Mpixels/s of full analyze (30-yr series), whole job over all GPUs, with
the FP64-VALU roofline fraction of the dominant kernel. Default workload = configs[1] (c2):
7000 x 7000 px x 30 years, 1 obs/yr, one GD rule, line_cost 10, on one MI355X. Inputs are
synthetic, generated directly in HBM before the timed region.

A step = one pass of the hot path over the rank's whole scene, as a queue of pixel tiles
(lt_analyze_tile launches on the current stream). Multi-GPU (torchrun, one process per GPU):
each rank analyses its own scene (weak scaling, no data-path collective) and gathers each tile's
label rasters to rank 0 over RCCL inside the step, asynchronously, so the transfer of tile t runs
while tile t+1 computes (the reference's output_reducer input; --no-gather
drops it).
"""
import argparse
import json
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from land_trendr_amd.distributed import LABEL_GATHER_FIELDS  # noqa: E402
from land_trendr_amd.engine import get_engine  # noqa: E402
from land_trendr_amd.scene import build_scene, parse_date  # noqa: E402
from land_trendr_amd.settings import compile_params  # noqa: E402
from land_trendr_amd.synth import make_scene  # noqa: E402

FP64_PEAK_TFLOPS = 78.6     # MI355X FP64 vector peak (spec)
HBM_PEAK_GBS = 8000.0       # MI355X_MICROARCH.md chip-level parameters

GD = [{'name': 'gd', 'val': 1, 'change_type': 'GD'}]
C3_RULES = [{'name': 'fd', 'val': 2, 'change_type': 'FD', 'onset_year': ['>=', 1995],
             'duration': ['<', 4]},
            {'name': 'gd', 'val': 3, 'change_type': 'GD', 'pre_threshold': ['>', 500]},
            {'name': 'ld', 'val': 4, 'change_type': 'LD', 'duration': ['>', 2]}]
CONFIGS = {
    'c2': dict(desc='c2: 7000x7000 px x 30 yr, 1 obs/yr, GD rule, line_cost 10', pixels=49_000_000,
               years=30, k=(1, 1), mask=0.0, line_cost=10.0, rules=GD, mode='reference',
               trendline=False),
    'c3': dict(desc='c3: 7000x7000 px x 30 yr, 1-4 obs/yr + cloud masks, FD/GD/LD rules',
               pixels=49_000_000, years=30, k=(1, 4), mask=0.2, line_cost=10.0, rules=C3_RULES,
               mode='documented', trendline=False),
    'c5': dict(desc='c5: 40-yr series, line_cost 1, full per-year trendline output',
               pixels=49_000_000, years=40, k=(1, 1), mask=0.0, line_cost=1.0, rules=GD,
               mode='reference', trendline=True),
}


def f_ref(n):
    """Algorithmic FP64 flops per pixel of the reference algorithm."""
    s3 = n * (n + 1) * (n + 2) // 6 - 3 * n + 2
    return 20 * s3 + n * (n + 1) + 24 * n


def bytes_per_pixel(cfg, n_obs, n_years, value_bytes=8):
    inp = n_obs * value_bytes + (n_obs if cfg['mask'] > 0 else 0)  # index values + mask
    lab = len(cfg['rules']) * (1 + 4 + 4 + 4 + 8)                 # matched/class/onset/dur/mag
    tl = n_years * (6 * 8 + 2 + 2) if cfg['trendline'] else 0     # 6 f64 + spike/vertex + winner
    return inp + lab + tl + 4                                     # + status


PMC_SUMMARY = os.path.join(ROOT, 'profiles', 'r01_pmc_c2.json')


def pmc_traffic(kernel, px_per_launch, input_mode):
    """HBM bytes per launch of `kernel` from the committed rocprofv3 --pmc summary of this build
    (FETCH_SIZE/WRITE_SIZE passes, gfx950-corrected: profiles/summarize_pmc.py), scaled to this
    launch's pixel count; None when absent."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
        if d.get('_input', 'index') != input_mode:
            return None
        return d[kernel]['hbm_bytes'] / d['_pixels_per_launch'] * px_per_launch
    except (OSError, KeyError, ValueError, TypeError, ZeroDivisionError):
        return None


def pmc_fp64_issued(kernel, px_per_launch, input_mode):
    """FP64 flops the hardware issued per launch of `kernel` (PMC SQ_INSTS_VALU_{ADD,MUL,FMA}_F64
    x 64 lanes, FMA = 2) from the committed summary, scaled to this launch's pixel count."""
    try:
        with open(PMC_SUMMARY) as f:
            d = json.load(f)
        if d.get('_input', 'index') != input_mode:
            return None
        k = d[kernel]
        wave_flops = (k['SQ_INSTS_VALU_ADD_F64'] + k['SQ_INSTS_VALU_MUL_F64'] +
                      2 * k['SQ_INSTS_VALU_FMA_F64'])
        return 64 * wave_flops / d['_pixels_per_launch'] * px_per_launch
    except (OSError, KeyError, ValueError, TypeError, ZeroDivisionError):
        return None


def cpu_baseline(cfg, seconds):
    """The oracle (C restatement, pthreads over all host cores) on a bounded sample."""
    from oracle import oracle
    threads = os.cpu_count() or 1
    try:
        threads = len(os.sched_getaffinity(0))
    except AttributeError:
        pass
    threads = min(threads, 64)
    sample = max(64, 16 * threads)
    rate = None
    while True:
        sc = make_scene(sample, n_years=cfg['years'], k_min=cfg['k'][0], k_max=cfg['k'][1],
                        mask_prob=cfg['mask'], seed=77, device='cpu')
        meta = build_scene(sc.dates, parse_date('2014-07-01'))
        params, _ = compile_params(cfg['line_cost'], cfg['rules'], cfg['mode'])
        vals = sc.values.numpy()
        valid = sc.valid.numpy() if sc.valid is not None else None
        t0 = time.perf_counter()
        oracle.analyze_tile(meta, params, vals, valid, n_threads=threads)
        dt = time.perf_counter() - t0
        rate = sample / dt
        if dt >= 0.5 * seconds or sample >= 2_000_000:
            break
        sample = int(min(2_000_000, max(sample * 2, rate * seconds)))
    return {'value': rate / 1e6, 'unit': 'Mpixels/s', 'cores': threads, 'kind': 'port',
            'sample': '%d synthetic px of the same config, oracle/lt_oracle.c, %.1f s' % (sample, dt)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--config', default='c2', choices=sorted(CONFIGS))
    ap.add_argument('--pixels', type=int, default=0, help='pixels per GPU (default: config)')
    ap.add_argument('--tile', type=int, default=0,
                    help='pixels per launch (0: 1<<24)')
    ap.add_argument('--no-gather', action='store_true',
                    help='N>1: skip the RCCL gather of label rasters to rank 0')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--group', type=int, default=0,
                    help='tiles per lt_analyze_tiles call (0: all, or 1 when gathering)')
    ap.add_argument('--serial-load', action='store_true',
                    help='run every tile\'s index_eqn kernel ahead of the analyze kernels on '
                         'one stream (default: load stage on its own stream, per-tile events)')
    ap.add_argument('--input', default='bands', choices=['bands', 'index'],
                    help='bands: int16 B1, B2 planes + index_eqn "B1 - B2" on the GPU (the '
                         'reference pipeline, SURVEY.md 8(d)); index: float64 index values')
    args = ap.parse_args()

    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    # LT_BENCH_DEVICE / LT_BENCH_BACKEND: rehearsal hooks only (several ranks on one GPU over
    # gloo, to exercise the N>1 path on a 1-GPU box); the driver's runs use neither
    local = int(os.environ.get('LT_BENCH_DEVICE', local))
    backend = os.environ.get('LT_BENCH_BACKEND', 'nccl')
    torch.cuda.set_device(local)
    dist = None
    if world > 1:
        import torch.distributed as dist
        if backend == 'nccl':
            dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        else:
            dist.init_process_group(backend)
    cfg = CONFIGS[args.config]
    P = args.pixels or cfg['pixels']
    dev = torch.device('cuda', local)

    bands_in = args.input == 'bands'
    sc = make_scene(P, n_years=cfg['years'], k_min=cfg['k'][0], k_max=cfg['k'][1],
                    mask_prob=cfg['mask'], seed=1000 + rank, device=dev, with_bands=bands_in)
    index_fn = index_buf = None
    if bands_in:  # the load stage: settings.json index_eqn on int16 bands, compiled with hiprtc
        from land_trendr_amd.index_eqn import IndexProgram
        sc.values = None  # only the bands travel
        torch.cuda.empty_cache()
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    params, rules = compile_params(cfg['line_cost'], cfg['rules'], cfg['mode'])
    eng = get_engine(local)
    if bands_in:
        index_fn = eng.compile_index(IndexProgram('B1 - B2', band_dtype='int16'))
        # the index raster of the whole scene ([K, P], like rast_algebra's per-scene output):
        # tile views share the row stride of the cloud-mask planes (one stride per tile input)
        index_buf = torch.empty((meta.n_obs, P), dtype=torch.int16, device=dev)
    idx_events = []
    fields = ['status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude']
    if cfg['trendline']:
        fields += ['winner', 'val_raw', 'val_fit', 'fit_m', 'fit_b', 'right_m', 'right_b',
                   'spike', 'vertex']
    gather = dist is not None and not args.no_gather
    if args.tile <= 0:
        # c2 sweep on one MI355X (profiles/r01_c2_tile_sweep.txt): 2 Mpx 1459, 4 Mpx 1569,
        # 8 Mpx 1627, 16 Mpx 1647, 25 Mpx 1650, one 49 Mpx tile 1629 Mpx/s — fewer launch tails
        args.tile = 1 << 24
    tiles = [(p0, min(P, p0 + args.tile)) for p0 in range(0, P, args.tile)]
    # tile-major output planes: tile t's [R|Y, tile] slab of every field is contiguous, so it can
    # be handed to RCCL as soon as its kernels are queued
    slabs = [eng.alloc_outputs(meta.n_years, params.n_rules, args.tile, fields) for _ in tiles]
    recv = None
    if gather and rank == 0:  # the writer's label rasters for the whole job, allocated once
        recv = {f: [[torch.empty_like(sl[f]) for sl in slabs] for _ in range(world)]
                for f in LABEL_GATHER_FIELDS}
    works = []

    # tiles per lt_analyze_tiles call: all of them, or groups whose label rasters go to RCCL
    # while the next group computes
    # (gathering: one tile per call, so tile t's label rasters travel while tile t+1 computes;
    # N=1 layout proxies on one MI355X: 16.8 Mpx x 1 per call 1629, 8.4 Mpx x 2 1613, 4.19 Mpx
    # x 4 1554 Mpx/s, profiles/r01_c2_tile_sweep.txt)
    group = args.group if args.group > 0 else (len(tiles) if not gather else 1)

    # the load stage runs on its own stream: tile t's analyze kernel waits only for tile t's
    # index raster, so later tiles' index kernels (HBM-bound) run beside earlier tiles' analyze
    # kernels (issue-bound) instead of all of them ahead of the first analyze
    load_stream = torch.cuda.Stream(dev) if bands_in and not args.serial_load else None

    def step(timed=False):
        values, ready = [], []
        main = torch.cuda.current_stream(dev)
        if load_stream is not None:  # the previous step's analyze kernels read index_buf
            load_stream.wait_stream(main)
        for t, (p0, p1) in enumerate(tiles):  # the load stage: index_eqn over every tile
            if bands_in:
                with torch.cuda.stream(load_stream if load_stream is not None else main):
                    e0 = e1 = None
                    if timed:
                        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(
                            enable_timing=True)
                        e0.record()
                    values.append(eng.index_tile(index_fn, sc.bands[:, :, p0:p1],
                                                 out=index_buf[:, p0:p1]))
                    if timed:
                        e1.record()
                        idx_events.append((e0, e1))
                    ev = None
                    if load_stream is not None:
                        ev = torch.cuda.Event()
                        ev.record()
                    ready.append(ev)
            else:
                values.append(sc.values[:, p0:p1])
                ready.append(None)
        for g0 in range(0, len(tiles), group):
            ts = range(g0, min(len(tiles), g0 + group))
            # analyze + label (tile t's resolve stage beside tile t+1's analyze stage)
            eng.analyze_tiles(
                meta, params,
                [(values[t], sc.valid[:, tiles[t][0]:tiles[t][1]] if sc.valid is not None
                  else None) for t in ts], fields,
                outs=[{f: x[..., :tiles[t][1] - tiles[t][0]] for f, x in slabs[t].items()}
                      for t in ts],
                ready=[ready[t] for t in ts] if load_stream is not None else None)
            if gather:  # these tiles' label rasters to the writer rank, on
                # RCCL's stream: they travel while the next group computes
                for t in ts:
                    for f in LABEL_GATHER_FIELDS:
                        works.append(dist.gather(
                            slabs[t][f],
                            [recv[f][r][t] for r in range(world)] if rank == 0 else None,
                            dst=0, async_op=True))
        while works:
            works.pop().wait()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    eng.set_timing(True)
    eng.stage_ms()  # reset
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(timed=True)
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    stages = eng.stage_ms()
    eng.set_timing(False)
    n_deferred_last = eng.last_deferred()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())

    # correctness gate on this run's own outputs: no pixel may be flagged as an unemulated path
    n_numeric = sum(int(((sl['status'][:p1 - p0] & 16) != 0).sum().item())
                    for sl, (p0, p1) in zip(slabs, tiles))

    total_px = P * world * args.steps
    value = total_px / elapsed / 1e6
    n_launch = max(1, stages['launches'])
    kern_ms = stages['analyze'] / n_launch
    resolve_ms = stages['resolve'] / n_launch
    px_per_launch = P * args.steps / n_launch
    flops = f_ref(cfg['years']) * px_per_launch
    achieved = flops / (kern_ms * 1e-3) / 1e12
    bpp = bytes_per_pixel(cfg, meta.n_obs, meta.n_years, 2 if bands_in else 8)
    index_ms = (sum(a.elapsed_time(b) for a, b in idx_events) / max(1, len(idx_events))
                if idx_events else None)
    hbm_gbs = bpp * px_per_launch / (kern_ms * 1e-3) / 1e9
    traffic = pmc_traffic('analyze', px_per_launch, args.input) if args.config == 'c2' else None
    issued = (pmc_fp64_issued('analyze', px_per_launch, args.input) if args.config == 'c2'
              else None)
    res = {
        'metric': 'Mpixels/sec full analyze (30-yr series)' if cfg['years'] == 30 else
                  'Mpixels/sec full analyze (%d-yr series)' % cfg['years'],
        'value': round(value, 4), 'unit': 'Mpixels/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 3),
        'higher_is_better': True, 'scaling': 'weak', 'vs_baseline': None, 'dtype': 'f64',
        'data': 'synthetic (SURVEY.md 8(d) generator, seeded, generated in HBM)',
        'config': {'workload': cfg['desc'], 'pixels_per_gpu': P, 'years': cfg['years'],
                   'obs': meta.n_obs, 'rules': len(rules), 'line_cost': cfg['line_cost'],
                   'tile_pixels': args.tile, 'gather': bool(gather),
                   'input': ('int16 bands B1, B2 + index_eqn "B1 - B2"' if bands_in else
                             'float64 index values'),
                   'parallelism': 'pixel tiles, 1 scene per GPU'},
        # dominant kernel: the analyze stage, FP64-VALU bound (O(n^2) DP per 240-byte series).
        # achieved = the reference algorithm's flops (F_ref) per launch / the
        # launch's HIP-event time: frac > 1 means faster than the reference's own arithmetic could
        # run at FP64 peak (the kernel proves most candidate fits irrelevant)
        'roofline': {'bound': 'fp64-valu', 'achieved': round(achieved, 3),
                     'peak': FP64_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                     'frac': round(achieved / FP64_PEAK_TFLOPS, 4),
                     'traffic': None if traffic is None else round(traffic),
                     'traffic_source': os.path.relpath(PMC_SUMMARY, ROOT) if traffic else None,
                     'kernel': 'analyze_fast_kernel', 'kernel_ms': round(kern_ms, 3),
                     'flops_per_px': f_ref(cfg['years']), 'flops_model': 'F_ref (SURVEY.md 8(d))',
                     'algorithmic_bytes_per_px': bpp,
                     'hbm': {'achieved': round(hbm_gbs, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                             'frac': round(hbm_gbs / HBM_PEAK_GBS, 4)},
                     # what the hardware executed: FP64 VALU flops from the PMC summary / this
                     # launch's time (the DP's integer, compare and select work is not counted)
                     'fp64_issued': None if issued is None else {
                         'achieved': round(issued / (kern_ms * 1e-3) / 1e12, 3),
                         'peak': FP64_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                         'frac': round(issued / (kern_ms * 1e-3) / 1e12 / FP64_PEAK_TFLOPS, 4),
                         'source': os.path.relpath(PMC_SUMMARY, ROOT)}},
        'status_numeric_pixels': n_numeric,
        'load_stage': None if index_ms is None else {
            'kernel': 'lt_index_kernel (hiprtc, index_eqn "B1 - B2", int16 bands -> int16)',
            'ms_per_launch': round(index_ms, 3),
            # on its own stream the index kernels share the CUs with analyze kernels, so a
            # launch lasts longer than alone (--serial-load: 0.13 ms, 5.5 TB/s on c2)
            'overlapped_with_analyze': load_stream is not None,
            'hbm_gbs_algorithmic': round(meta.n_obs * 6 * px_per_launch / (index_ms * 1e-3) / 1e9,
                                         1)},
        'resolve_stage': {'ms_per_launch': round(resolve_ms, 3),
                          'deferred_pixels_last_tile': n_deferred_last,
                          'last_tile_pixels': tiles[-1][1] - tiles[-1][0]},
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res['cpu_baseline'] = cpu_baseline(cfg, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
