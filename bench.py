"""Benchmark: full LandTrendr analyze + label of Landsat-scene-sized stacks on 1..N GPUs.

Metric (BASELINE.json): Mpixels/s of full analyze (30-yr series), whole job over all GPUs, with
the roofline fraction of the dominant kernel. Default workload = configs[1] (c2): one
7000 x 7000 px x 30 year scene per GPU, 1 obs/yr, one GD rule, line_cost 10 (weak scaling).
--config c4 = configs[3]: ONE 4-scene mosaic (4 x 49 Mpx x 30 yr) whose pixel tiles are dealt
round-robin to the ranks (strong scaling). Inputs are synthetic, int16 bands
generated in HBM before the timed region.

A step = one pass of the hot path over the job (land_trendr_amd/runner.py, the code path the job
runner uses too): per tile, the index_eqn load kernel (B1 - B2) on the load stream, analyze +
label, then the tile's label rasters sent point-to-point to rank 0 over RCCL (N > 1), travelling
while the next tile computes. After the timed steps: the correctness gate (a seeded sample of
every rank's pixels re-analysed by the CPU oracle and compared with every plane the timed steps
wrote; any difference fails the run, exit status 3), the load kernel timed alone (its HBM
roofline) and, unless --e2e-steps 0, end-to-end steps that add H2D of the pinned int16 bands and
D2H of the label rasters (and, for c5, of every per-year trendline plane) to the same pipeline.
The oracle (oracle/, test infrastructure) is only the checker and the CPU baseline here: it never
produces a measured output.
"""
import argparse
import json
import math
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from land_trendr_amd._abi import build_hash  # noqa: E402
from land_trendr_amd.distributed import Mosaic, TrendlineStream  # noqa: E402
from land_trendr_amd.engine import get_engine, valid_bytes  # noqa: E402
from land_trendr_amd.index_eqn import IndexProgram  # noqa: E402
from land_trendr_amd.runner import MosaicRunner  # noqa: E402
from land_trendr_amd.scene import build_scene, parse_date  # noqa: E402
from land_trendr_amd.settings import compile_params  # noqa: E402
from land_trendr_amd.synth import make_scene, mosaic_inputs  # noqa: E402

# MI355X peaks (MI355X_MICROARCH.md)
FP64_PEAK_TFLOPS = 78.6          # 256 CUs x 4 SIMDs x 16 lanes x 2 (FMA) x 2.4 GHz
HBM_PEAK_GBS = 8000.0
SIMDS, CLOCK_GHZ = 1024, 2.4
VALU_PEAK_FILE = os.path.join('profiles', 'r05_valu_peak.json')


def valu_peak():
    """The VALU issue peak the analyze kernel's roofline is priced against: measured on the box
    by tools/valu_peak.hip (profiles/r05_valu_peak.json) — the chip's wave64 VALU instructions/s
    for a register-only stream of the c2 analyze kernel's instruction mix (PMC: 21 % FP64, 2 %
    INT64, the rest 32-bit, half as many SALU) at 8 waves per SIMD, the rate the SIMDs reach at
    full occupancy (the 4-wave rate of the kernel's own occupancy hid the occupancy
    cost; it is reported beside it). Returns (G instructions/s, source, details)."""
    try:
        with open(os.path.join(ROOT, VALU_PEAK_FILE)) as f:
            d = json.load(f)
        by = {(r['kind'], r['waves_per_simd']): r for r in d['results']}
        mix = by[('mix_c2', 8)]
        det = {k: round(by[(k, 4)]['cycles_per_valu_simd_nominal'], 3)
               for k in ('add_u32', 'cndmask_b32', 'cmp_gt_u32', 'fma_f32', 'add_f64', 'fma_f64',
                         'mul_f64', 'rcp_f64', 'lshlrev_b64', 'mix_c2', 'mov_b32', 'mov_b64',
                         'cmp_cndmask_vcc', 'cmp_cnd2_vcc', 'cndmask_vcc_valu')
               if (k, 4) in by}
        det['mix_c2_at_4_waves_g_per_s'] = round(by[('mix_c2', 4)]['g_valu_per_s_chip'], 2)
        return mix['g_valu_per_s_chip'], VALU_PEAK_FILE, det
    except (OSError, ValueError, KeyError):
        # not measured: the 4-cycle-per-instruction model (an assumption, flagged in the line)
        return SIMDS * CLOCK_GHZ / 4, 'model: 4 cycles per wave64 VALU instruction', None


TARGET = '2014-07-01'

GD = [{'name': 'gd', 'val': 1, 'change_type': 'GD'}]
C3_RULES = [{'name': 'fd', 'val': 2, 'change_type': 'FD', 'onset_year': ['>=', 1995],
             'duration': ['<', 4]},
            {'name': 'gd', 'val': 3, 'change_type': 'GD', 'pre_threshold': ['>', 500]},
            {'name': 'ld', 'val': 4, 'change_type': 'LD', 'duration': ['>', 2]}]
CONFIGS = {
    'c2': dict(desc='c2: 7000x7000 px x 30 yr, 1 obs/yr, GD rule, line_cost 10', pixels=49_000_000,
               years=30, k=(1, 1), mask=0.0, line_cost=10.0, rules=GD, mode='reference',
               trendline=False, seed=1000),
    'c3': dict(desc='c3: 7000x7000 px x 30 yr, 1-4 obs/yr + cloud masks, FD/GD/LD rules',
               pixels=49_000_000, years=30, k=(1, 4), mask=0.2, line_cost=10.0, rules=C3_RULES,
               mode='documented', trendline=False, seed=1000),
    'c4': dict(desc='c4: 4-scene mosaic (4 x 7000x7000 px = 196 Mpx) x 30 yr, GD rule, '
                    'line_cost 10, tiles round-robin over the GPUs', pixels=49_000_000, scenes=4,
               years=30, k=(1, 1), mask=0.0, line_cost=10.0, rules=GD, mode='reference',
               trendline=False, seed=4000),
    'c5': dict(desc='c5: 40-yr series, line_cost 1, full per-year trendline output',
               pixels=49_000_000, years=40, k=(1, 1), mask=0.0, line_cost=1.0, rules=GD,
               mode='reference', trendline=True, seed=1000),
}
TRENDLINE_FIELDS = ['winner', 'val_raw', 'val_fit', 'fit_m', 'fit_b', 'right_m', 'right_b',
                    'spike', 'vertex']
# the label planes a rank copies to its host in the end-to-end 'own' mode (what the gather sends)
LABEL_D2H_FIELDS = ['status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude']


def f_ref(n):
    """Algorithmic FP64 flops per pixel of the reference algorithm."""
    s3 = n * (n + 1) * (n + 2) // 6 - 3 * n + 2
    return 20 * s3 + n * (n + 1) + 24 * n


def bytes_per_pixel(cfg, n_obs, n_years, fused=True):
    """Algorithmic HBM bytes per pixel of the analyze kernel: the inputs (the two int16 band
    planes with the fused load stage, else the int16 index raster; + mask), the label planes, the
    per-year planes when the config asks for them, status."""
    inp = n_obs * (4 if fused else 2) + (n_obs if cfg['mask'] > 0 else 0)
    lab = len(cfg['rules']) * (1 + 4 + 4 + 4 + 8)                 # matched/class/onset/dur/mag
    tl = n_years * (6 * 8 + 2 + 2) if cfg['trendline'] else 0     # 6 f64 + spike/vertex + winner
    return inp + lab + tl + 4


def pmc_summary(config, build):
    """The committed rocprofv3 --pmc summary for `config` (profiles/summarize_pmc.py:
    per-launch counters of one 16.8 Mpx launch; c4 runs c2's kernel instance): the one collected
    on this kernel build (its '_build' equals `build`, _abi.build_hash) if committed, else the
    newest, whose '_matches_build' is then False and whose counters describe another build."""
    name = {'c4': 'c2'}.get(config, config)
    found = []
    for rnd in ('r06', 'r05', 'r04', 'r03', 'r02'):  # newest first
        path = os.path.join(ROOT, 'profiles', '%s_pmc_%s.json' % (rnd, name))
        try:
            with open(path) as f:
                d = json.load(f)
        except (OSError, ValueError):
            continue
        d['_path'] = os.path.relpath(path, ROOT)
        d['_matches_build'] = d.get('_build') == build
        found.append(d)
    for d in found:
        if d['_matches_build']:
            return d
    return found[0] if found else None


def per_px(pmc, kernel, counter):
    try:
        return pmc[kernel][counter] / pmc['_pixels_per_launch']
    except (KeyError, TypeError, ZeroDivisionError):
        return None


def host_cores():
    """Threads this process may run on, and the CPUs its cgroup quota grants (the GPU box shows
    the whole machine's CPUs but gives each job a share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    quota = None
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            quota = int(q) / int(per)
    except (OSError, ValueError):
        pass
    return n, quota


def cpu_baseline(cfg, seconds):
    """The oracle (C restatement, pthreads over every host core this process may use) on a
    bounded sample of the same configuration."""
    from oracle import oracle
    avail, quota = host_cores()
    # one thread per core the process may use: the cgroup quota when set (the GPU box shows the
    # whole machine but grants a share; more threads than that only time-slice)
    threads = avail if quota is None else max(1, min(avail, int(math.ceil(quota))))
    sample = max(64, 16 * threads)
    rate = None
    while True:
        sc = make_scene(sample, n_years=cfg['years'], k_min=cfg['k'][0], k_max=cfg['k'][1],
                        mask_prob=cfg['mask'], seed=77, device='cpu')
        meta = build_scene(sc.dates, parse_date(TARGET))
        params, _ = compile_params(cfg['line_cost'], cfg['rules'], cfg['mode'])
        vals = sc.values.numpy()
        valid = sc.valid.numpy() if sc.valid is not None else None
        t0 = time.perf_counter()
        oracle.analyze_tile(meta, params, vals, valid, n_threads=threads)
        dt = time.perf_counter() - t0
        rate = sample / dt
        if dt >= 0.5 * seconds or sample >= 4_000_000:
            break
        sample = int(min(4_000_000, max(sample * 2, rate * seconds)))
    return {'value': rate / 1e6, 'unit': 'Mpixels/s', 'cores': threads, 'kind': 'port',
            'threads': threads, 'host_cpus_visible': avail, 'cgroup_cpu_quota': quota,
            'sample': '%d synthetic px of the same config, oracle/lt_oracle.c, %d threads, %.1f s'
                      % (sample, threads, dt)}


def parity_sample(runner, params, n_sample, threads, seed=12345):
    """The oracle leg's correctness gate: a seeded sample of this rank's pixels,
    re-analysed by the oracle (oracle/lt_oracle.c, the CPU checker) from the same index rasters
    the timed steps read, against every output plane the timed steps wrote for them (labels only
    where the rule matched: elsewhere both sides hold NODATA placeholders). Returns (pixels,
    mismatching values, {field: mismatches})."""
    import numpy as np
    from oracle import oracle
    items = runner.items
    sizes = np.array([it.tile.n for it in items], np.int64)
    if sizes.sum() == 0:
        return 0, 0, {}
    rng = np.random.default_rng(seed + runner.m.rank)
    n = int(min(n_sample, sizes.sum()))
    flat = np.sort(rng.choice(int(sizes.sum()), n, replace=False))
    starts = np.concatenate([[0], np.cumsum(sizes)[:-1]])
    tile_of = np.searchsorted(starts, flat, side='right') - 1
    bad, per_field, checked = 0, {}, 0
    for k in np.unique(tile_of):
        it = items[k]
        if runner.fused:  # the fused steps read the band planes: the load kernel's raster of them
            runner.materialise_index(k)
        cols = torch.from_numpy(flat[tile_of == k] - starts[k]).to(it.values.device)
        vals = it.values[:, cols].double().cpu().numpy()
        valid = None if it.valid is None else valid_bytes(it.valid[:, cols],
                                                          it.scene.n_obs).cpu().numpy()
        exp = oracle.analyze_tile(it.scene, params, vals, valid, n_threads=threads)
        m = exp['matched'].astype(bool)
        for f, plane in runner.outs[k].items():
            got = plane[..., cols].cpu().numpy()
            e = exp[f][:got.shape[0]] if got.ndim == 2 else exp[f]
            if f in ('class_val', 'onset_year', 'duration', 'magnitude', 'initial_val'):
                got, e = np.where(m[:got.shape[0]], got, 0), np.where(m[:got.shape[0]], e, 0)
            if got.dtype.kind == 'f':
                same = (got.view(np.int64) == e.view(np.int64)) | (np.isnan(got) & np.isnan(e))
            else:
                same = got == e
            nb = int((~same).sum())
            if nb:
                per_field[f] = per_field.get(f, 0) + nb
                bad += nb
        checked += len(cols)
    return checked, bad, per_field


def _pinned_like(t):
    """A pinned, compact host copy of the [K, NB, n] bands t in t's layout: planar, or
    pixel-interleaved (a [K, n, NB] buffer viewed as [K, NB, n])."""
    K, NB, n = t.shape
    if t.stride(1) == 1 and NB > 1:
        h = torch.empty((K, n, NB), dtype=t.dtype, pin_memory=True).permute(0, 2, 1)
    else:
        h = torch.empty((K, NB, n), dtype=t.dtype, pin_memory=True)
    h.copy_(t)
    return h


class _PinnedBands:
    """stage_in for MosaicRunner.step: tile k's int16 bands H2D from pinned host memory into
    device slab k % 2 on a copy stream, once the load kernel of tile k - 2 has read that slab."""

    def __init__(self, items, dev):
        # host copies in the bands' own layout (planar or pixel-interleaved), compact; each device
        # slab is flat and a tile's view of it has the host copy's exact strides, so every H2D is
        # one contiguous copy (a shorter last tile sliced out of a full-size view had strides of
        # the full tile and was not)
        self.host = [_pinned_like(it.bands) for it in items]
        big = max(self.host, key=lambda b: b.numel())
        self.slab = [torch.empty(big.numel(), dtype=big.dtype, device=dev) for _ in range(2)]
        self.free = [None, None]
        self.stream = torch.cuda.Stream(dev)
        self.bytes = 0

    def fetch(self, k):
        s = k % 2
        h = self.host[k]
        with torch.cuda.stream(self.stream):
            if self.free[s] is not None:
                self.stream.wait_event(self.free[s])
            dst = self.slab[s][:h.numel()].as_strided(h.size(), h.stride())
            dst.copy_(h, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record()
        self.bytes += h.numel() * h.element_size()
        return dst, ev

    def consumed(self, k, ev):
        self.free[k % 2] = ev


def end_to_end(runner, cfg, steps, labels='gather'):
    """Steps of the same pipeline with the data movement a job has: each tile's int16 bands H2D
    from pinned host memory before its load kernel (_PinnedBands), the label rasters D2H, and for
    trendline configs every per-year plane of every tile D2H through TrendlineStream (tile k-1's
    planes queued behind tile k's kernels). labels: 'gather' — the writer's label rasters D2H
    after the exchange (every rank's labels cross the writer's one PCIe link); 'own' — the runner
    exchanges nothing and each rank copies its own tiles' label planes to its host, tile k-1's
    behind tile k's kernels (the writer's link would otherwise carry N scenes'
    labels per step). Returns (seconds, H2D bytes, D2H bytes)."""
    dev = runner.eng.device
    stage = _PinnedBands(runner.items, dev)
    tl = list(TRENDLINE_FIELDS) if cfg['trendline'] else []
    own = [f for f in LABEL_D2H_FIELDS if f in runner.fields] if labels == 'own' else []
    W = runner.m.tile
    d2h = TrendlineStream(W * 8, dev, depth=8) if (tl or own) else None
    ex = runner.exchange
    lab_host = ({f: torch.empty(t.shape, dtype=t.dtype, pin_memory=True)
                 for f, t in ex.full.items()} if labels == 'gather' and ex.is_writer and ex.full
                else {})
    items = runner.items
    bytes_d2h = 0

    def planes(k):
        return {f: runner.outs[k][f] for f in tl + own}

    def after(k):
        if d2h is not None and k > 0:
            d2h.push(planes(k - 1), items[k - 1].tile.n)

    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(steps):
        runner.step(after_tile=after, stage_in=stage)
        if d2h is not None and items:
            d2h.push(planes(len(items) - 1), items[-1].tile.n)
        for f, t in lab_host.items():  # the writer's label rasters, for its GeoTIFF writer
            t.copy_(ex.full[f], non_blocking=True)
            bytes_d2h += t.numel() * t.element_size()
        torch.cuda.synchronize()
        if d2h is not None:
            d2h.drain()
    dt = time.perf_counter() - t0
    return dt, stage.bytes, bytes_d2h + (d2h.bytes if d2h is not None else 0)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--gpus', type=int, default=1)
    ap.add_argument('--steps', type=int, default=3)
    ap.add_argument('--warmup', type=int, default=1)
    ap.add_argument('--config', default='c2', choices=sorted(CONFIGS))
    ap.add_argument('--pixels', type=int, default=0, help='pixels per scene (default: config)')
    ap.add_argument('--tile', type=int, default=0,
                    help='pixels per tile (0: the whole scene for a labels-only config on one '
                         'GPU, else 1<<24; scene/8 for the c4 mosaic)')
    ap.add_argument('--no-gather', action='store_true',
                    help='N>1: skip the exchange of label rasters to rank 0')
    ap.add_argument('--cpu-seconds', type=float, default=15.0)
    ap.add_argument('--no-cpu-baseline', action='store_true')
    ap.add_argument('--no-overlap', action='store_true',
                    help='complete each step (its last resolve / expand stages, and at N > 1 '
                         'its label exchange) before the next step starts')
    ap.add_argument('--e2e-steps', type=int, default=1,
                    help='end-to-end steps (H2D bands, D2H outputs) after the timed ones; 0: none')
    ap.add_argument('--group', type=int, default=0,
                    help='tiles per lt_analyze_tiles call (0: all of a scene, or 1 when gathering)')
    ap.add_argument('--no-trendline', action='store_true',
                    help='attribution runs only: leave out the per-year trendline planes of a '
                         'trendline config (c5)')
    ap.add_argument('--parity-sample', type=int, default=16384,
                    help='pixels per rank re-analysed by the oracle after the timed steps and '
                         'compared with every plane they wrote (0: skip; A/B timing runs only)')
    ap.add_argument('--serial-load', action='store_true',
                    help='run the index_eqn kernels on the analyze stream (no load stream)')
    ap.add_argument('--tiled-steps', type=int, default=3,
                    help='N = 1, labels-only configs: steps of the N > 1 tiling (16.8 Mpx tiles) '
                         'timed after the main ones (0: skip)')
    ap.add_argument('--strong', action='store_true',
                    help='strong scaling of ONE scene (the north_star shape: one 7000 x 7000 '
                         'scene over N GPUs): its pixel tiles dealt round-robin to the ranks, '
                         'labels sent to rank 0 (default: one scene per GPU, weak scaling)')
    ap.add_argument('--e2e-labels', choices=('auto', 'gather', 'own'), default='auto',
                    help='end-to-end steps: the writer copies the gathered label rasters to its '
                         'host (gather), or every rank copies its own (own); auto: own at N > 1')
    ap.add_argument('--index-eqn', default='B1 - B2',
                    help='attribution runs: another index_eqn over the same two int16 bands, e.g. '
                         '"(B1 - B2) * 2 / 2" (the same values through a program that is not a '
                         'linear form: the JIT-fused load stage, lt_jit.h)')
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
    cfg = dict(CONFIGS[args.config])
    if args.no_trendline:
        cfg['trendline'] = False
        cfg['desc'] += ' (attribution run: trendline planes left out)'
    P = args.pixels or cfg['pixels']
    dev = torch.device('cuda', local)
    mosaic_cfg = 'scenes' in cfg or args.strong
    if args.strong and 'scenes' not in cfg:
        cfg['scenes'] = 1
        cfg['desc'] += ' (strong scaling: one scene, tiles round-robin over the GPUs)'
    if mosaic_cfg:  # one mosaic for the whole job, tiles round-robin over the ranks
        # four tiles per rank (at N = 8 the 32 tiles of P / 8 the round-robin was built for; at
        # N = 1 one launch per scene, as c2: 32 launches of 6.1 Mpx ran 2615 Mpx/s, each paying
        # a launch drain), no tile larger than a scene
        total = P * cfg['scenes']
        tile = args.tile or min(P, ((total + 4 * world - 1) // (4 * world) + 63) // 64 * 64)
        mosaic = Mosaic([P] * cfg['scenes'], tile, world, rank, 'round_robin')
    else:  # one scene per rank (weak scaling)
        # one launch per scene on one GPU for the labels-only configs (fewer launch drains and
        # resolve launches: c2 2619-2630 vs 2577-2592, c3 1995 vs 1971 Mpx/s with 16.8 Mpx tiles,
        # profiles/r04_run23); 16.8 Mpx tiles when the writer's label exchange can overlap the
        # next tile (N > 1) or the config writes the per-year planes
        whole = world == 1 and not cfg['trendline'] and P <= (1 << 26)
        tile = args.tile or (P if whole else (1 << 24))
        mosaic = Mosaic([P] * world, tile, world, rank, 'by_scene')
    fused = os.environ.get('LT_FUSED_INDEX', '1') != '0'
    items = mosaic_inputs(mosaic, cfg['years'], cfg['k'][0], cfg['k'][1], cfg['mask'],
                          cfg['seed'], dev, TARGET,
                          band_layout=os.environ.get('LT_BAND_LAYOUT',
                                                     'pixel' if fused else 'planar'),
                          mask_format=os.environ.get('LT_MASK_FORMAT', 'bits'))
    params, rules = compile_params(cfg['line_cost'], cfg['rules'], cfg['mode'])
    eng = get_engine(local)
    index_fn = eng.compile_index(IndexProgram(args.index_eqn, band_dtype='int16'))
    fields = ['status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude']
    if cfg['trendline']:
        fields += TRENDLINE_FIELDS
    runner = MosaicRunner(eng, mosaic, params, items, fields, index_fn, dist,
                          exchange_fields=() if args.no_gather else
                          ('class_val', 'onset_year', 'duration', 'magnitude'),
                          load_stream=not args.serial_load, group=args.group)
    gather = world > 1 and not args.no_gather

    # the JIT module of every scene this rank runs, compiled before the warmup (lt_jit_prepare):
    # no step waits for hiprtc, and no timed tile may run on the precompiled fallback
    runner.prepare_jit(wait=True)
    for _ in range(args.warmup):
        runner.step()
    torch.cuda.synchronize()
    if dist is not None:
        dist.barrier()
    jit0 = eng.jit_stats()
    eng.set_timing(True)
    eng.stage_ms()  # reset
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    # the steps are pipelined as for a stream of scenes (runner.step overlap): a step's last
    # resolve runs beside the next step's first analyze, and at N > 1 its label exchange stays in
    # flight into the next step (tile k's kernels wait only for the previous step's send of tile
    # k); every tile's stages and transfers are complete before the clock stops (finish)
    for _ in range(args.steps):
        runner.step(timed=True, overlap=not args.no_overlap)
    runner.finish()
    torch.cuda.synchronize()
    t1 = time.perf_counter()
    if dist is not None:
        dist.barrier()
    stages = eng.stage_ms()
    eng.set_timing(False)
    jit1 = eng.jit_stats()
    jit = {'tiles_jit_timed': jit1['jit_tiles'] - jit0['jit_tiles'],
           'tiles_fallback_timed': jit1['fallback_tiles'] - jit0['fallback_tiles'],
           'modules': jit1['modules'], 'compiles': jit1['compiles'],
           'disk_hits': jit1['disk_hits'], 'failures': jit1['failures'],
           'override': os.environ.get('LT_JIT_OVERRIDE_DIR')}
    n_deferred_last = eng.last_deferred()
    elapsed = torch.tensor([t1 - t0], dtype=torch.float64, device=dev)
    if dist is not None:
        dist.all_reduce(elapsed, op=dist.ReduceOp.MAX)
    elapsed = float(elapsed.item())
    index_ms = runner.index_ms()

    # correctness gate on this run's own outputs: no pixel may be flagged as an unemulated path,
    # and a seeded sample of the pixels must match the oracle in every plane the steps wrote
    n_numeric = sum(int(((o['status'][:it.tile.n] & 16) != 0).sum().item())
                    for o, it in zip(runner.outs, items))
    psample = None
    if args.parity_sample > 0:
        avail, quota = host_cores()
        thr = avail if quota is None else max(1, min(avail, int(math.ceil(quota))))
        t_ps = time.perf_counter()
        checked, bad, per_field = parity_sample(runner, params, args.parity_sample, thr)
        res_t = torch.tensor([checked, bad], dtype=torch.float64, device=dev)
        if dist is not None:
            dist.all_reduce(res_t)
        psample = {'pixels': int(res_t[0].item()), 'mismatched_values': int(res_t[1].item()),
                   'fields': sorted(runner.fields), 'mismatches_rank0': per_field,
                   'seconds_rank0': round(time.perf_counter() - t_ps, 2),
                   'checker': 'oracle/lt_oracle.c on a seeded sample of each rank\'s pixels, '
                              'from the index rasters of the bands the timed steps read '
                              '(lt_index_apply)'}
    # the exchange (N > 1): every label tile the writer received equals the owner's copy,
    # compared as per-(tile, field) position-weighted byte sums all-reduced to every rank
    xcheck = None
    if gather:
        ex = runner.exchange
        own = ex.checksums(mosaic.mine)
        tot = own.to(dev)
        dist.all_reduce(tot)  # each tile's sums come from its owner alone
        if ex.is_writer:
            got = ex.checksums(mosaic.tiles)
            bad = int((got.to(dev) != tot).any(dim=1).sum().item())
            xcheck = {'tiles': len(mosaic.tiles), 'fields': list(ex.fields),
                      'mismatched_tiles': bad,
                      'check': 'per-(tile, field) position-weighted byte sums of the writer\'s '
                               'received label planes vs the owners\' (all-reduced)'}
    # the load kernel alone (its HBM roofline): one tile, serially, after the timed region
    it0 = items[0]
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    eng.index_tile(index_fn, it0.bands, out=it0.values)
    ev[0].record()
    for _ in range(5):
        eng.index_tile(index_fn, it0.bands, out=it0.values)
    ev[1].record()
    torch.cuda.synchronize()
    index_alone_ms = ev[0].elapsed_time(ev[1]) / 5
    K0 = it0.scene.n_obs
    index_bytes = K0 * it0.tile.n * 6  # two int16 band planes read, one int16 plane written

    # the dominant kernel with no previous step's resolve beside it: in the pipelined timed steps
    # each analyze launch shares the CUs with the previous step's resolve for part of its time
    # (its HIP-event time includes that); two joined steps, their HIP-event stage times
    #  and the whole-step rate of joined steps, beside the pipelined headline: a
    # pipelined step is safe for inputs that change between steps (runner.step, tile_done), but
    # the job runner's per-tile ring (job.py) runs joined steps
    kern_ms_joined = None
    joined = None
    if not args.no_overlap:
        eng.set_timing(True)
        eng.stage_ms()  # reset
        n_joined = 2
        torch.cuda.synchronize()
        if dist is not None:
            dist.barrier()
        tj = time.perf_counter()
        for _ in range(n_joined):
            runner.step()
        torch.cuda.synchronize()
        tj = time.perf_counter() - tj
        st2 = eng.stage_ms()
        eng.set_timing(False)
        kern_ms_joined = st2['analyze'] / max(1, st2['launches'])
        tjt = torch.tensor([tj], dtype=torch.float64, device=dev)
        if dist is not None:
            dist.all_reduce(tjt, op=dist.ReduceOp.MAX)
        tj = float(tjt.item())
        joined = {'value': round(mosaic.n_pix * n_joined / tj / 1e6, 3), 'unit': 'Mpixels/s',
                  'steps': n_joined, 'ms_per_step': round(tj / n_joined * 1e3, 3),
                  'note': 'each step completes (every resolve, every transfer) before the next '
                          'starts: the job runner\'s mode; `value` pipelines consecutive steps '
                          '(runner.step overlap, safe for changing inputs)'}

    e2e = None
    if args.e2e_steps > 0:
        if dist is not None:
            dist.barrier()
        e2e_runner, e2e_tile = runner, mosaic.tile
        if mosaic.tile > (1 << 24):
            # the bands cross PCIe per tile, overlapped with the previous tile's kernels: a
            # whole-scene tile would leave the copy unhidden, so these steps use 16.8 Mpx tiles
            m2 = Mosaic(mosaic.scene_pixels, 1 << 24, world, rank, mosaic.assign)
            items2 = mosaic_inputs(m2, cfg['years'], cfg['k'][0], cfg['k'][1], cfg['mask'],
                                   cfg['seed'], dev, TARGET,
                                   band_layout=os.environ.get('LT_BAND_LAYOUT',
                                                              'pixel' if fused else 'planar'),
                                   mask_format=os.environ.get('LT_MASK_FORMAT', 'bits'))
            e2e_runner = MosaicRunner(eng, m2, params, items2, fields, index_fn, dist,
                                      exchange_fields=() if args.no_gather else
                                      ('class_val', 'onset_year', 'duration', 'magnitude'),
                                      load_stream=not args.serial_load, group=args.group)
            e2e_runner.step()  # warm
            torch.cuda.synchronize()
            e2e_tile = m2.tile
        labels = args.e2e_labels if args.e2e_labels != 'auto' else (
            'own' if world > 1 else 'gather')
        if labels == 'own' and gather:
            # the labels stay with their ranks: a runner that exchanges nothing
            m_e = e2e_runner.m
            e2e_runner = MosaicRunner(eng, m_e, params, e2e_runner.items, fields, index_fn, dist,
                                      exchange_fields=(), load_stream=not args.serial_load,
                                      group=args.group)
            e2e_runner.step()  # warm
            torch.cuda.synchronize()
        dt, bh, bd = end_to_end(e2e_runner, cfg, args.e2e_steps, labels)
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        if dist is not None:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        e2e = {'value': round(mosaic.n_pix * args.e2e_steps / dt / 1e6, 3), 'unit': 'Mpixels/s',
               'tile_pixels': e2e_tile,
               'ms_per_step': round(dt / args.e2e_steps * 1e3, 3), 'steps': args.e2e_steps,
               'labels': labels,
               'h2d_bytes_per_step_rank0': bh // args.e2e_steps,
               'd2h_bytes_per_step_rank0': bd // args.e2e_steps,
               'includes': 'H2D of pinned int16 bands per tile (copy stream, overlapped), '
                           'index_eqn, analyze, ' +
                           ('label exchange, D2H of the writer\'s label rasters'
                            if labels == 'gather' else
                            'D2H of each rank\'s own label planes per tile (no exchange)') +
                           (' and of every per-year trendline plane per tile '
                            '(TrendlineStream)' if cfg['trendline'] else '')}

    # N = 1: the rate of the N > 1 pipeline on this GPU (16.8 Mpx tiles of the scene in one call,
    # per-tile completion events as the label exchange uses them), so the driver's N = 1 point and
    # its N > 1 points can be compared pipeline for pipeline
    tiled = None
    if world == 1 and not mosaic_cfg and mosaic.tile > (1 << 24) and args.tiled_steps > 0:
        m3 = Mosaic([P], 1 << 24, 1, 0, 'by_scene')
        items3 = mosaic_inputs(m3, cfg['years'], cfg['k'][0], cfg['k'][1], cfg['mask'],
                               cfg['seed'], dev, TARGET,
                               band_layout=os.environ.get('LT_BAND_LAYOUT',
                                                          'pixel' if fused else 'planar'),
                               mask_format=os.environ.get('LT_MASK_FORMAT', 'bits'))
        r3 = MosaicRunner(eng, m3, params, items3, fields, index_fn, None, exchange_fields=(),
                          load_stream=not args.serial_load, group=args.group)
        r3.gathering = True  # the N > 1 call pattern: completion events, no per-call join
        r3.prepare_jit(wait=True)
        r3.step()
        torch.cuda.synchronize()
        t3 = time.perf_counter()
        for _ in range(args.tiled_steps):
            r3.step(overlap=not args.no_overlap)
        r3.finish()
        torch.cuda.synchronize()
        dt3 = time.perf_counter() - t3
        tiled = {'tile_pixels': m3.tile, 'tiles': len(m3.tiles), 'steps': args.tiled_steps,
                 'value': round(P * args.tiled_steps / dt3 / 1e6, 3), 'unit': 'Mpixels/s',
                 'ms_per_step': round(dt3 / args.tiled_steps * 1e3, 3),
                 'pipeline': 'the N > 1 one: 16.8 Mpx tiles, one lt_analyze_tiles_ev call per '
                             'scene with per-tile completion events (no exchange at N = 1)'}
        del r3, items3
        torch.cuda.empty_cache()

    total_px = mosaic.n_pix * args.steps
    value = total_px / elapsed / 1e6
    n_launch = max(1, stages['launches'])
    kern_ms = stages['analyze'] / n_launch
    resolve_ms = stages['resolve'] / n_launch
    my_px = sum(it.tile.n for it in items)
    px_per_launch = my_px * args.steps / n_launch
    meta = items[0].scene
    build = build_hash()
    pmc = pmc_summary(args.config, build)
    # a summary taken on another kernel build describes other code: refused for the roofline
    # (achieved / frac / traffic null), its figures kept beside it, marked as another build's
    pmc_other = None
    if pmc is not None and not pmc['_matches_build']:
        pmc_other, pmc = pmc, None
    peak_g, peak_src, peak_cyc = valu_peak()
    valu_px = per_px(pmc, 'analyze', 'SQ_INSTS_VALU')
    achieved = (valu_px * px_per_launch / (kern_ms * 1e-3) / 1e9) if valu_px else None
    pmc_frac = None
    if pmc and 'GRBM_GUI_ACTIVE' in pmc.get('analyze', {}):
        a = pmc['analyze']  # the PMC launch alone: its VALU rate against the same peak
        pmc_ms = a['GRBM_GUI_ACTIVE'] / 8 / (CLOCK_GHZ * 1e6)
        pmc_frac = a['SQ_INSTS_VALU'] / (pmc_ms * 1e-3) / 1e9 / peak_g
    step_valu = None
    if pmc:
        tot = sum(per_px(pmc, k, 'SQ_INSTS_VALU') or 0.0 for k in ('analyze', 'resolve', 'index'))
        step_valu = tot * my_px * args.steps / elapsed / 1e9
    f64_px = None
    if pmc:
        a = pmc.get('analyze', {})
        if 'SQ_INSTS_VALU_FMA_F64' in a:
            f64_px = 64 * (a['SQ_INSTS_VALU_ADD_F64'] + a['SQ_INSTS_VALU_MUL_F64'] +
                           2 * a['SQ_INSTS_VALU_FMA_F64']) / pmc['_pixels_per_launch']
    traffic_px = per_px(pmc, 'analyze', 'hbm_bytes')
    bpp = bytes_per_pixel(cfg, meta.n_obs, meta.n_years, runner.fused)
    hbm_gbs = bpp * px_per_launch / (kern_ms * 1e-3) / 1e9
    ref_equiv = f_ref(cfg['years']) * px_per_launch / (kern_ms * 1e-3) / 1e12

    def r(x, n=4):
        return None if x is None else round(x, n)

    res = {
        'metric': 'Mpixels/sec full analyze (%d-yr series)' % cfg['years'],
        'value': round(value, 4), 'unit': 'Mpixels/s', 'n_gpus': world, 'steps': args.steps,
        'warmup': args.warmup, 'ms_per_step': round(elapsed / args.steps * 1e3, 3),
        'higher_is_better': True, 'scaling': 'strong' if mosaic_cfg else 'weak',
        'vs_baseline': None, 'dtype': 'f64',
        'data': 'synthetic (SURVEY.md 8(d) generator, seeded per scene, generated in HBM)',
        'config': {'workload': cfg['desc'], 'pixels_per_scene': P, 'scenes': len(
                       mosaic.scene_pixels), 'total_pixels': mosaic.n_pix, 'years': cfg['years'],
                   'obs': meta.n_obs, 'rules': len(rules), 'line_cost': cfg['line_cost'],
                   'tile_pixels': tile, 'tiles': len(mosaic.tiles), 'tiles_rank0': len(items),
                   'gather': bool(gather),
                   'exchange_pipelined': bool(gather and runner.exchange.can_overlap
                                              and not args.no_overlap),
                   'steps_pipelined': not args.no_overlap,
                   'input': 'int16 bands B1, B2 + index_eqn "%s"' % args.index_eqn +
                            (' (fused into the analyze kernel%s)'
                             % (': JIT kernels, lt_jit.h' if runner.jit is not None else '')
                             if runner.fused else ''),
                   'parallelism': ('one mosaic, tiles round-robin over %d GPU(s), labels sent '
                                   'to rank 0' % world) if mosaic_cfg else
                                  ('one scene per GPU (%d), labels sent to rank 0' % world)},
        # dominant kernel: analyze (>= 80 % of the GPU time), bound by VALU instruction issue —
        # not HBM (145 B/px on c2) and not FP64 throughput (23 % of its VALU work). achieved =
        # the VALU wave-instructions it issues per launch (PMC SQ_INSTS_VALU per pixel, committed
        # summary of this build) x pixels per launch / the launch's live HIP-event time; peak =
        # the measured issue rate of a register-only stream of the same instruction mix at full
        # occupancy, 8 waves per SIMD (tools/valu_peak.hip, profiles/r05_valu_peak.json)
        'roofline': {'bound': 'valu-issue', 'achieved': r(achieved, 2), 'peak': round(peak_g, 2),
                     'unit': 'G VALU wave-instr/s',
                     'frac': r(achieved / peak_g if achieved else None),
                     # against the same mix at the kernel's own occupancy (4 waves per SIMD,
                     # 128 VGPRs): how close the kernel is to what its occupancy allows
                     # the same kernel in joined steps (no resolve of a previous step beside it)
                     'kernel_ms_joined': r(kern_ms_joined, 3),
                     'frac_joined': r(valu_px * px_per_launch / (kern_ms_joined * 1e-3) / 1e9 /
                                      peak_g if valu_px and kern_ms_joined else None),
                     'frac_at_kernel_occupancy': r(
                         achieved / peak_cyc['mix_c2_at_4_waves_g_per_s']
                         if achieved and peak_cyc else None),
                     'peak_source': peak_src, 'peak_waves_per_simd': 8,
                     'cycles_per_valu_at_4_waves': peak_cyc,
                     'build': build, 'pmc_build': pmc.get('_build') if pmc else None,
                     'pmc_matches_build': bool(pmc and pmc['_matches_build']),
                     'pmc_refused': None if pmc_other is None else {
                         'source': pmc_other['_path'], 'build': pmc_other.get('_build'),
                         'reason': 'counters of another kernel build',
                         'valu_instr_per_px': r(per_px(pmc_other, 'analyze', 'SQ_INSTS_VALU'), 2)},
                     'traffic': None if traffic_px is None else round(traffic_px * px_per_launch),
                     'traffic_source': pmc['_path'] if traffic_px is not None else None,
                     'kernel': ('lt_jit_analyze (analyze_body JIT-compiled for this launch, '
                                'lt_jit.h)' if runner.jit is not None else
                                'analyze_fast_kernel'), 'kernel_ms': round(kern_ms, 3),
                     'valu_instr_per_px': r(valu_px, 2),
                     'pmc_valu_issue_frac': r(pmc_frac),  # the PMC launch alone (GRBM cycles at 2.4 GHz)
                     'step_valu_issue_frac': r(step_valu / peak_g if step_valu else None),
                     'fp64': None if f64_px is None else {
                         'achieved': r(f64_px * px_per_launch / (kern_ms * 1e-3) / 1e12, 3),
                         'peak': FP64_PEAK_TFLOPS, 'unit': 'TFLOP/s',
                         'frac': r(f64_px * px_per_launch / (kern_ms * 1e-3) / 1e12 /
                                   FP64_PEAK_TFLOPS)},
                     'hbm': {'achieved': round(hbm_gbs, 2), 'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                             'frac': r(hbm_gbs / HBM_PEAK_GBS),
                             'algorithmic_bytes_per_px': bpp},
                     'source': pmc['_path'] if pmc else None,
                     # the reference algorithm's FP64 work (F_ref) per launch /
                     # launch time: a work-equivalent speed, not a fraction of any peak (the
                     # kernel proves most candidate fits irrelevant and never computes them)
                     'reference_work_equivalent_tflops': round(ref_equiv, 2)},
        'jit': jit,
        'status_numeric_pixels': n_numeric,
        'parity_sample': psample,
        'exchange_check': xcheck,
        'load_stage': {
            'fused': runner.fused,
            'kernel': (('%s (index_eqn "%s" %s, evaluated on each winner\'s '
                        'band values; lt_index_kernel4 below only for comparison)'
                        % ('lt_jit_analyze' if runner.jit is not None else 'analyze_fast_kernel',
                           args.index_eqn, 'inlined into the JIT kernels (lt_jit.h)'
                           if runner.jit is not None else 'as lt_index_lin'))
                       if runner.fused else
                       'lt_index_kernel4 (hiprtc, index_eqn "%s", int16 bands -> int16)'
                       % args.index_eqn),
            'ms_per_launch_overlapped': r(index_ms, 3),
            'alone': {'ms': round(index_alone_ms, 4), 'pixels': it0.tile.n,
                      'bytes': index_bytes,
                      'achieved': round(index_bytes / (index_alone_ms * 1e-3) / 1e9, 1),
                      'peak': HBM_PEAK_GBS, 'unit': 'GB/s',
                      'frac': round(index_bytes / (index_alone_ms * 1e-3) / 1e9 / HBM_PEAK_GBS,
                                    4)}},
        'expand_stage': {'ms_per_launch': round(stages.get('expand', 0.0) / n_launch, 3),
                         'kernel': 'trendline_expand_kernel (per-year planes from the compact '
                                   'trendline, on its own stream beside the next analyze)'}
        if cfg['trendline'] else None,
        'resolve_stage': {'ms_per_launch': round(resolve_ms, 3),
                          'deferred_pixels_last_tile': n_deferred_last,
                          'last_tile_pixels': items[-1].tile.n},
        'joined_steps': joined,
        'end_to_end': e2e,
        'n_gt_1_tiling': None if tiled is None else dict(
            tiled, ratio_to_value=round(tiled['value'] / value, 4)),
    }
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        res['cpu_baseline'] = cpu_baseline(cfg, args.cpu_seconds)
    if rank == 0:
        print(json.dumps(res), flush=True)
    if dist is not None:
        dist.destroy_process_group()
    if psample is not None and psample['mismatched_values'] != 0:
        print('bench: %d values of the parity sample differ from the oracle'
              % psample['mismatched_values'], file=sys.stderr)
        sys.exit(3)
    if xcheck is not None and xcheck['mismatched_tiles'] != 0:
        print('bench: %d exchanged label tiles differ from their owners\' planes'
              % xcheck['mismatched_tiles'], file=sys.stderr)
        sys.exit(3)


if __name__ == '__main__':
    main()
