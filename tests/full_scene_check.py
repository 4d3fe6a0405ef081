"""Whole-scene parity check (a script, not a pytest case: minutes of oracle time).

Runs bench.py's exact input and code path on cuda:0 — rank 0's seeded scene of a BASELINE config
(SURVEY.md 8(d) generator, synth.mosaic_inputs), int16 bands -> hiprtc index_eqn 'B1 - B2' on the
load stream -> lt_analyze_tiles_after in 16.8 Mpx tiles (runner.MosaicRunner) — then re-analyses
EVERY pixel of a range with the CPU oracle (oracle/lt_oracle.c, test infrastructure), fed the
index raster the load kernel wrote, and compares every output field the config writes bit for
bit: status and the label rasters, and the per-year planes (c2/c3: val_fit, vertex; c5: all nine
trendline planes — winner, val_raw, val_fit, fit_m, fit_b, right_m, right_b, spike, vertex).
Prints one progress line per chunk and writes a JSON summary.

Usage (GPU box): python tests/full_scene_check.py --config c2 --out gpurun_out/full_c2.json
(--first/--last: re-analyse one pixel range of the scene, to split a long check over calls;
--labels-only: only the label rasters, as bench.py requests them for c2/c3, so the analyze kernel
takes its certified labels-only path; --whole --bench-fields: bench.py's exact timed launch on
one GPU, the whole scene as one tile with bench's fields)
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

import bench  # noqa: E402
from land_trendr_amd.distributed import Mosaic  # noqa: E402
from land_trendr_amd.engine import get_engine, valid_bytes  # noqa: E402
from land_trendr_amd.index_eqn import IndexProgram  # noqa: E402
from land_trendr_amd.runner import MosaicRunner  # noqa: E402
from land_trendr_amd.settings import compile_params  # noqa: E402
from land_trendr_amd.synth import mosaic_inputs  # noqa: E402
from oracle import oracle  # noqa: E402

LABELS = ('status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c2', choices=['c2', 'c3', 'c5'])
    ap.add_argument('--pixels', type=int, default=0)
    ap.add_argument('--chunk', type=int, default=1 << 21)
    ap.add_argument('--first', type=int, default=0, help='first pixel the oracle re-analyses')
    ap.add_argument('--last', type=int, default=0, help='end of that range (0: the scene end)')
    ap.add_argument('--threads', type=int, default=0)
    ap.add_argument('--labels-only', action='store_true',
                    help="the bench's own fields (label rasters only, the analyze kernel's "
                         "certified labels path) instead of adding val_fit / vertex")
    ap.add_argument('--whole', action='store_true',
                    help="bench.py's exact launch on one GPU for a labels-only config: the whole "
                         "scene as one tile (one analyze launch, one resolve launch)")
    ap.add_argument('--bench-fields', action='store_true',
                    help="exactly bench.py's output fields (with --labels-only: without "
                         "initial_val), so the kernel instance is the one bench.py times")
    ap.add_argument('--out', default='')
    args = ap.parse_args()
    c = bench.CONFIGS[args.config]
    P = args.pixels or c['pixels']
    if args.labels_only:
        fields = LABELS if args.bench_fields else LABELS + ('initial_val',)
    else:
        fields = LABELS + (tuple(bench.TRENDLINE_FIELDS) if c['trendline'] else
                           ('val_fit', 'vertex'))
    t0 = time.time()
    eng = get_engine(0)
    m = Mosaic([P], P if args.whole else 1 << 24, 1, 0, 'by_scene')
    items = mosaic_inputs(m, c['years'], c['k'][0], c['k'][1], c['mask'], c['seed'],
                          eng.device, bench.TARGET)
    params, _ = compile_params(c['line_cost'], c['rules'], c['mode'])
    fn = eng.compile_index(IndexProgram('B1 - B2', band_dtype='int16'))
    runner = MosaicRunner(eng, m, params, items, fields, fn)
    runner.step()
    for k in range(len(items)):  # the fused steps read the bands: the oracle reads their raster
        runner.materialise_index(k)
    torch.cuda.synchronize()
    print('gpu done: %d px in %d tiles, %.1f s' % (P, len(items), time.time() - t0), flush=True)
    threads = args.threads or min(len(os.sched_getaffinity(0)), 64)
    diff = {f: 0 for f in fields}
    end = args.last or P
    meta = items[0].scene
    for a in range(args.first, end, args.chunk):
        b = min(end, a + args.chunk)
        for k, it in enumerate(items):  # the chunk's part in each tile
            lo, hi = max(a, it.tile.p0), min(b, it.tile.p1)
            if lo >= hi:
                continue
            sl = slice(lo - it.tile.p0, hi - it.tile.p0)
            vals = it.values[:, sl].double().cpu().numpy()
            valid = (valid_bytes(it.valid[:, sl], meta.n_obs).cpu().numpy()
                     if it.valid is not None else None)
            want = oracle.analyze_tile(meta, params, vals, valid, n_threads=threads)
            for f in fields:
                x = want[f]
                y = runner.outs[k][f][..., sl].cpu().numpy()
                x = x[:y.shape[0]] if x.ndim == 2 else x
                same = ((x.view(np.int64) == y.view(np.int64)) | (np.isnan(x) & np.isnan(y))
                        if x.dtype.kind == 'f' else x == y)
                diff[f] += int((~same).sum())
        print('oracle %d/%d px, differing values so far %d, %.0f s' % (
            b, end, sum(diff.values()), time.time() - t0), flush=True)
    res = {'config': args.config, 'labels_only': args.labels_only, 'pixels': P,
           'bench_fields': args.bench_fields, 'whole_scene_launch': args.whole,
           'kernel': 'lt_jit_analyze (JIT)' if runner.jit is not None else 'precompiled',
           'deferred_pixels_last_launch': eng.last_deferred(),
           'checked': [args.first, end],
           'tile_pixels': m.tile, 'seed': c['seed'],
           'input': 'int16 bands + index_eqn "B1 - B2" (bench.py rank 0 scene, runner path)',
           'fields': list(fields), 'differing_values': diff,
           'bit_exact': sum(diff.values()) == 0, 'oracle_threads': threads,
           'seconds': round(time.time() - t0, 1)}
    print(json.dumps(res), flush=True)
    if args.out:
        with open(args.out, 'w') as fh:
            json.dump(res, fh, indent=1)
    return 0 if res['bit_exact'] else 1


if __name__ == '__main__':
    sys.exit(main())
