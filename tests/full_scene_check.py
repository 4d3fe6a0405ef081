"""Whole-scene parity check (a script, not a pytest case: minutes of oracle time).

Runs bench.py's exact input and layout on cuda:0 — rank 0's seeded scene of a BASELINE config
(SURVEY.md 8(d) generator), int16 bands -> hiprtc index_eqn 'B1 - B2' on the load stream ->
lt_analyze_tiles_after in 16.8 Mpx tiles — then re-analyses EVERY pixel with the CPU oracle
(oracle/lt_oracle.c, test infrastructure) in chunks and compares the label rasters, status, the
fitted values and the vertex flags bit for bit. Prints one progress line per chunk and writes a
JSON summary.

Usage (GPU box): python tests/full_scene_check.py --config c2 --out gpurun_out/full_c2.json
(--first/--last: re-analyse one pixel range of the whole scene, to split a long check in calls)
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
from land_trendr_amd.engine import get_engine  # noqa: E402
from land_trendr_amd.index_eqn import IndexProgram  # noqa: E402
from land_trendr_amd.scene import build_scene, parse_date  # noqa: E402
from land_trendr_amd.settings import compile_params  # noqa: E402
from land_trendr_amd.synth import make_scene  # noqa: E402
from oracle import oracle  # noqa: E402

FIELDS = ('status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude', 'val_fit',
          'vertex')


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c2', choices=sorted(bench.CONFIGS))
    ap.add_argument('--pixels', type=int, default=0)
    ap.add_argument('--chunk', type=int, default=1 << 21)
    ap.add_argument('--first', type=int, default=0, help='first pixel the oracle re-analyses')
    ap.add_argument('--last', type=int, default=0, help='end of that range (0: the scene end)')
    ap.add_argument('--out', default='')
    args = ap.parse_args()
    c = bench.CONFIGS[args.config]
    P = args.pixels or c['pixels']
    dev = torch.device('cuda', 0)
    t0 = time.time()
    sc = make_scene(P, n_years=c['years'], k_min=c['k'][0], k_max=c['k'][1],
                    mask_prob=c['mask'], seed=1000, device=dev, with_bands=True)
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    params, _ = compile_params(c['line_cost'], c['rules'], c['mode'])
    eng = get_engine(0)
    fn = eng.compile_index(IndexProgram('B1 - B2', band_dtype='int16'))
    index = torch.empty((meta.n_obs, P), dtype=torch.int16, device=dev)
    out = eng.alloc_outputs(meta.n_years, params.n_rules, P, FIELDS)
    tile = 1 << 24
    spans = [(a, min(P, a + tile)) for a in range(0, P, tile)]
    main_s = torch.cuda.current_stream(dev)
    load = torch.cuda.Stream(dev)
    load.wait_stream(main_s)
    ready = []
    with torch.cuda.stream(load):
        for a, b in spans:
            eng.index_tile(fn, sc.bands[:, :, a:b], out=index[:, a:b])
            ev = torch.cuda.Event()
            ev.record()
            ready.append(ev)
    eng.analyze_tiles(meta, params,
                      [(index[:, a:b], sc.valid[:, a:b] if sc.valid is not None else None)
                       for a, b in spans], FIELDS,
                      outs=[{f: t[..., a:b] for f, t in out.items()} for a, b in spans],
                      ready=ready)
    torch.cuda.synchronize()
    print('gpu done: %d px in %d tiles, %.1f s' % (P, len(spans), time.time() - t0), flush=True)
    assert torch.equal(index.to(torch.float64), sc.values), 'index raster != synthetic index'
    threads = min(len(os.sched_getaffinity(0)), 64)
    diff = {f: 0 for f in FIELDS}
    end = args.last or P
    for a in range(args.first, end, args.chunk):
        b = min(end, a + args.chunk)
        vals = sc.values[:, a:b].cpu().numpy()
        valid = sc.valid[:, a:b].cpu().numpy() if sc.valid is not None else None
        want = oracle.analyze_tile(meta, params, vals, valid, n_threads=threads)
        for f in FIELDS:
            x, y = want[f], out[f][..., a:b].cpu().numpy()
            same = ((x.view(np.int64) == y.view(np.int64)) | (np.isnan(x) & np.isnan(y))
                    if x.dtype.kind == 'f' else x == y)
            diff[f] += int((~same).sum())
        print('oracle %d/%d px, differing values so far %d, %.0f s' % (
            b, end, sum(diff.values()), time.time() - t0), flush=True)
    res = {'config': args.config, 'pixels': P, 'checked': [args.first, end],
           'tile_pixels': tile, 'seed': 1000,
           'input': 'int16 bands + index_eqn "B1 - B2" (bench.py rank 0 scene)',
           'fields': list(FIELDS), 'differing_values': diff,
           'bit_exact': sum(diff.values()) == 0, 'oracle_threads': threads,
           'seconds': round(time.time() - t0, 1)}
    print(json.dumps(res), flush=True)
    if args.out:
        with open(args.out, 'w') as fh:
            json.dump(res, fh, indent=1)
    return 0 if res['bit_exact'] else 1


if __name__ == '__main__':
    sys.exit(main())
