"""Cost of non-integer index data: one 4.2 Mpx x 30-year tile, labels only
(the c2 rule), analysed with the index raster as int16 (bench's path), as float32 values with a
fractional part (binary32-exact: the lazy path with a binary32 LDS series) and as float64
NDVI-like values (not binary32-exact: every pixel takes the binary64 resolve stage). Reports the
time per call (HIP events around lt_analyze_tile) and the deferred-pixel counts; a 4096-pixel
sample of each is checked against the oracle.

Usage (GPU box): python profiles/float_index.py OUT.json
"""
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    from land_trendr_amd.engine import LABEL_FIELDS, get_engine
    from land_trendr_amd.scene import build_scene, parse_date
    from land_trendr_amd.settings import compile_params
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    P = 1 << 22
    sc = make_scene(P, n_years=30, seed=21, device='cuda')
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    params, _ = compile_params(10.0, [{'name': 'gd', 'val': 1, 'change_type': 'GD'}])
    eng = get_engine(0)
    base = sc.values  # integer-valued float64 [K, P]
    g = torch.Generator(device='cuda').manual_seed(5)
    frac = torch.randint(0, 8, base.shape, generator=g, device='cuda').double() / 8.0
    kinds = {
        'int16': base.to(torch.int16),
        'float32_eighths': (base + frac).float(),          # binary32-exact, non-integer
        'float64_ndvi': (base / 2000.0 + frac * 1e-3),      # NDVI-like: not binary32-exact
    }
    fields = LABEL_FIELDS + ('initial_val',)
    res = {'pixels': P, 'years': 30, 'fields': list(fields), 'kinds': {}}
    rng = np.random.default_rng(3)
    sample = np.sort(rng.choice(P, 4096, replace=False))
    for name, vals in kinds.items():
        out = eng.analyze_tile(meta, params, vals, None, fields)  # warm-up (and compile)
        torch.cuda.synchronize()
        ts = []
        for _ in range(3):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            e0.record()
            out = eng.analyze_tile(meta, params, vals, None, fields, out=out)
            e1.record()
            torch.cuda.synchronize()
            ts.append(e0.elapsed_time(e1))
        defer = eng.last_deferred() if hasattr(eng, 'last_deferred') else None
        v = vals[:, sample].double().cpu().numpy()
        want = oracle.analyze_tile(meta, params, v, None, n_threads=os.cpu_count() or 1)
        bad = 0
        for f in fields:
            a, b = want[f], out[f][..., sample].cpu().numpy()
            same = ((a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
                    if a.dtype.kind == 'f' else a == b)
            bad += int((~same).sum())
        ms = min(ts)
        res['kinds'][name] = {'ms_per_tile': round(ms, 3), 'mpx_per_s': round(P / ms / 1e3, 1),
                              'deferred': defer, 'sample_mismatches': bad}
        print(name, res['kinds'][name], flush=True)
    json.dump(res, open(sys.argv[1], 'w'), indent=1)
    assert all(k['sample_mismatches'] == 0 for k in res['kinds'].values())


if __name__ == '__main__':
    main()
