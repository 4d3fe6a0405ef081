"""Job-level throughput: the whole local job
(land_trendr_amd/job.py: setup -> parse -> analysis -> output) on a Landsat-scene-sized stack,
timed per stage.

The stack is generated on the box, not shipped: the seeded SURVEY §8(d) scene (synth.make_scene,
on the GPU) written as one LZW GeoTIFF per acquisition — two int16 bands (B1, B2 = B1 - index),
GDAL-like ~8 KB strips, north-up georeferencing — named like the reference's LEDAPS keys
(filename2date reads the year and day of year), plus settings.json ('B1 - B2', line_cost 10, one
GD rule: the c2 configuration). The job then runs exactly as `python -m land_trendr_amd.job`
would, on cuda:0, and the script prints one JSON line:
  * per stage: seconds; parse also as decoded band GB/s and Mpx/s;
  * the whole job in Mpx/s (setup + parse + analysis + output);
  * a seeded sample of pixels re-analysed by the CPU oracle from the job's own ingested bands,
    compared with every output plane (the oracle is the checker here, never a producer).

    python tools/job_bench.py --rows 7000 --cols 7000 --years 30 [--trendline] [--check 20000]
"""
import argparse
import json
import os
import shutil
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))

GT = (500000.0, 30.0, 0.0, 4200000.0, 0.0, -30.0)
SETTINGS = {'index_eqn': 'B1 - B2', 'line_cost': 10, 'target_date': '2014-07-01',
            'label_rules': [{'name': 'gd', 'val': 1, 'change_type': 'GD'}]}


def make_stack(root, job, rows, cols, years, seed, mask_prob):
    """The job directory: one two-band int16 LZW GeoTIFF per acquisition date (raster order:
    pixel p of the scene at row p // cols, column p % cols) and, with mask_prob > 0, a cloudmask
    raster per date. Returns (seconds, bytes written)."""
    import torch
    from land_trendr_amd.raster import write_geotiff
    from land_trendr_amd.synth import make_scene
    t0 = time.time()
    rdir = os.path.join(root, job, 'input', 'rasters')
    os.makedirs(rdir, exist_ok=True)
    with open(os.path.join(root, job, 'input', 'settings.json'), 'w') as f:
        json.dump(SETTINGS, f)
    dev = 'cuda' if torch.cuda.is_available() else 'cpu'
    sc = make_scene(rows * cols, n_years=years, k_min=1, k_max=1, mask_prob=mask_prob, seed=seed,
                    device=dev, with_bands=True)
    sc.values = None
    nbytes = 0
    for k, d in enumerate(sc.dates):
        stem = 'LT5045029_%d_%03d_20120124_104859' % (d.year, d.timetuple().tm_yday)
        img = sc.bands[k].reshape(2, rows, cols).cpu().numpy()
        fn = os.path.join(rdir, stem + '_ledaps.tif')
        write_geotiff(fn, img, geotransform=GT, nodata=None)
        nbytes += os.path.getsize(fn)
        if sc.valid is not None:
            m = sc.valid[k].reshape(rows, cols).cpu().numpy()
            mf = os.path.join(rdir, stem + '_cloudmask.tif')
            write_geotiff(mf, m, geotransform=GT, nodata=None)
            nbytes += os.path.getsize(mf)
        if k % 5 == 4:
            print('  %d rasters written (%.0f s)' % (k + 1, time.time() - t0), file=sys.stderr,
                  flush=True)
    del sc
    if dev == 'cuda':
        torch.cuda.empty_cache()
    return time.time() - t0, nbytes


def check_sample(j, n, seed=11):
    """A seeded sample of the job's pixels: the oracle on the job's own ingested bands vs every
    output plane. Returns (pixels, {plane: mismatches})."""
    from golden_io import _bits_equal
    from land_trendr_amd import _abi
    from land_trendr_amd.ingest import host_threads
    from land_trendr_amd.scene import build_scene, parse_date
    from land_trendr_amd.settings import compile_params
    from oracle import oracle
    st = j.stack
    P = st['n_pix']
    cols_s = np.sort(np.random.default_rng(seed).choice(P, min(P, n), replace=False))
    b = st['bands'][:, :, cols_s]
    idx = (b[:, 0].astype(np.int32) - b[:, 1]).astype(np.int16)
    meta = build_scene(st['dates'], parse_date(SETTINGS['target_date']))
    params, _ = compile_params(SETTINGS['line_cost'], SETTINGS['label_rules'])
    exp = oracle.analyze_tile(meta, params, idx.astype(np.float64),
                              np.ascontiguousarray(st['valid'][:, cols_s]),
                              n_threads=host_threads())
    bad = np.flatnonzero(exp['status'] & ~_abi.LT_ST_EMPTY)  # on_error='skip'
    exp['matched'][:, bad] = 0
    mism = {}
    for k, a in j.planes.items():
        a = a[..., cols_s]
        e = exp[k][:a.shape[0]] if a.ndim == 2 else exp[k]
        if k == 'winner':
            e = e.copy()
            e[:, bad] = -1
        if k in ('onset_year', 'duration', 'class_val', 'magnitude', 'initial_val'):
            m = exp['matched'][:a.shape[0]].astype(bool)
            a, e = np.where(m, a, 0), np.where(m, e, 0)
        same = _bits_equal(a, e) if a.dtype.kind == 'f' else (a == e)
        mism[k] = int((~same).sum())
    return len(cols_s), mism


def diag(j):
    """Where parse and output spend their time: one input raster opened and decoded on 1 and on
    all host threads; output() run again under cProfile (top entries to stderr)."""
    import cProfile
    import io
    import pstats
    from land_trendr_amd.geotiff import GeoTiff
    from land_trendr_amd.ingest import host_threads
    d = {}
    fn = j.rast_fns[1]
    t0 = time.time()
    g = GeoTiff(fn)
    d['open_s'] = round(time.time() - t0, 3)
    for th in (1, host_threads()):
        t0 = time.time()
        a = g.read(threads=th)
        d['decode_%d_threads_s' % th] = round(time.time() - t0, 3)
        d['decode_%d_threads_gb_per_s' % th] = round(a.nbytes / (time.time() - t0) / 1e9, 3)
    pr = cProfile.Profile()
    t0 = time.time()
    pr.enable()
    j.output()
    pr.disable()
    d['output_again_s'] = round(time.time() - t0, 3)
    buf = io.StringIO()
    pstats.Stats(pr, stream=buf).sort_stats('cumulative').print_stats(25)
    print(buf.getvalue(), file=sys.stderr, flush=True)
    return d


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--rows', type=int, default=7000)
    ap.add_argument('--cols', type=int, default=7000)
    ap.add_argument('--years', type=int, default=30)
    ap.add_argument('--mask', type=float, default=0.0)
    ap.add_argument('--seed', type=int, default=1000)
    ap.add_argument('--tile', type=int, default=1 << 24, help='job tile pixels')
    ap.add_argument('--trendline', action='store_true',
                    help='also the per-year trendline rasters (8 per acquisition date)')
    ap.add_argument('--check', type=int, default=20000, help='oracle sample (0: none)')
    ap.add_argument('--work', default='/tmp/ltjob_bench')
    ap.add_argument('--keep', action='store_true')
    ap.add_argument('--diag', action='store_true',
                    help='after the job: one raster opened / decoded on 1 and all threads, and a '
                         'cProfile of output() run again (stderr)')
    ap.add_argument('--profile', default=None, choices=('setup', 'parse', 'analyze', 'output'),
                    help='run this step under cProfile (top entries by own time to stderr)')
    a = ap.parse_args()
    import torch
    from land_trendr_amd.ingest import host_threads
    from land_trendr_amd.job import LocalJob
    shutil.rmtree(a.work, ignore_errors=True)
    os.makedirs(a.work)
    try:
        gen_s, in_bytes = make_stack(a.work, 'bench', a.rows, a.cols, a.years, a.seed, a.mask)
        print('stack written: %.1f s, %.2f GB' % (gen_s, in_bytes / 1e9), file=sys.stderr,
              flush=True)
        P = a.rows * a.cols
        j = LocalJob(a.work, 'bench', device=0, tile_pixels=a.tile, trendline=a.trendline,
                     on_error='skip')
        t = {}
        files = None
        for step in ('setup', 'parse', 'analyze', 'output'):
            t0 = time.time()
            if step == a.profile:  # this step under cProfile (top entries to stderr)
                import cProfile
                import io
                import pstats
                pr = cProfile.Profile()
                pr.enable()
                res = getattr(j, step)()
                torch.cuda.synchronize()
                pr.disable()
                buf = io.StringIO()
                pstats.Stats(pr, stream=buf).sort_stats('tottime').print_stats(25)
                print(buf.getvalue(), file=sys.stderr, flush=True)
            else:
                res = getattr(j, step)()
            torch.cuda.synchronize()
            t[step] = time.time() - t0
            if step == 'output':
                files = res
            print('%s %.2f s' % (step, t[step]), file=sys.stderr, flush=True)
        total = sum(t.values())
        K = len(j.stack['dates'])
        decoded = K * 2 * P * 2  # two int16 bands per acquisition
        out_bytes = sum(os.path.getsize(p) for v in files.values() for p in v)
        res = {'workload': 'job: %d x %d px x %d acquisitions, 2 int16 bands each (LZW GeoTIFF), '
                           "index_eqn 'B1 - B2', line_cost 10, one GD rule%s"
                           % (a.rows, a.cols, K, ', per-year trendline rasters' if a.trendline
                              else ''),
               'pixels': P, 'acquisitions': K, 'host_threads': host_threads(),
               'input_bytes': in_bytes, 'generate_s': round(gen_s, 2),
               'seconds': {k: round(v, 3) for k, v in t.items()},
               'job_s': round(total, 3), 'job_mpx_per_s': round(P / total / 1e6, 3),
               'parse_decoded_gb_per_s': round(decoded / t['parse'] / 1e9, 3),
               'parse_mpx_per_s': round(P / t['parse'] / 1e6, 2),
               'analyze_mpx_per_s': round(P / t['analyze'] / 1e6, 2),
               'output_rasters': len(files), 'output_bytes': out_bytes,
               'raster_order': j._raster_hw is not None,
               'jit': getattr(j, 'jit_stats', None),
               'analyze_parts_s': {k: round(v, 3) for k, v in getattr(j, 'analyze_s', {}).items()},
               'upload': os.environ.get('LT_JOB_UPLOAD', 'whole')}
        if a.diag:
            res['diag'] = diag(j)
        if a.check > 0:
            n, mism = check_sample(j, a.check)
            res['check'] = {'pixels': n, 'mismatches': mism,
                            'checker': 'oracle/lt_oracle.c on the job\'s ingested bands'}
        print(json.dumps(res), flush=True)
        if a.check > 0 and any(res['check']['mismatches'].values()):
            sys.exit(3)
    finally:
        if not a.keep:
            shutil.rmtree(a.work, ignore_errors=True)


if __name__ == '__main__':
    main()
