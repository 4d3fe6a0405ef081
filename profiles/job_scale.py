"""Scale run of the local job runner (land_trendr_amd/job.py) on a multi-Mpx synthetic job.

The job directory has the layout of tests/jobfixture.make_job: int16 two-band 'ledaps' rasters
(B1 = B2 + index), every third one tar.gz-compressed as the reference's S3 objects are, cloud masks
for the even dates, one raster with a shifted geotransform. The job runs setup -> parse ->
analysis -> output on cuda:0 (LZW GeoTIFF label rasters, assembled on the GPU); the script reports
the wall time of each step and checks a random sample of pixels against the CPU oracle (the
oracle is the checker here, as in tests/test_gpu_job.py).

Usage (GPU box): python profiles/job_scale.py ROWS COLS YEARS OUT.json [--trendline]
"""
import json
import os
import shutil
import sys
import tempfile
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, 'tests'))


def main():
    rows, cols, years, out_json = int(sys.argv[1]), int(sys.argv[2]), int(sys.argv[3]), sys.argv[4]
    trendline = '--trendline' in sys.argv
    import torch
    from golden_io import _bits_equal
    from jobfixture import SETTINGS, make_job
    from land_trendr_amd import _abi
    from land_trendr_amd.job import LocalJob
    from land_trendr_amd.scene import build_scene, parse_date
    from land_trendr_amd.settings import compile_params
    from oracle import oracle

    root = tempfile.mkdtemp(prefix='ltjob_', dir='/tmp')
    try:
        t = {}
        t0 = time.time()
        make_job(root, rows=rows, cols=cols, n_years=years, seed=7)
        t['make_job_s'] = time.time() - t0
        j = LocalJob(root, 'synth', device=0, tile_pixels=1 << 22, trendline=trendline,
                     on_error='skip')
        for step in ('setup', 'parse', 'analyze', 'output'):
            t0 = time.time()
            res = getattr(j, step)()
            torch.cuda.synchronize()
            t[step + '_s'] = time.time() - t0
            print(step, '%.2f s' % t[step + '_s'], flush=True)
        files = res
        st = j.stack
        P = st['n_pix']
        rng = np.random.default_rng(11)
        cols_s = np.sort(rng.choice(P, min(P, 20000), replace=False))
        idx = (st['bands'][:, 0, cols_s].astype(np.int32) - st['bands'][:, 1, cols_s]).astype(
            np.int16)
        meta = build_scene(st['dates'], parse_date(SETTINGS['target_date']))
        params, _ = compile_params(SETTINGS['line_cost'], SETTINGS['label_rules'])
        exp = oracle.analyze_tile(meta, params, idx.astype(np.float64),
                                  np.ascontiguousarray(st['valid'][:, cols_s]),
                                  n_threads=os.cpu_count() or 1)
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
        out_bytes = sum(os.path.getsize(p) for v in files.values() for p in v)
        res = {'rows': rows, 'cols': cols, 'pixels': P, 'years': years, 'obs': int(meta.n_obs),
               'trendline': trendline, 'rules': len(SETTINGS['label_rules']),
               'times': {k: round(v, 3) for k, v in t.items()},
               'analysis_mpx_per_s': round(P / t['analyze_s'] / 1e6, 2),
               'output_rasters': len(files), 'output_bytes': out_bytes,
               'sample_pixels': int(len(cols_s)), 'sample_mismatches': mism,
               'sample_status_nonzero': int((exp['status'] & ~_abi.LT_ST_EMPTY != 0).sum())}
        json.dump(res, open(out_json, 'w'), indent=1)
        print(json.dumps(res))
        assert not any(mism.values()), mism
    finally:
        shutil.rmtree(root, ignore_errors=True)


if __name__ == '__main__':
    main()
