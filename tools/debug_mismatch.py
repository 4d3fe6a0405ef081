"""Locate and isolate parity mismatches of a bench config's timed launch (debugging aid): runs
bench.py's exact launch for --config, samples pixels against the oracle, lists mismatching pixels
with the differing fields, then re-runs (a) those pixels alone and (b) their whole 64-pixel waves
(original neighbours, original lane positions) through the same JIT path, to tell a per-pixel
defect from a lockstep (wave-neighbour) one. Prints one JSON object."""
import argparse
import json
import os
import sys

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

FIELDS = ['status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude']


def same(a, b):
    if a.dtype.kind == 'f':
        return (a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
    return a == b


def compare(want, got):
    """{column: [differing fields]} (bench.parity_sample's comparison, per pixel)."""
    bad = {}
    m = want['matched'].astype(bool)
    for f in FIELDS:
        g = got[f]
        e = want[f][:g.shape[0]] if g.ndim == 2 else want[f]
        if f in ('class_val', 'onset_year', 'duration', 'magnitude'):
            g, e = np.where(m[:g.shape[0]], g, 0), np.where(m[:g.shape[0]], e, 0)
        s = same(e, g)
        for c in np.where(~s.reshape(-1, s.shape[-1]).all(axis=0))[0]:
            bad.setdefault(int(c), []).append(f)
    return bad


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('--config', default='c3')
    ap.add_argument('--sample', type=int, default=200000)
    ap.add_argument('--pixels', type=int, default=0)
    ap.add_argument('--no-rerun', action='store_true', help='skip the isolation reruns')
    ap.add_argument('--poison', default=None,
                    help='HEX[,HEX]: before step 1 (and 2) fill every SIMD\'s register file with '
                         'this 32-bit pattern (build/bin/libreg_poison.so, tools/reg_poison.hip)')
    ap.add_argument('--stagger', default=None,
                    help='START_MS,SPREAD_MS: before each step hold every wave slot for START_MS, '
                         'then free the slots one by one over SPREAD_MS, so the launch\'s first '
                         'generation of waves starts staggered (build/bin/libstagger.so, '
                         'tools/stagger.hip)')
    ap.add_argument('--hold', default=None,
                    help='WAVES,MS,BIG: before each step start WAVES waves that keep their slots '
                         'for MS (BIG 1: the variant\'s size, 128 VGPRs and its LDS; 0: a few '
                         'VGPRs), so the step runs beside them; where they ran is reported '
                         '(build/bin/libstagger.so, tools/stagger.hip)')
    ap.add_argument('--guard', default=None,
                    help='WAVES,MS: before each step start WAVES guard waves (128 VGPRs each, '
                         'filled with a pattern) that hold their slots for MS beside the step and '
                         'report which of their registers changed (build/bin/libreg_guard.so, '
                         'tools/reg_guard.hip)')
    a = ap.parse_args()
    pois = None
    if a.poison:
        import ctypes
        pl = ctypes.CDLL(os.path.join(ROOT, 'build', 'bin', 'libreg_poison.so'))
        pl.lt_reg_poison.argtypes = [ctypes.c_uint32, ctypes.c_int, ctypes.c_void_p]
        pats = [int(x, 16) for x in a.poison.split(',')]
        pats = pats + pats[-1:] * (2 - len(pats))

        def pois(k):  # one wave per SIMD: 4 waves per CU x 256 CUs, 4x over
            torch.cuda.synchronize()
            rc = pl.lt_reg_poison(pats[k], 4096, ctypes.c_void_p(torch.cuda.current_stream().cuda_stream))
            torch.cuda.synchronize()
            assert rc == 0, rc
    if a.stagger:
        import ctypes
        import time
        sl = ctypes.CDLL(os.path.join(ROOT, 'build', 'bin', 'libstagger.so'))
        sl.lt_stagger.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_double]
        st_start, st_spread = (float(x) for x in a.stagger.split(','))
        inner = pois

        def pois(k):  # noqa: F811 (poison first, if asked, then the blocker)
            if inner:
                inner(k)
            torch.cuda.synchronize()
            rc = sl.lt_stagger(4096, st_start, st_spread)
            assert rc == 0, rc
            time.sleep(st_start / 2000.0)  # the blocker resident before the step is queued
    hold_where = []
    if a.hold:
        import ctypes
        import time
        hl = ctypes.CDLL(os.path.join(ROOT, 'build', 'bin', 'libstagger.so'))
        hl.lt_hold.argtypes = [ctypes.c_int, ctypes.c_double, ctypes.c_int]
        h_waves, h_ms, h_big = a.hold.split(',')
        h_waves, h_ms, h_big = int(h_waves), float(h_ms), int(h_big)
        inner2 = pois

        def pois(k):  # noqa: F811
            if inner2:
                inner2(k)
            torch.cuda.synchronize()
            rc = hl.lt_hold(h_waves, h_ms, h_big)
            assert rc == 0, rc
            time.sleep(0.005)  # the hold waves resident before the step is queued

        def hold_report():
            assert hl.lt_stagger_wait() == 0
            ids = np.zeros(2 * h_waves, dtype=np.uint32)
            assert hl.lt_hold_ids(ids.ctypes.data_as(ctypes.c_void_p), h_waves) == 0
            hw, xcc = ids[0::2].astype(np.int64), ids[1::2].astype(np.int64) & 15
            simd = (xcc << 16) | (((hw >> 13) & 7) << 8) | (((hw >> 12) & 1) << 7) | \
                (((hw >> 8) & 15) << 2) | ((hw >> 4) & 3)
            _, cnt = np.unique(simd, return_counts=True)
            hold_where.append({'simds_used': int(len(cnt)),
                               'waves_per_used_simd': np.bincount(cnt).tolist()})
    guard_found = []
    if a.guard:
        import ctypes
        import time
        gl = ctypes.CDLL(os.path.join(ROOT, 'build', 'bin', 'libreg_guard.so'))
        gl.lt_reg_guard.argtypes = [ctypes.c_int, ctypes.c_double]
        g_waves, g_ms = a.guard.split(',')
        g_waves, g_ms = int(g_waves), float(g_ms)
        inner3 = pois

        def pois(k):  # noqa: F811
            if inner3:
                inner3(k)
            torch.cuda.synchronize()
            assert gl.lt_reg_guard(g_waves, g_ms) == 0
            time.sleep(0.005)  # the guard waves resident before the step is queued

        def guard_report():
            assert gl.lt_reg_guard_wait() == 0
            masks = np.zeros(4 * g_waves, dtype=np.uint32)
            vals = np.zeros(16 * 64 * g_waves, dtype=np.uint32)
            assert gl.lt_reg_guard_read(masks.ctypes.data_as(ctypes.c_void_p),
                                        vals.ctypes.data_as(ctypes.c_void_p), g_waves) == 0
            mk = masks.reshape(g_waves, 4).astype(np.uint64)
            bits = [int(k) for k in range(128) if ((mk[:, k // 32] >> np.uint64(k % 32)) & np.uint64(1)).any()]
            hit = (mk != 0).any(axis=1)
            kept = list(range(8)) + list(range(120, 128))
            v = vals.reshape(g_waves, 16, 64)
            ex = []
            for w in np.where(hit)[0][:4]:
                for i, r in enumerate(kept):
                    d = np.where(v[w, i] != (0xA5A50000 | r))[0]
                    if len(d):
                        ex.append({'wave': int(w), 'reg': 'v%d' % r, 'lanes': len(d),
                                   'values': ['%08x' % x for x in v[w, i, d[:6]]]})
            guard_found.append({'guard_waves_changed': int(hit.sum()), 'registers_changed': bits,
                                'registers_changed_per_wave_hist': np.bincount(
                                    [bin(int(m[0]) | int(m[1]) << 32 | int(m[2]) << 64 |
                                         int(m[3]) << 96).count('1') for m in mk[hit]] or [0]).tolist(),
                                'examples': ex[:16]})
    c = bench.CONFIGS[a.config]
    P = a.pixels or c['pixels']
    eng = get_engine(0)
    dev = eng.device
    m = Mosaic([P], P, 1, 0, 'by_scene')
    items = mosaic_inputs(m, c['years'], c['k'][0], c['k'][1], c['mask'], c['seed'], dev,
                          bench.TARGET)
    params, _ = compile_params(c['line_cost'], c['rules'], c['mode'])
    fn = eng.compile_index(IndexProgram('B1 - B2', band_dtype='int16'))
    r = MosaicRunner(eng, m, params, items, FIELDS, fn)
    if a.stagger or a.hold or a.guard:  # the module loaded and the buffers made before a blocked step is queued
        r.step()
        torch.cuda.synchronize()
    import time as _t
    step_s = []
    if pois:
        pois(0)
    t = _t.perf_counter()
    r.step()
    torch.cuda.current_stream().synchronize()  # the step's own work (not a blocker's)
    step_s.append(_t.perf_counter() - t)
    torch.cuda.synchronize()
    if a.hold:
        hold_report()
    if a.guard:
        guard_report()
    print('step 1 done', file=sys.stderr, flush=True)
    first = {f: r.outs[0][f].clone() for f in FIELDS}
    # determinism: the same launch again, every output plane compared bitwise with the first
    if pois:
        pois(1)
    t = _t.perf_counter()
    r.step()
    torch.cuda.current_stream().synchronize()  # the step's own work (not a blocker's)
    step_s.append(_t.perf_counter() - t)
    torch.cuda.synchronize()
    if a.hold:
        hold_report()
    if a.guard:
        guard_report()
    print('step 2 done', file=sys.stderr, flush=True)
    diff = torch.zeros(P, dtype=torch.bool, device=dev)
    for f in FIELDS:
        a0, a1 = first[f], r.outs[0][f]
        if a0.dtype.is_floating_point:
            a0, a1 = a0.view(torch.int64), a1.view(torch.int64)
        d = a0 != a1
        diff |= d.reshape(-1, P).any(dim=0)
    # where in the launch the run-to-run differences sit: 64 equal bins over the pixel range
    # (blocks are dispatched in order, so a bin is a span of dispatch time), and the first ones
    dix = torch.nonzero(diff).flatten().cpu().numpy()
    where = {'step2_differs_from_step1_pixels': int(diff.sum()),
             'diff_hist64': np.histogram(dix, bins=64, range=(0, P))[0].tolist(),
             'diff_first': dix[:40].tolist(),
             'diff_lane_hist': np.bincount(dix % 64, minlength=64).tolist()}
    print(json.dumps(where), file=sys.stderr, flush=True)
    r.materialise_index(0)
    torch.cuda.synchronize()
    it = items[0]
    rng = np.random.default_rng(5)
    idx = np.sort(rng.choice(P, min(P, a.sample), replace=False))
    cols = torch.from_numpy(idx).to(dev)
    vals = it.values[:, cols].double().cpu().numpy()
    vb = valid_bytes(it.valid[:, cols], it.scene.n_obs).cpu().numpy() if it.valid is not None else None
    want = oracle.analyze_tile(it.scene, params, vals, vb, n_threads=min(os.cpu_count() or 1, 16))
    got = {f: r.outs[0][f][..., cols].cpu().numpy() for f in FIELDS}
    bad = compare(want, got)
    bad_px = [int(idx[c]) for c in sorted(bad)]
    res = {'config': a.config, 'jit_defines': os.environ.get('LT_JIT_DEFINES'),
           'sampled': len(idx), 'mismatching_pixels': len(bad_px),
           'step2_differs_from_step1_pixels': int(diff.sum()),
           'diff_hist64': where['diff_hist64'], 'diff_first': where['diff_first'],
           'diff_lane_hist': where['diff_lane_hist'],
           'mismatching_pixels_that_differ_between_steps': int(diff[cols].cpu().numpy()[sorted(bad)].sum()) if bad else 0,
           'examples': [{'pixel': int(idx[c]), 'lane': int(idx[c]) % 64, 'fields': bad[c],
                         'want': {f: (want[f][..., c].tolist()) for f in bad[c]},
                         'got': {f: (got[f][..., c].tolist()) for f in bad[c]}}
                        for c in sorted(bad)[:12]]}
    if bad_px and not a.no_rerun:
        # (a) alone: the pixels side by side in one small tile; (b) their waves, same lanes
        def rerun(pix):
            pt = torch.tensor(pix, device=dev)
            K = it.bands.shape[0]
            inter = torch.empty((K, len(pix), 2), dtype=torch.int16, device=dev).permute(0, 2, 1)
            inter.copy_(it.bands[:, :, pt])
            valid = it.valid[:, pt].contiguous() if it.valid is not None else None  # bit planes
            out = eng.analyze_tiles(it.scene, params, [(inter, valid)], FIELDS, index=fn)[0]
            torch.cuda.synchronize()
            g = {f: out[f].cpu().numpy() for f in FIELDS}
            pos = [pix.index(p) for p in bad_px]
            sel = torch.tensor(bad_px, device=dev)
            v2 = it.values[:, sel].double().cpu().numpy()  # the index raster (materialised)
            vb2 = valid_bytes(it.valid[:, sel], it.scene.n_obs).cpu().numpy() if it.valid is not None else None
            w2 = oracle.analyze_tile(it.scene, params, v2, vb2)
            g2 = {f: g[f][..., pos] for f in FIELDS}
            return len(compare(w2, g2))
        res['alone_mismatching'] = rerun(bad_px)
        waves = sorted({p // 64 for p in bad_px})
        wpix = [p for w in waves for p in range(w * 64, min(P, w * 64 + 64))]
        res['in_their_waves_mismatching'] = rerun(wpix)
    # which code ran: disk_hits counts the LT_JIT_OVERRIDE_DIR code objects loaded (or cached)
    res['jit'] = {k: v for k, v in eng.jit_stats().items() if k != 'last_error'}
    res['jit_override_dir'] = os.environ.get('LT_JIT_OVERRIDE_DIR')
    res['poison'] = a.poison
    res['stagger'] = a.stagger
    res['hold'] = a.hold
    res['hold_where'] = hold_where
    res['guard'] = a.guard
    res['guard_found'] = guard_found
    res['step_wall_ms'] = [round(x * 1e3, 3) for x in step_s]
    print(json.dumps(res), flush=True)


if __name__ == '__main__':
    main()
