"""JIT module lifecycle on the GPU (lt_jit.h, lt_abi.hip): the
kernel headers embedded in liblt_hip.so, the precompiled fallback when a module cannot be built or
is still compiling, asynchronous compiles, and the least-recently-used module cap. Every path is
checked against the oracle (oracle/lt_oracle.c, fed the load kernel's index raster of the same
bands, as the reference's apply_grid reads float(val) of the rast_algebra raster,
/root/reference/utils.py:447-484, :357)."""
import os
import zlib

import numpy as np
import pytest
import torch

from land_trendr_amd import index_eqn
from land_trendr_amd.engine import Engine, valid_bytes
from land_trendr_amd.scene import build_scene, parse_date
from land_trendr_amd.settings import compile_params

pytestmark = pytest.mark.gpu
FIELDS = ('status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude', 'val_fit',
          'vertex')


def _bits_equal(a, b):
    if a.dtype.kind == 'f':
        return (a.view(np.int64) == b.view(np.int64)) | (np.isnan(a) & np.isnan(b))
    return a == b


def _tiles(eng, eqn, masked, n_tiles=2, P=3000, seed=0):
    """n_tiles tiles of one scene: pixel-interleaved int16 band pairs (the fused layout), an
    optional mask as bit planes."""
    from land_trendr_amd.engine import pack_valid_bits
    rng = np.random.default_rng(zlib.crc32(('%s%s%d' % (eqn, masked, seed)).encode()))
    Y = 30
    k_per = rng.integers(1, 4, Y) if masked else np.ones(Y, int)
    dates = ['%d-%02d-%02d' % (1990 + y, rng.integers(5, 10), rng.integers(1, 28))
             for y in range(Y) for _ in range(k_per[y])]
    K = len(dates)
    meta = build_scene(dates, parse_date('2014-07-01'))
    tiles = []
    for _ in range(n_tiles):
        base = rng.integers(-3000, 3001, (1, 2, P))
        b = np.clip(base + rng.integers(-400, 401, (K, 2, P)), -32768, 32767).astype(np.int16)
        inter = torch.empty((K, P, 2), dtype=torch.int16, device=eng.device).permute(0, 2, 1)
        inter.copy_(torch.from_numpy(b))
        valid = None
        if masked:
            valid = pack_valid_bits(torch.from_numpy(
                (rng.random((K, P)) > 0.2).astype(np.uint8)).to(eng.device))
        tiles.append((inter, valid))
    params, _ = compile_params(10.0, [{'name': 'gd', 'val': 1, 'change_type': 'GD'},
                                      {'name': 'ld', 'val': 2, 'change_type': 'LD',
                                       'duration': ['>', 2]}])
    return meta, params, tiles


def _check_vs_oracle(eng, fn, meta, params, tiles, outs):
    from oracle import oracle
    for (bands, valid), got in zip(tiles, outs):
        idx = eng.index_tile(fn, bands)
        vb = valid_bytes(valid, meta.n_obs)
        want = oracle.analyze_tile(meta, params, idx.double().cpu().numpy(),
                                   None if vb is None else vb.cpu().numpy(),
                                   n_threads=min(os.cpu_count() or 1, 16))
        for f in FIELDS:
            g = got[f].cpu().numpy()
            w = want[f][:g.shape[0]] if g.ndim == 2 else want[f]
            if f in ('class_val', 'onset_year', 'duration', 'magnitude'):
                mt = want['matched'].astype(bool)[:g.shape[0]]
                g, w = np.where(mt, g, 0), np.where(mt, w, 0)
            assert _bits_equal(w, g).all(), (f, int((~_bits_equal(w, g)).sum()))


@pytest.mark.parametrize('eqn', ['B1 - B2', '(B1 - B2) * 2 / 2'])
@pytest.mark.parametrize('masked', [False, True])
def test_jit_failure_falls_back_to_precompiled_kernels(tmp_path, monkeypatch, eqn, masked):
    """LT_SRC_DIR naming an empty directory makes every JIT compile fail (no kernel headers): the
    tiles then run on the precompiled kernels — a linear program through its lt_index_lin form,
    '(B1 - B2) * 2 / 2' through its index raster written by the load kernel into the context's
    scratch — with the oracle's results, and lt_ctx_jit_stats reports the fallback."""
    monkeypatch.setenv('LT_SRC_DIR', str(tmp_path))
    eng = Engine(0)
    try:
        fn = eng.compile_index(index_eqn.IndexProgram(eqn, band_dtype='int16'))
        assert (fn.lin is not None) == (eqn == 'B1 - B2')
        meta, params, tiles = _tiles(eng, eqn, masked)
        outs = eng.analyze_tiles(meta, params, tiles, FIELDS, index=fn)
        torch.cuda.synchronize()
        st = eng.jit_stats()
        assert st['fallback_tiles'] == len(tiles) and st['jit_tiles'] == 0, st
        assert st['failures'] >= 1 and 'not found' in st['last_error'], st
        _check_vs_oracle(eng, fn, meta, params, tiles, outs)
    finally:
        eng.close()


def test_embedded_headers_need_no_source_tree(tmp_path):
    """The library compiles its JIT kernels from the headers embedded in it: a copy of
    liblt_hip.so in a directory with no csrc/ tree beside it (LT_HIP_LIB) still builds and runs
    the JIT module (a child process: the copy is a second library instance)."""
    import shutil
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    lib = tmp_path / 'liblt_hip.so'
    shutil.copy(os.path.join(root, 'land_trendr_amd', 'liblt_hip.so'), lib)
    code = r'''
import sys, torch
sys.path.insert(0, %r)
from land_trendr_amd.engine import Engine
from land_trendr_amd import index_eqn
import tests.test_gpu_jit as t
eng = Engine(0)
fn = eng.compile_index(index_eqn.IndexProgram('(B1 - B2) * 2 / 2', band_dtype='int16'))
meta, params, tiles = t._tiles(eng, '(B1 - B2) * 2 / 2', True, n_tiles=1)
outs = eng.analyze_tiles(meta, params, tiles, t.FIELDS, index=fn)
torch.cuda.synchronize()
st = eng.jit_stats()
assert st['jit_tiles'] == 1 and st['fallback_tiles'] == 0, st
t._check_vs_oracle(eng, fn, meta, params, tiles, outs)
print('ok', st)
''' % root
    env = dict(os.environ, LT_HIP_LIB=str(lib), LT_JIT_CACHE=str(tmp_path / 'jit'))
    env.pop('LT_SRC_DIR', None)
    r = subprocess.run([sys.executable, '-c', code], env=env, cwd=root, capture_output=True,
                       text=True, timeout=240)
    assert r.returncode == 0, r.stdout[-2000:] + r.stderr[-4000:]
    assert 'ok' in r.stdout


def test_async_compile_runs_precompiled_until_ready(monkeypatch):
    """LT_JIT_ASYNC: the module compiles on a worker thread (disk cache off, so it really
    compiles) while the first call's tiles run on the precompiled kernels; once lt_jit_prepare has
    waited for it, the same tiles run on the JIT kernels. Both calls write the oracle's results."""
    monkeypatch.setenv('LT_JIT_CACHE', '')
    eng = Engine(0)
    try:
        eqn = '(B1 - B2) * 5 / 5'
        fn = eng.compile_index(index_eqn.IndexProgram(eqn, band_dtype='int16'))
        meta, params, tiles = _tiles(eng, eqn, True, n_tiles=3, seed=1)
        eng.set_jit_mode(True)
        first = eng.analyze_tiles(meta, params, tiles, FIELDS, index=fn)
        torch.cuda.synchronize()
        s1 = eng.jit_stats()
        assert s1['fallback_tiles'] + s1['jit_tiles'] == 3, s1
        assert s1['fallback_tiles'] >= 1, s1  # a cold hiprtc compile takes seconds
        eng.jit_prepare(meta, params, tiles[0][0], tiles[0][1], FIELDS, fn, wait=True)
        second = eng.analyze_tiles(meta, params, tiles, FIELDS, index=fn)
        torch.cuda.synchronize()
        s2 = eng.jit_stats()
        assert s2['jit_tiles'] == s1['jit_tiles'] + 3 and s2['compiles'] == 1, s2
        for a, b in zip(first, second):
            for f in FIELDS:
                assert _bits_equal(a[f].cpu().numpy(), b[f].cpu().numpy()).all(), f
        _check_vs_oracle(eng, fn, meta, params, tiles, second)
    finally:
        eng.set_jit_mode(False)
        eng.close()


def test_module_cap_evicts_least_recently_used(monkeypatch):
    """LT_JIT_MAX_MODULES=1: alternating two programs unloads the other module each time (after
    its last launch), and a reloaded module writes what it wrote before."""
    monkeypatch.setenv('LT_JIT_MAX_MODULES', '1')
    eng = Engine(0)
    try:
        fa = eng.compile_index(index_eqn.IndexProgram('(B1 - B2) * 2 / 2', band_dtype='int16'))
        fb = eng.compile_index(index_eqn.IndexProgram('(B1 - B2) * 3 / 3', band_dtype='int16'))
        meta, params, tiles = _tiles(eng, 'lru', False, n_tiles=1, seed=2)
        a1 = eng.analyze_tiles(meta, params, tiles, FIELDS, index=fa)
        b1 = eng.analyze_tiles(meta, params, tiles, FIELDS, index=fb)
        a2 = eng.analyze_tiles(meta, params, tiles, FIELDS, index=fa)
        torch.cuda.synchronize()
        st = eng.jit_stats()
        assert st['evictions'] >= 2 and st['modules'] == 1 and st['jit_tiles'] == 3, st
        for f in FIELDS:  # the same values through both programs, and the module reloaded
            assert _bits_equal(a1[0][f].cpu().numpy(), a2[0][f].cpu().numpy()).all(), f
            assert _bits_equal(a1[0][f].cpu().numpy(), b1[0][f].cpu().numpy()).all(), f
        _check_vs_oracle(eng, fa, meta, params, tiles, a2)
    finally:
        eng.close()
