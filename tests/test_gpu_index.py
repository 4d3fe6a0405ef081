"""Load stage on the GPU: hiprtc-compiled index kernels against the numpy oracle (bit-exact), the
reference's rast_algebra test on its own TIFF fixture, and int16 bands -> index raster -> analyze
end to end against the CPU oracle."""
import os
import zlib

import numpy as np
import pytest
import torch

from land_trendr_amd import index_eqn
from land_trendr_amd.geotiff import read_bands
from land_trendr_amd.scene import build_scene, parse_date
from land_trendr_amd.settings import compile_params
from oracle import index_oracle, oracle

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.fixture(scope='module')
def engine():
    from land_trendr_amd.engine import get_engine
    return get_engine(0)


def _bits_equal(a, b):
    if a.dtype.kind == 'f':
        ai = a.view(np.int32 if a.itemsize == 4 else np.int64)
        bi = b.view(np.int32 if b.itemsize == 4 else np.int64)
        return (ai == bi) | (np.isnan(a) & np.isnan(b))
    return a == b


INT16_EQNS = ['B1 - B2', '(B4 - B3) / (B4 + B3)', 'B1 * 10000', 'B2 + 40000', '(B1 - B2) * 0.5',
              'B3 // 7 - -B1', '-B1 / 3 + 1000', '(B2 - B1) / (B2 + B1) * 1000.0', 'B1 + 0.5']


@pytest.mark.parametrize('eqn', INT16_EQNS)
def test_index_kernel_int16_vs_numpy(engine, eqn):
    prog = index_eqn.IndexProgram(eqn, band_dtype=np.int16)
    fn = engine.compile_index(prog)
    rng = np.random.default_rng(zlib.crc32(eqn.encode()))
    K, NB, P = 3, len(prog.bands), 20000
    b = rng.integers(-32768, 32768, (K, NB, P)).astype(np.int16)
    b[:, :, :8] = np.array([0, -1, 1, 32767, -32768, 2, -2, 7], np.int16)  # edge values
    b[0, :, 8:16] = 0  # x / 0 and 0 / 0
    got = engine.index_tile(fn, torch.from_numpy(b).to(engine.device))
    torch.cuda.synchronize()
    got = got.cpu().numpy()
    for k in range(K):
        want = index_oracle.evaluate(prog, b[k])
        same = _bits_equal(want, got[k])
        assert same.all(), '%s obs %d: %d of %d differ' % (eqn, k, (~same).sum(), P)


@pytest.mark.parametrize('eqn', ['B1 - B2', '(B4 - B3) / (B4 + B3)', 'B1 * 10000',
                                 'B1 + B2 - B3 // 3'])
@pytest.mark.parametrize('P', [20000, 20003, 3])
def test_index_kernel_pixel_interleaved_bands(engine, eqn, P):
    """Pixel-interleaved bands (band stride 1, pixel stride NB: the layout the fused load stage
    reads) go through lt_index_kernel4i on the 4-aligned head and the scalar kernel on the tail,
    bit-exact against the numpy oracle; a tile view (pixel offset) and a ragged P included."""
    prog = index_eqn.IndexProgram(eqn, band_dtype=np.int16)
    fn = engine.compile_index(prog)
    rng = np.random.default_rng(zlib.crc32(eqn.encode()) + P)
    K, NB = 3, len(prog.bands)
    b = rng.integers(-32768, 32768, (K, NB, P)).astype(np.int16)
    b[:, :, :min(P, 8)] = np.array([0, -1, 1, 32767, -32768, 2, -2, 7], np.int16)[:min(P, 8)]
    inter = torch.from_numpy(np.ascontiguousarray(b.transpose(0, 2, 1))).to(engine.device)
    view = inter.permute(0, 2, 1)  # [K, NB, P] with strides (NB*P, 1, NB)
    assert NB == 1 or (view.stride(1) == 1 and view.stride(2) == NB)
    got = engine.index_tile(fn, view).cpu().numpy()
    for k in range(K):
        same = _bits_equal(index_oracle.evaluate(prog, b[k]), got[k])
        assert same.all(), '%s obs %d: %d of %d differ' % (eqn, k, (~same).sum(), P)
    if P > 8:  # a tile view starting at pixel 4 (the head stays 4-aligned) and at pixel 1
        for a in (4, 1):
            got = engine.index_tile(fn, view[:, :, a:]).cpu().numpy()
            for k in range(K):
                same = _bits_equal(index_oracle.evaluate(prog, b[k, :, a:]), got[k])
                assert same.all(), '%s offset %d obs %d: %d differ' % (eqn, a, k, (~same).sum())


def test_index_kernel_float32_and_uint16(engine):
    rng = np.random.default_rng(3)
    for eqn, bt, ot in [('B1/2', np.float32, np.float32), ('(B1 - B2) / (B1 + B2)', np.float32,
                                                            np.float32),
                        ('B1 - B2', np.uint16, np.uint16), ('B2 - B1 * 3', np.uint16, np.int16),
                        ('B1 // B2', np.float32, np.float32)]:
        prog = index_eqn.IndexProgram(eqn, band_dtype=bt, out_dtype=ot)
        fn = engine.compile_index(prog)
        if np.dtype(bt).kind == 'f':
            b = (rng.normal(0, 1000, (2, len(prog.bands), 5000))).astype(bt)
        else:
            b = rng.integers(0, 65536, (2, len(prog.bands), 5000)).astype(bt)
        got = engine.index_tile(fn, torch.from_numpy(b).to(engine.device)).cpu().numpy()
        for k in range(2):
            same = _bits_equal(index_oracle.evaluate(prog, b[k]), got[k])
            assert same.all(), '%s: %d differ' % (eqn, (~same).sum())


def test_reference_rast_algebra_half_on_fixture_gpu(engine):
    """utils_test.py:119-125: rast_algebra(template, 'B1/2') sums to half the template."""
    bands = read_bands(os.path.join(ROOT, 'tests', 'golden', 'files', 'dummy_single_band.tif'))
    prog = index_eqn.IndexProgram('B1/2', band_dtype=np.float32)
    fn = engine.compile_index(prog)
    b = torch.from_numpy(bands.reshape(1, 1, -1).copy()).to(engine.device)
    alg = engine.index_tile(fn, b).cpu().numpy().reshape(bands.shape[1:])
    assert np.sum(bands) / 2 == np.sum(alg)
    assert _bits_equal(index_oracle.evaluate(prog, bands), alg).all()


def test_bands_to_index_to_analyze_vs_oracle(engine):
    """int16 bands (B1 = B2 + index) -> 'B1 - B2' on the GPU -> int16 index raster -> analyze,
    bit-exact against the CPU oracle on float(index)."""
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    sc = make_scene(6000, seed=21, n_years=30, k_min=1, k_max=3, mask_prob=0.15,
                    with_bands=True)
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    params, _ = compile_params(10.0, [{'name': 'gd', 'val': 1, 'change_type': 'GD'}])
    prog = index_eqn.IndexProgram('B1 - B2', band_dtype=np.int16)
    fn = engine.compile_index(prog)
    dev = engine.device
    index = engine.index_tile(fn, sc.bands.to(dev))
    assert index.dtype == torch.int16
    valid = sc.valid.to(dev)
    out = engine.analyze_tile(meta, params, index, valid)
    torch.cuda.synchronize()
    got = {k: t.cpu().numpy() for k, t in out.items()}
    vals = index.cpu().numpy().astype(np.float64)
    assert (vals == sc.values.numpy()).all()
    want = oracle.analyze_tile(meta, params, vals, sc.valid.numpy(),
                               n_threads=os.cpu_count() or 1)
    for f in want:
        same = _bits_equal(want[f], got[f])
        assert same.all(), '%s: %d differ' % (f, (~same).sum())


def test_analysis_reducer_batch_from_bands(engine):
    """The batched reducer fed raw band planes (index_eqn on the GPU) equals the one fed the
    index values; extra unused planes are skipped by band number."""
    from land_trendr_amd.synth import make_scene
    from land_trendr_amd.utils import analysis_reducer_batch
    sc = make_scene(3000, seed=5, n_years=25, with_bands=True)
    dev = engine.device
    settings = {'line_cost': 10, 'target_date': '2014-07-01', 'index_eqn': 'B4 - B2',
                'label_rules': [{'name': 'gd', 'val': 1, 'change_type': 'GD'}]}
    K, _, P = sc.bands.shape
    junk = torch.zeros((K, 1, P), dtype=torch.int16)
    planes = torch.cat([junk, sc.bands[:, 1:2], junk, sc.bands[:, 0:1]], dim=1).to(dev)
    a = analysis_reducer_batch(sc.dates, None, None, settings, bands=planes,
                               band_numbers=[1, 2, 3, 4])
    b = analysis_reducer_batch(sc.dates, sc.values.to(dev), None, settings)
    for f in ('status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude'):
        assert torch.equal(a[f], b[f]), f

def test_load_stage_on_own_stream_with_ready_events(engine):
    """Tile t's index raster written on a load stream, its analyze kernel waiting on tile t's
    event alone (lt_analyze_tiles_after): bit-exact against the oracle on float(index), and
    equal to the serial bands -> index -> lt_analyze_tiles order."""
    from land_trendr_amd.synth import make_scene
    from oracle import oracle
    sc = make_scene(24000, seed=33, n_years=30, k_min=1, k_max=2, mask_prob=0.1,
                    with_bands=True)
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    params, _ = compile_params(10.0, [{'name': 'gd', 'val': 1, 'change_type': 'GD'}])
    fn = engine.compile_index(index_eqn.IndexProgram('B1 - B2', band_dtype=np.int16))
    dev = engine.device
    bands, valid = sc.bands.to(dev), sc.valid.to(dev)
    K, _, P = bands.shape
    cuts = [0, 5000, 11000, 11001, 24000]  # uneven tiles, one of a single pixel
    spans = list(zip(cuts[:-1], cuts[1:]))
    main = torch.cuda.current_stream(dev)
    load = torch.cuda.Stream(dev)
    load.wait_stream(main)
    index = torch.empty((K, P), dtype=torch.int16, device=dev)
    ready = []
    with torch.cuda.stream(load):
        for a, b in spans:
            engine.index_tile(fn, bands[:, :, a:b], out=index[:, a:b])
            ev = torch.cuda.Event()
            ev.record()
            ready.append(ev)
    tiles = [(index[:, a:b], valid[:, a:b]) for a, b in spans]
    over = engine.analyze_tiles(meta, params, tiles, ready=ready)
    torch.cuda.synchronize()
    serial_index = engine.index_tile(fn, bands)
    serial = engine.analyze_tiles(meta, params, [(serial_index[:, a:b], valid[:, a:b])
                                                 for a, b in spans])
    torch.cuda.synchronize()
    assert torch.equal(index, serial_index)
    vals = serial_index.cpu().numpy().astype(np.float64)
    want = oracle.analyze_tile(meta, params, vals, sc.valid.numpy(),
                               n_threads=os.cpu_count() or 1)
    for (a, b), o, s in zip(spans, over, serial):
        for f in o:
            x, y = o[f].cpu().numpy(), s[f].cpu().numpy()
            assert x.tobytes() == y.tobytes(), (a, b, f)
            if f in ('class_val', 'onset_year', 'duration', 'magnitude', 'initial_val'):
                continue  # unmatched slots hold no defined value
            same = _bits_equal(want[f][..., a:b], x)
            assert same.all(), (a, b, f, int((~same).sum()))


FUSED = [('B1 - B2', np.int16, None), ('B1 * 300 - B2 * 300', np.int16, None),
         ('-(B1 - 2 * B3) + 30000', np.int16, None), ('B1 - B2', np.uint16, np.int16),
         ('(B2 - B1) * 2', np.uint16, None), ('B1 + B2 - 100', np.uint8, None),
         ('3 * B1 - B2', np.int32, None), ('B1 - B2', np.int16, np.float32),
         ('B1 + 70000 - B2', np.int16, np.int16), ('B1 + 2 - B2 + B3 - B4', np.int16, None),
         ('B1 - B2', np.int16, np.float64)]


@pytest.mark.parametrize('eqn,bt,ot', FUSED)
@pytest.mark.parametrize('masked', [False, True])
def test_fused_load_stage_matches_index_raster_path(engine, eqn, bt, ot, masked):
    """The analyze kernel evaluating a linear index_eqn on the winners' band values (lt_tile_in
    obs_bands + lt_index_lin) writes exactly what it writes from the load kernel's index raster
    of the same bands, in every output plane (wrapping and saturating values included)."""
    from land_trendr_amd.engine import ALL_FIELDS
    prog = index_eqn.IndexProgram(eqn, band_dtype=bt, out_dtype=ot)
    fn = engine.compile_index(prog)
    assert fn.lin is not None
    rng = np.random.default_rng(zlib.crc32((eqn + str(bt) + str(masked)).encode()))
    Y, P = 30, 6000
    k_per = rng.integers(1, 4, Y) if masked else np.ones(Y, int)
    dates = []
    for y in range(Y):
        for _ in range(k_per[y]):
            dates.append('%d-%02d-%02d' % (1990 + y, rng.integers(5, 10), rng.integers(1, 28)))
    K = len(dates)
    meta = build_scene(dates, parse_date('2014-07-01'))
    info = np.iinfo(np.dtype(bt))
    lo, hi = max(int(info.min), -3000), min(int(info.max), 3000)
    base = rng.integers(lo, hi + 1, (1, len(prog.bands), P))
    b = np.clip(base + rng.integers(-400, 401, (K, len(prog.bands), P)), info.min, info.max)
    b[:, :, :16] = rng.integers(info.min, int(info.max) + 1, (K, len(prog.bands), 16))  # extremes
    bands = torch.from_numpy(b.astype(bt)).to(engine.device)
    valid = None
    if masked:
        valid = torch.from_numpy((rng.random((K, P)) > 0.2).astype(np.uint8)).to(engine.device)
    params, _ = compile_params(1.0, [{'name': 'gd', 'val': 1, 'change_type': 'GD'},
                                     {'name': 'fd', 'val': 2, 'change_type': 'FD'}])
    idx = engine.index_tile(fn, bands)
    want = engine.analyze_tile(meta, params, idx, valid, ALL_FIELDS)
    got = engine.analyze_tile(meta, params, bands, valid, ALL_FIELDS, lin=fn.lin)
    torch.cuda.synchronize()
    for f in ALL_FIELDS:
        w, g = want[f].cpu().numpy(), got[f].cpu().numpy()
        same = _bits_equal(w, g)
        assert same.all(), '%s %s: %s differs in %d places' % (eqn, bt, f, (~same).sum())


def test_fused_load_stage_one_pixel_planar_band_slice(engine):
    """A planar one-pixel tile whose two int16 bands are a slice of a 3-band stack ([K, 3, 1]
    viewed as bands 1:3: band stride 1, pixel stride 1, data 2 bytes off a 4-byte boundary, obs
    stride 3) is not a pixel-interleaved pair: the fused kernel reads it band by band and writes
    what the index-raster path writes (it used to take the 32-bit pair load)."""
    from land_trendr_amd.engine import ALL_FIELDS
    from land_trendr_amd.synth import make_scene
    sc = make_scene(1, seed=5, n_years=30, with_bands=True)
    K = sc.bands.shape[0]
    stack = torch.zeros((K, 3, 1), dtype=torch.int16)
    stack[:, 1:3] = sc.bands
    b = stack.to(engine.device)[:, 1:3]
    assert b.stride() == (3, 1, 1) and b.data_ptr() % 4 == 2
    meta = build_scene(sc.dates, parse_date('2014-07-01'))
    params, _ = compile_params(10.0, [{'name': 'gd', 'val': 1, 'change_type': 'GD'}])
    fn = engine.compile_index(index_eqn.IndexProgram('B1 - B2', band_dtype=np.int16))
    want = engine.analyze_tile(meta, params, engine.index_tile(fn, b), None, ALL_FIELDS)
    got = engine.analyze_tile(meta, params, b, None, ALL_FIELDS, lin=fn.lin)
    torch.cuda.synchronize()
    assert int(want['n_years'][0]) == 30
    for f in ALL_FIELDS:
        assert _bits_equal(want[f].cpu().numpy(), got[f].cpu().numpy()).all(), f


JIT = [('(B1 - B2) * 1000 / (B1 + B2)', np.int16, None),   # NDVI-like: int16 floor division
       ('(B1 - B2) * 2 / 2', np.int16, None),              # bench.py's attribution program
       ('B1 / 2.0 - B2', np.int16, None),                  # a float64 node, stored into int16
       ('B1 * B2 / 100', np.int16, np.float64),            # a product of bands, stored binary64
       ('(B2 - B1) // 7 + B3', np.uint16, None)]           # unsigned floor division


@pytest.mark.parametrize('eqn,bt,ot', JIT)
@pytest.mark.parametrize('masked', [False, True])
def test_jit_fused_load_stage_matches_index_raster_path(engine, eqn, bt, ot, masked):
    """Programs that are not linear forms (divisions, float nodes, products of bands): the JIT
    analyze / resolve kernels with the program inlined (lt_jit.h, lt_tile_in.index) write exactly
    what the precompiled kernels write from the load kernel's index raster of the same bands, in
    every output plane (x / 0 = 0 and wrapping values included)."""
    from land_trendr_amd.engine import ALL_FIELDS
    prog = index_eqn.IndexProgram(eqn, band_dtype=bt, out_dtype=ot)
    fn = engine.compile_index(prog)
    assert fn.lin is None
    rng = np.random.default_rng(zlib.crc32((eqn + str(bt) + str(masked) + 'jit').encode()))
    Y, P = 30, 6000
    k_per = rng.integers(1, 4, Y) if masked else np.ones(Y, int)
    dates = []
    for y in range(Y):
        for _ in range(k_per[y]):
            dates.append('%d-%02d-%02d' % (1990 + y, rng.integers(5, 10), rng.integers(1, 28)))
    K = len(dates)
    meta = build_scene(dates, parse_date('2014-07-01'))
    info = np.iinfo(np.dtype(bt))
    lo, hi = max(int(info.min), -3000), min(int(info.max), 3000)
    base = rng.integers(lo, hi + 1, (1, len(prog.bands), P))
    b = np.clip(base + rng.integers(-400, 401, (K, len(prog.bands), P)), info.min, info.max)
    b[:, :, :16] = rng.integers(info.min, int(info.max) + 1, (K, len(prog.bands), 16))  # extremes
    b[:, :, 16:32] = 0  # zero denominators
    bands = torch.from_numpy(b.astype(bt)).to(engine.device)
    valid = None
    if masked:
        valid = torch.from_numpy((rng.random((K, P)) > 0.2).astype(np.uint8)).to(engine.device)
    params, _ = compile_params(1.0, [{'name': 'gd', 'val': 1, 'change_type': 'GD'},
                                     {'name': 'fd', 'val': 2, 'change_type': 'FD'}])
    idx = engine.index_tile(fn, bands)
    want = engine.analyze_tile(meta, params, idx, valid, ALL_FIELDS)
    got = engine.analyze_tile(meta, params, bands, valid, ALL_FIELDS, index=fn)
    torch.cuda.synchronize()
    for f in ALL_FIELDS:
        w, g = want[f].cpu().numpy(), got[f].cpu().numpy()
        same = _bits_equal(w, g)
        assert same.all(), '%s %s: %s differs in %d places' % (eqn, bt, f, (~same).sum())
    # and against the CPU checkers alone (VERDICT r04 weak #1 gap 2): the program evaluated by
    # numpy (oracle/index_oracle.py), analysed by the C oracle, on the first 1500 pixels
    n = 1500
    vals = index_oracle.evaluate(prog, np.moveaxis(b[:, :, :n], 1, 0)).astype(np.float64)
    vb = valid[:, :n].cpu().numpy() if valid is not None else None
    want_o = oracle.analyze_tile(meta, params, np.ascontiguousarray(vals), vb,
                                 n_threads=os.cpu_count() or 1)
    for f in want_o:
        g = got[f].cpu().numpy()[..., :n]
        w = want_o[f][:g.shape[0]] if g.ndim == 2 else want_o[f]
        if f in ('class_val', 'onset_year', 'duration', 'magnitude', 'initial_val'):
            mt = want_o['matched'].astype(bool)[:g.shape[0]]
            g, w = np.where(mt, g, 0), np.where(mt, w, 0)
        same = _bits_equal(w, g)
        assert same.all(), '%s %s: %s differs from the oracle in %d places' % (
            eqn, bt, f, (~same).sum())


def test_jit_fused_runner_matches_oracle(engine):
    """The mosaic runner with a non-linear program takes the JIT-fused path (runner.jit) and its
    labels equal the oracle's on the index raster of the same bands."""
    from land_trendr_amd.distributed import Mosaic
    from land_trendr_amd.engine import valid_bytes
    from land_trendr_amd.runner import MosaicRunner
    from land_trendr_amd.synth import mosaic_inputs
    from oracle import oracle
    m = Mosaic([20000], 8192, 1, 0, 'by_scene')
    items = mosaic_inputs(m, 30, 1, 3, 0.2, 91, engine.device, '2014-07-01')
    params, _ = compile_params(10.0, [{'name': 'gd', 'val': 1, 'change_type': 'GD'}])
    fn = engine.compile_index(index_eqn.IndexProgram('(B1 - B2) * 3 / 3', band_dtype=np.int16))
    fields = ['status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude', 'val_fit',
              'vertex']
    r = MosaicRunner(engine, m, params, items, fields, fn)
    assert r.fused and r.jit is fn and r.lin is None
    r.step()
    torch.cuda.synchronize()
    for k, it in enumerate(r.items):
        r.materialise_index(k)
        vals = it.values.double().cpu().numpy()
        want = oracle.analyze_tile(it.scene, params, vals,
                                   valid_bytes(it.valid, it.scene.n_obs).cpu().numpy(),
                                   n_threads=os.cpu_count() or 1)
        for f in fields:
            g = r.outs[k][f][..., :it.tile.n].cpu().numpy()
            w = want[f][:g.shape[0]] if g.ndim == 2 else want[f]
            if f in ('class_val', 'onset_year', 'duration', 'magnitude'):
                mt = want['matched'].astype(bool)[:g.shape[0]]
                g, w = np.where(mt, g, 0), np.where(mt, w, 0)
            assert _bits_equal(w, g).all(), (k, f)
