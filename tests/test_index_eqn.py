"""Load stage (index_eqn, utils.py:447-484) on the CPU: equation parsing with the reference's own
test cases, numpy 1.x dtype rules (known answers), the generated HIP source (valid, compiles for
gfx950), the numpy oracle on the reference's TIFF fixture, and the GeoTIFF reader."""
import ctypes
import os
import subprocess

import numpy as np
import pytest

from land_trendr_amd import _abi, index_eqn
from land_trendr_amd.geotiff import GeoTiff, read_bands
from oracle import index_oracle

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TIF = os.path.join(ROOT, 'tests', 'golden', 'files', 'dummy_single_band.tif')


# ---- the reference's own tests (tests/utils_test.py:44-63) ----
def test_parse_eqn_bands_reference_cases():
    assert index_eqn.parse_eqn_bands('') == []
    assert index_eqn.parse_eqn_bands('12 - 4') == []
    assert index_eqn.parse_eqn_bands('B1') == [1]
    assert set(index_eqn.parse_eqn_bands('(B2-B2)/(B3+B4)-B6')) == {2, 3, 4, 6}


def test_multiple_replace_reference_case():
    replacements = {'X': '3', 'Y': '2', 'Z': '1'}
    assert index_eqn.multiple_replace('(X + Y) / (X-Y) = Z', replacements) == '(3 + 2) / (3-2) = 1'


# ---- numpy 1.x legacy promotion (value-based casting), known answers ----
@pytest.mark.parametrize('a,b,want', [
    (np.dtype(np.int16), 1, np.int16), (np.dtype(np.int16), -1, np.int16),
    (np.dtype(np.int16), 40000, np.int32), (np.dtype(np.int16), 0.5, np.float64),
    (np.dtype(np.float32), 2, np.float32), (np.dtype(np.float32), 0.5, np.float32),
    (np.dtype(np.uint8), -1, np.int16), (np.dtype(np.uint8), 300, np.uint16),
    (np.dtype(np.int16), np.dtype(np.int16), np.int16),
    (np.dtype(np.int16), np.dtype(np.uint16), np.int32),
    (np.dtype(np.uint16), np.dtype(np.float32), np.float32),
    (np.dtype(np.int32), np.dtype(np.float32), np.float64),
    (np.dtype(np.int8), 1000, np.int16)])
def test_legacy_result_dtype(a, b, want):
    assert index_eqn.result_dtype(a, b) == np.dtype(want)
    assert index_eqn.result_dtype(b, a) == np.dtype(want)


def test_program_types_and_errors():
    p = index_eqn.IndexProgram('B1 - B2')
    assert p.result_dtype == np.int16 and p.bands == [1, 2]
    p = index_eqn.IndexProgram('(B4 - B3) * 0.5 + 2 / 4', out_dtype=np.int16)
    assert p.result_dtype == np.float64  # 2 / 4 folds to 0 (Py2 int division)
    assert index_eqn.IndexProgram('B2 + 40000').result_dtype == np.int32
    with pytest.raises(Exception, match='Band 7 not present'):
        index_eqn.IndexProgram('B7 - B1', raster_count=6)
    with pytest.raises(Exception, match='Invalid band'):
        index_eqn.IndexProgram('B0 + B1')
    for bad in ('np.where(B1 > 0, B1, 0)', 'B1 ** 2', '__import__("os")', 'B1 % 3', 'C1 + B1'):
        with pytest.raises(ValueError):
            index_eqn.IndexProgram(bad)


# ---- generated source ----
EQNS = ['B1 - B2', '(B4 - B3) / (B4 + B3)', 'B1 * 10000', 'B2 + 40000', '(B1 - B2) * 0.5',
        'B3 // 7 - -B1', '-B1 / 3 + 1000']


def _codegen(prog):
    lib = _abi.load_lib()
    p = prog.to_c()
    n = lib.lt_index_codegen(ctypes.byref(p), None, 0)
    assert n > 0
    buf = ctypes.create_string_buffer(n + 1)
    assert lib.lt_index_codegen(ctypes.byref(p), buf, n + 1) == n
    return buf.value.decode()


def test_codegen_compiles_for_gfx950(tmp_path):
    for k, eqn in enumerate(EQNS):
        src = _codegen(index_eqn.IndexProgram(eqn))
        assert 'lt_index_kernel' in src and eqn not in src
        f = tmp_path / ('idx%d.hip' % k)
        f.write_text('#include <hip/hip_runtime.h>\n' + src)  # hiprtc provides it implicitly
        subprocess.check_call(['/opt/rocm/bin/hipcc', '-x', 'hip', '--offload-arch=gfx950',
                               '--cuda-device-only', '-c', '-O3', '-ffp-contract=off', '-o',
                               str(tmp_path / ('idx%d.o' % k)), str(f)])


def test_codegen_rejects_malformed_programs():
    lib = _abi.load_lib()
    p = index_eqn.IndexProgram('B1 - B2').to_c()
    p.n_ops = 2  # stack left unbalanced
    assert lib.lt_index_codegen(ctypes.byref(p), None, 0) < 0
    p = index_eqn.IndexProgram('B1 - B2').to_c()
    p.ops[0].ival = 5  # band slot out of range
    assert lib.lt_index_codegen(ctypes.byref(p), None, 0) < 0


# ---- oracle and the reference's rast_algebra test on its own fixture (utils_test.py:119-125) ----
def test_oracle_int16_wrap_and_floor_division():
    b = np.array([[32767, -32768, 7, -7, 5, 0], [-1, 1, 2, 2, 0, 0]], np.int16)
    got = index_oracle.evaluate(index_eqn.IndexProgram('B1 - B2'), b)
    assert got.tolist() == [-32768, 32767, 5, -9, 5, 0]
    got = index_oracle.evaluate(index_eqn.IndexProgram('B1 / B2'), b)
    assert got.tolist() == [-32767, -32768, 3, -4, 0, 0]  # floor; x / 0 -> 0


def test_reference_rast_algebra_half_on_fixture():
    bands = read_bands(TIF)
    assert bands.shape == (1, 45, 54) and bands.dtype == np.float32
    prog = index_eqn.IndexProgram('B1/2', band_dtype=np.float32)
    assert prog.result_dtype == np.float32 and prog.out_dtype == np.float32
    alg = index_oracle.evaluate(prog, bands)
    assert np.sum(bands) / 2 == np.sum(alg)


def test_geotiff_reader_fixture_metadata():
    g = GeoTiff(TIF)
    assert (g.width, g.height, g.bands) == (54, 45, 1)
    assert g.pixel_scale[:2] == (30.0, 30.0)
    assert g.width * g.height == 2430  # utils_test.py:130 test_grid count


# ---- the fused load stage: lt_index_linearize (lt_index.h) ----------------------------------

def _lin_eval(lin, bands):
    """The linear form's value as the analyze kernel computes it (lt_pixel.h lin_value /
    lt_fast.h's fused batch): the sum modulo 2^64, the wrap to the node type, the store."""
    M = 1 << 64
    acc = np.full(bands.shape[1:], lin.c0 % M, dtype=object)
    for s in range(lin.n_bands):
        acc = (acc + (lin.coef[s] % M) * bands[s].astype(np.int64).astype(object)) % M
    w = np.dtype(index_eqn.CODES[lin.wrap_type])
    bits = w.itemsize * 8
    r = acc % (1 << bits)
    if w.kind == 'i':
        r = np.where(r >= 1 << (bits - 1), r - (1 << bits), r)
    out = np.dtype(index_eqn.CODES[lin.out_type])
    if out.kind == 'f':
        return np.array([out.type(int(v)) for v in r.ravel()], out).reshape(r.shape)
    info = np.iinfo(out)
    return np.clip(r, info.min, info.max).astype(out)


LINEAR = [('B1 - B2', 'int16', None), ('B1 + B2 * 3 - 7', 'int16', None),
          ('B1 * 300 - B2 * 300', 'int16', None), ('-(B1 - 2 * B3) + 30000', 'int16', None),
          ('(B2 - B1) * 2', 'uint16', None), ('B1 - B2', 'uint16', 'int16'),
          ('B1 + B2 - 100', 'uint8', None), ('3 * B1 - B2', 'int32', None),
          ('B1 - B2', 'int16', 'float32'), ('B1 + 70000 - B2', 'int16', 'int16'),
          ('B1', 'int16', None), ('B1 * -1', 'uint8', 'int16'), ('B1 + 2 - B2 + B3 - B4', 'int16', None)]
NONLINEAR = [('B1 * B2', 'int16'), ('B1 / 2', 'int16'), ('B1 // B2', 'int16'),
             ('B1 - B2 + 0.5', 'int16'), ('(B1 - B2) + 40000', 'int16'), ('B1 - B2', 'float32'),
             ('B1 + B2 + B3 + B4 + B5', 'int16'), ('B1 - B2', 'int8'),
             ('-(B1 - 2 * B3) + 40000', 'int16')]


@pytest.mark.parametrize('eqn,bt,ot', LINEAR)
def test_linear_form_matches_numpy_evaluation(eqn, bt, ot):
    """Every program lt_index_linearize accepts gives, through its form, exactly what the numpy
    restatement of rast_algebra + its store gives (wrapping and saturating values included)."""
    from land_trendr_amd.engine import linear_form
    prog = index_eqn.IndexProgram(eqn, band_dtype=bt, out_dtype=ot)
    lin = linear_form(prog)
    assert lin is not None, eqn
    rng = np.random.default_rng(7)
    info = np.iinfo(np.dtype(bt))
    b = rng.integers(info.min, int(info.max) + 1, size=(len(prog.bands), 4000)).astype(bt)
    b[:, :8] = info.min
    b[:, 8:16] = info.max
    want = index_oracle.evaluate(prog, b)
    got = _lin_eval(lin, b)
    assert got.dtype == want.dtype
    np.testing.assert_array_equal(got, want)


@pytest.mark.parametrize('eqn,bt', NONLINEAR)
def test_nonlinear_programs_keep_the_load_kernel(eqn, bt):
    from land_trendr_amd.engine import linear_form
    assert linear_form(index_eqn.IndexProgram(eqn, band_dtype=bt)) is None
