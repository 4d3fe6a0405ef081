"""Compressed GeoTIFF IO: the native LZW codec (liblt_io.so, include/lt_io.h)
and the reader / writer around it, checked against libtiff — the library GDAL itself uses for TIFF
compression — through Pillow's libtiff plugin when it is importable (CPU-only tests)."""
import io
import os

import numpy as np
import pytest

from land_trendr_amd import raster, tiffcodec
from land_trendr_amd.geotiff import GeoTiff

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
TIF = os.path.join(ROOT, 'tests', 'golden', 'files', 'dummy_single_band.tif')

try:
    from PIL import Image, features
    HAVE_LIBTIFF = features.check('libtiff')
except ImportError:  # pragma: no cover
    HAVE_LIBTIFF = False
needs_libtiff = pytest.mark.skipif(not HAVE_LIBTIFF, reason='Pillow with libtiff not importable')


@pytest.mark.parametrize('kind', ['empty', 'one', 'zeros', 'ramp', 'random', 'lowentropy', 'big'])
def test_lzw_round_trip(kind):
    rng = np.random.default_rng(len(kind))
    data = {'empty': b'', 'one': b'\x07', 'zeros': bytes(100000),
            'ramp': bytes(range(256)) * 300,
            'random': rng.integers(0, 256, 70000, dtype=np.uint8).tobytes(),
            'lowentropy': rng.integers(0, 3, 300000, dtype=np.uint8).tobytes(),
            'big': (np.arange(2_000_000) % 251).astype(np.uint8).tobytes()}[kind]
    enc = tiffcodec.lzw_encode(data)
    assert tiffcodec.lzw_decode(enc, len(data)).tobytes() == data
    if kind in ('zeros', 'lowentropy'):
        assert len(enc) < len(data) // 4


def test_lzw_decodes_the_tiff_spec_stream_shape():
    """A hand-built code stream: Clear, 'A' 'B', the new code 258 ('AB'), EOI (9-bit codes, MSB
    first), decodes to 'ABAB'."""
    codes = [256, 65, 66, 258, 257]
    bits = ''.join(format(c, '09b') for c in codes)
    bits += '0' * (-len(bits) % 8)
    stream = bytes(int(bits[i:i + 8], 2) for i in range(0, len(bits), 8))
    assert tiffcodec.lzw_decode(stream, 4).tobytes() == b'ABAB'


def _pil_write(path, a, compression):
    Image.fromarray(a).save(path, compression=compression)


def _pil_read(path):
    return np.array(Image.open(path))


@needs_libtiff
@pytest.mark.parametrize('dtype', [np.uint8, np.uint16, np.float32, np.int32])
@pytest.mark.parametrize('compression', ['tiff_lzw', 'tiff_adobe_deflate', 'packbits'])
def test_reader_decodes_libtiff_output(tmp_path, dtype, compression):
    rng = np.random.default_rng(7)
    a = (rng.normal(300, 90, (123, 457))).astype(dtype) if dtype != np.float32 else \
        rng.normal(0, 1, (123, 457)).astype(np.float32)
    a[:, :40] = a[0, 0]  # some runs
    p = str(tmp_path / 'x.tif')
    _pil_write(p, a, compression)
    g = GeoTiff(p)
    assert g.compression in (5, 8, 32946, 32773)
    got = g.read()[0]
    assert got.dtype == a.dtype and np.array_equal(got, a)


@needs_libtiff
@pytest.mark.parametrize('dtype', [np.uint8, np.uint16, np.float32, np.int32])
@pytest.mark.parametrize('compress,predictor', [('lzw', 1), ('deflate', 1), ('lzw', 2)])
def test_writer_output_decodes_in_libtiff(tmp_path, dtype, compress, predictor):
    if predictor == 2 and dtype == np.float32:
        pytest.skip('horizontal predictor is for integer samples')
    rng = np.random.default_rng(11)
    a = rng.integers(0, 200, (301, 77)).astype(dtype)
    a[100:150] = 5
    p = str(tmp_path / 'y.tif')
    raster.write_geotiff(p, a, template=TIF, compress=compress, predictor=predictor)
    assert np.array_equal(_pil_read(p), a)
    g = GeoTiff(p)
    assert np.array_equal(g.read()[0], a) and g.compression == (5 if compress == 'lzw' else 8)


def test_writer_round_trip_all_types_and_bands(tmp_path):
    tmpl = GeoTiff(TIF)
    for dt in (np.uint8, np.int8, np.int16, np.uint16, np.int32, np.float32, np.float64):
        a = (np.arange(3 * 45 * 54).reshape(3, 45, 54) % 117 - 40).astype(dt)
        for compress in ('lzw', 'deflate', None):
            f = str(tmp_path / ('o_%s_%s.tif' % (np.dtype(dt).name, compress)))
            raster.write_geotiff(f, a, template=tmpl, compress=compress)
            g = GeoTiff(f)
            assert np.array_equal(g.read(), a) and g.read().dtype == dt
            assert g.pixel_scale == tmpl.pixel_scale and g.geokeys == tmpl.geokeys


def test_lzw_scene_sized_raster_is_fast_enough(tmp_path):
    """A 7000 x 7000 GDT_Byte label raster (what output_reducer writes per key) in seconds."""
    import time
    rng = np.random.default_rng(3)
    a = np.where(rng.random((7000, 7000)) < 0.3, rng.integers(0, 255, (7000, 7000)), 0).astype(
        np.uint8)
    p = str(tmp_path / 'big.tif')
    t0 = time.perf_counter()
    raster.write_geotiff(p, a, compress='lzw')
    t1 = time.perf_counter()
    got = GeoTiff(p).read()[0]
    t2 = time.perf_counter()
    assert np.array_equal(got, a)
    assert t1 - t0 < 30 and t2 - t1 < 30, (t1 - t0, t2 - t1)


def _fp_predict(row_bytes, item, spp):
    """libtiff's fpDiff (PREDICTOR_FLOATINGPOINT encode) of one row of little-endian samples:
    bytes regrouped into planes, most significant first, then differenced with a stride of one
    pixel (spp bytes)."""
    b = np.frombuffer(row_bytes, np.uint8)
    wc = len(b) // item
    planes = b.reshape(wc, item)[:, ::-1].T.reshape(-1)  # MSB plane first
    d = planes.astype(np.int16)
    d[spp:] = d[spp:] - planes[:-spp].astype(np.int16)
    return (d & 0xff).astype(np.uint8)


@pytest.mark.parametrize('spp', [1, 3])
@pytest.mark.parametrize('dtype', [np.float32, np.float64])
def test_floating_point_predictor_undo_with_chunky_bands(spp, dtype):
    """Predictor 3 on a chunky raster of spp samples per pixel (PlanarConfiguration 1): libtiff
    accumulates the byte planes with a stride of spp, not 1."""
    rng = np.random.default_rng(spp)
    rows, width = 5, 17
    a = rng.normal(0, 1000, (rows, width * spp)).astype(dtype)
    item = np.dtype(dtype).itemsize
    enc = np.stack([_fp_predict(a[r].astype('<' + np.dtype(dtype).str[1:]).tobytes(), item, spp)
                    for r in range(rows)])
    block = np.frombuffer(enc.tobytes(), '<' + np.dtype(dtype).str[1:]).reshape(rows, width * spp)
    got = tiffcodec.undo_predictor(block.copy(), 3, np.dtype('<' + np.dtype(dtype).str[1:]),
                                   width, spp)
    assert np.array_equal(got.astype(dtype), a)


def _strip_tiff(path, a, bo='<', planar=2, predictor=1, compression=5, rps=3):
    """A strip TIFF written by hand (any byte order, chunky or planar, predictor 2), the reader's
    reference being its own per-strip path."""
    import struct
    from land_trendr_amd import tiffcodec
    nb, rows, cols = a.shape
    a = a.astype(a.dtype.newbyteorder(bo))
    strips = []
    if planar == 2:
        blocks = [a[b, y:y + rps] for b in range(nb) for y in range(0, rows, rps)]
        spp = 1
    else:
        blocks = [a[:, y:y + rps].transpose(1, 2, 0) for y in range(0, rows, rps)]
        spp = nb
    for blk in blocks:
        blk = np.ascontiguousarray(blk).reshape(blk.shape[0], -1)
        if predictor == 2:
            nat = blk.astype(blk.dtype.newbyteorder('='))
            d = nat.reshape(blk.shape[0], cols, spp).copy()
            d[:, 1:] = d[:, 1:] - d[:, :-1]
            blk = d.reshape(blk.shape).astype(blk.dtype)
        strips.append(tiffcodec.encode(compression, np.ascontiguousarray(blk).tobytes()))
    tags = [(256, 4, [cols]), (257, 4, [rows]), (258, 3, [a.dtype.itemsize * 8] * nb),
            (259, 3, [compression]), (262, 3, [1]), (273, 4, None), (277, 3, [nb]),
            (278, 4, [rps]), (279, 4, [len(s) for s in strips]), (284, 3, [planar]),
            (317, 3, [predictor]), (339, 3, [2 if a.dtype.kind == 'i' else 1] * nb)]
    fmt = {3: 'H', 4: 'I'}
    n = len(tags)
    extra_off = 8 + 2 + 12 * n + 4
    payloads = {}
    extra = b''
    data_off = extra_off + 4096
    offs, o = [], data_off
    for st in strips:
        offs.append(o)
        o += len(st)
    ifd = struct.pack(bo + 'H', n)
    for tag, typ, vals in tags:
        if vals is None:
            vals = offs
        payload = struct.pack(bo + fmt[typ] * len(vals), *vals)
        if len(payload) <= 4:
            ifd += struct.pack(bo + 'HHI', tag, typ, len(vals)) + payload.ljust(4, b'\x00')
        else:
            ifd += struct.pack(bo + 'HHII', tag, typ, len(vals), extra_off + len(extra))
            extra += payload
    ifd += struct.pack(bo + 'I', 0)
    assert len(extra) <= 4096
    with open(path, 'wb') as f:
        f.write((b'II' if bo == '<' else b'MM') + struct.pack(bo + 'HI', 42, 8))
        f.write(ifd)
        f.write(extra.ljust(4096, b'\x00'))
        for st in strips:
            f.write(st)


@pytest.mark.parametrize('dtype,bo,planar,predictor,compression', [
    (np.int16, '<', 2, 1, 5), (np.int16, '>', 2, 2, 5), (np.uint16, '<', 1, 2, 5),
    (np.int32, '>', 1, 1, 1), (np.uint8, '<', 2, 2, 5), (np.int16, '<', 1, 1, 1)])
def test_native_strip_decode_matches_per_strip_path(tmp_path, dtype, bo, planar, predictor,
                                                   compression):
    """liblt_io.so lt_tiff_decode_strips (threads, byte swap, predictor 2, chunky de-interleave,
    a short last strip) reads what the per-strip path reads."""
    from land_trendr_amd.geotiff import GeoTiff
    rng = np.random.default_rng(3)
    a = rng.integers(-3000 if np.dtype(dtype).kind == 'i' else 0, 3000, (3, 11, 7)).astype(dtype)
    p = str(tmp_path / 'x.tif')
    _strip_tiff(p, a, bo, planar, predictor, compression, rps=4)
    g = GeoTiff(p)
    want = g.read(native=False)
    assert np.array_equal(want, a)
    for threads in (1, 3):
        got = g.read(threads=threads)
        assert got.dtype == want.dtype and np.array_equal(got, want)
    # decoded in place into a caller's array (ingest_stack's raster-order path), and refused
    # for a wrongly shaped one
    buf = np.full(want.shape, 77, want.dtype)
    assert g.read(threads=2, out=buf) is buf and np.array_equal(buf, want)
    with pytest.raises(ValueError):
        tiffcodec.decode_strips(g._d, g.tags[273], g.tags[279], g.compression, g.predictor,
                                g.dtype, g._bo == '>', 7, 11, 3, g.planar, 4, 1,
                                out=np.empty((3, 7, 11), want.dtype))


def test_native_strip_encode_matches_per_strip_encoder(tmp_path):
    """write_geotiff's threaded strips (lt_tiff_encode_strips) are byte for byte the per-strip
    encoder's, and read back."""
    from land_trendr_amd import tiffcodec
    from land_trendr_amd.geotiff import GeoTiff
    from land_trendr_amd.raster import write_geotiff
    rng = np.random.default_rng(4)
    a = rng.integers(-500, 500, (2, 37, 29)).astype(np.int16)
    for predictor in (1, 2):
        data, sizes = tiffcodec.encode_strips(a, 5, 5, predictor, 3)
        ref = []
        for b in range(2):
            for y in range(0, 37, 5):
                blk = a[b, y:y + 5]
                if predictor == 2:
                    blk = tiffcodec.apply_predictor2(blk, 29, 1)
                ref.append(tiffcodec.encode(5, np.ascontiguousarray(blk).tobytes()))
        assert list(sizes) == [len(r) for r in ref]
        assert data.tobytes() == b''.join(ref)
        p = str(tmp_path / ('p%d.tif' % predictor))
        write_geotiff(p, a, predictor=predictor, rows_per_strip=5)
        assert np.array_equal(GeoTiff(p).read(), a)
