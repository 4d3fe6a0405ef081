"""TIFF strip / tile codecs for the GeoTIFF reader and writer (what GDAL does for the reference:
ds2array decodes any compression, utils.py:272-282; array2raster writes COMPRESS=LZW, :386).

  * LZW (Compression 5): native, land_trendr_amd/liblt_io.so (include/lt_io.h);
  * Deflate (Compression 8 and the old 32946): zlib;
  * PackBits (Compression 32773): restated here (run-length, byte oriented);
  * Predictor 2 (horizontal differencing, integer samples) undone / applied per row;
    Predictor 3 (floating point) is decoded too (byte planes, then differencing).
"""
import ctypes
import os
import zlib

import numpy as np

_LIB = None
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'liblt_io.so')


def _lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError('%s not built: run __graft_entry__.build()' % LIB_PATH)
        L = ctypes.CDLL(LIB_PATH)
        for f in (L.lt_lzw_decode, L.lt_lzw_encode):
            f.argtypes = [ctypes.c_char_p, ctypes.c_int64, ctypes.c_void_p, ctypes.c_int64]
            f.restype = ctypes.c_int64
        i64, vp, ci = ctypes.c_int64, ctypes.c_void_p, ctypes.c_int
        L.lt_tiff_decode_strips.argtypes = [vp, i64, vp, vp, i64, ci, ci, ci, ci, i64, i64, ci, ci,
                                            i64, vp, ci]
        L.lt_tiff_decode_strips.restype = i64
        L.lt_tiff_encode_strips.argtypes = [vp, ci, i64, i64, ci, i64, ci, ci, vp, i64, vp, ci]
        L.lt_tiff_encode_strips.restype = i64
        _LIB = L
    return _LIB


def lzw_decode(data, size):
    """One LZW strip -> `size` raw bytes (a short strip is zero-padded, as libtiff does)."""
    out = np.zeros(size, np.uint8)
    n = _lib().lt_lzw_decode(bytes(data), len(data), out.ctypes.data, size)
    if n < 0:
        raise ValueError('LZW: corrupt strip (%d)' % n)
    out[n:] = 0  # (the decoder may leave scratch bytes past the end of a short strip)
    return out


def lzw_encode(raw):
    raw = bytes(raw)
    cap = len(raw) * 3 // 2 + 16
    out = np.empty(cap, np.uint8)
    n = _lib().lt_lzw_encode(raw, len(raw), out.ctypes.data, cap)
    if n < 0:
        raise ValueError('LZW: encode failed (%d)' % n)
    return out[:n].tobytes()


def packbits_decode(data, size):
    out = bytearray()
    i, d = 0, bytes(data)
    while i < len(d) and len(out) < size:
        n = d[i] - 256 if d[i] > 127 else d[i]
        i += 1
        if n >= 0:
            out += d[i:i + n + 1]
            i += n + 1
        elif n != -128:
            out += d[i:i + 1] * (1 - n)
            i += 1
    out = out[:size]
    return np.frombuffer(bytes(out) + b'\x00' * (size - len(out)), np.uint8)


def decode(compression, data, size):
    """Raw bytes of one strip or tile."""
    if compression == 1:
        b = np.frombuffer(bytes(data[:size]), np.uint8)
        return b if len(b) == size else np.concatenate([b, np.zeros(size - len(b), np.uint8)])
    if compression == 5:
        return lzw_decode(data, size)
    if compression in (8, 32946):
        raw = zlib.decompress(bytes(data))
        b = np.frombuffer(raw[:size], np.uint8)
        return b if len(b) == size else np.concatenate([b, np.zeros(size - len(b), np.uint8)])
    if compression == 32773:
        return packbits_decode(data, size)
    raise ValueError('TIFF compression %d is not supported' % compression)


def encode(compression, raw):
    if compression == 1:
        return bytes(raw)
    if compression == 5:
        return lzw_encode(raw)
    if compression == 8:
        return zlib.compress(bytes(raw), 6)
    raise ValueError('TIFF compression %d is not supported for writing' % compression)


def undo_predictor(block, predictor, dtype, width, spp):
    """block: [rows, width * spp] samples of one strip / tile (file byte order) -> undone."""
    if predictor == 1:
        return block
    if predictor == 2:
        rows = block.shape[0]
        a = block.reshape(rows, width, spp)
        # cumulative sum along each row in the sample type: integer wrap, as libtiff's
        # horizontal accumulation does
        u = a.astype(a.dtype.newbyteorder('='))
        acc = np.cumsum(u, axis=1, dtype=u.dtype)
        return acc.astype(a.dtype).reshape(rows, width * spp)
    if predictor == 3:  # floating point: bytes split into planes (MSB first), then differenced
        rows = block.shape[0]
        item = dtype.itemsize
        # libtiff's fpAcc: the byte differencing runs with a stride of one pixel (spp bytes)
        raw = block.view(np.uint8).reshape(rows, width * item, spp)
        raw = np.cumsum(raw, axis=1, dtype=np.uint8).reshape(rows, width * spp * item)
        planes = raw.reshape(rows, item, width * spp)
        be = planes.transpose(0, 2, 1)  # [rows, samples, bytes MSB first]
        out = np.ascontiguousarray(be).view(dtype.newbyteorder('>')).reshape(rows, width * spp)
        return out.astype(dtype)
    raise ValueError('TIFF predictor %d is not supported' % predictor)


def apply_predictor2(block, width, spp):
    rows = block.shape[0]
    a = block.reshape(rows, width, spp)
    d = a.copy()
    d[:, 1:] = a[:, 1:] - a[:, :-1]  # wraps in the integer type
    return d.reshape(rows, width * spp)


def native_strips(compression, predictor, bits):
    """Whether lt_tiff_decode_strips / lt_tiff_encode_strips take this layout (else the
    per-strip Python path)."""
    return compression in (1, 5) and predictor in (1, 2) and bits in (8, 16, 32, 64)


def decode_strips(buf, offsets, counts, compression, predictor, dtype, big_endian, width, height,
                  bands, planar, rows_per_strip, threads, out=None):
    """Every strip of a strip-organised image, decoded on `threads` threads (liblt_io.so
    lt_tiff_decode_strips) -> [bands, height, width] in native byte order (into `out`, a C-contiguous
    array of that shape and type, when given)."""
    want = np.dtype(dtype).newbyteorder('=')
    if out is None:
        out = np.empty((bands, height, width), want)
    elif (out.shape != (bands, height, width) or out.dtype != want or
          not out.flags.c_contiguous or not out.flags.writeable):
        raise ValueError('decode_strips: out must be a writable C-contiguous %s array of shape %s'
                         % (want, (bands, height, width)))
    offs = np.ascontiguousarray(offsets, np.uint64)
    cnts = np.ascontiguousarray(counts, np.uint64)
    src = np.frombuffer(buf, np.uint8)
    rc = _lib().lt_tiff_decode_strips(src.ctypes.data, src.size, offs.ctypes.data, cnts.ctypes.data,
                                      len(offs), compression, predictor, out.itemsize,
                                      1 if big_endian else 0, width, height, bands, planar,
                                      rows_per_strip, out.ctypes.data, max(1, int(threads)))
    if rc < 0:
        raise ValueError('TIFF strips: corrupt or unsupported data (%d)' % rc)
    return out


def encode_strips(a, rows_per_strip, compression, predictor, threads):
    """[bands, rows, cols] little-endian samples -> (the strips back to back as bytes, their
    sizes), encoded on `threads` threads (liblt_io.so lt_tiff_encode_strips)."""
    a = np.ascontiguousarray(a)
    nb, rows, cols = a.shape
    n = nb * (-(-rows // rows_per_strip))
    raw = rows * cols * a.itemsize * nb
    cap = raw * 3 // 2 + 16 * n + 16 if compression == 5 else raw
    out = np.empty(cap, np.uint8)
    sizes = np.zeros(n, np.int64)
    m = _lib().lt_tiff_encode_strips(a.ctypes.data, nb, rows, cols, a.itemsize, rows_per_strip,
                                     compression, predictor, out.ctypes.data, cap,
                                     sizes.ctypes.data, max(1, int(threads)))
    if m < 0:
        raise ValueError('TIFF strips: encode failed (%d)' % m)
    return out[:m], sizes
