"""Minimal GeoTIFF reader for co-registered Landsat stacks (SURVEY.md §8(f)-2 ingest, first piece).

The reference reads rasters with GDAL (`ds2array`, utils.py:272-282; `rast_algebra` :447-484);
GDAL is not in this image. This reads the TIFF subset such stacks use: little- or big-endian
classic TIFF, strips or tiles, uncompressed, LZW, Deflate or PackBits (tiffcodec.py; LZW
native), horizontal / floating-point predictors, chunky or planar bands, sample formats
uint/int/float of 8/16/32/64 bits, plus the GeoTIFF/GDAL tags kept as raw values
(ModelPixelScale, ModelTiepoint, GeoKeyDirectory, GDAL_NODATA). Returns numpy arrays in the
file's sample type, [bands, rows, cols] — what `ds2array(ds, b)` gives per band.
"""
import mmap
import os
import struct

import numpy as np

from . import tiffcodec

_TYPES = {1: ('B', 1), 2: ('s', 1), 3: ('H', 2), 4: ('I', 4), 5: ('II', 8), 6: ('b', 1),
          7: ('B', 1), 8: ('h', 2), 9: ('i', 4), 10: ('ii', 8), 11: ('f', 4), 12: ('d', 8),
          16: ('Q', 8), 17: ('q', 8)}
_SAMPLE = {(1, 8): np.uint8, (1, 16): np.uint16, (1, 32): np.uint32, (1, 64): np.uint64,
           (2, 8): np.int8, (2, 16): np.int16, (2, 32): np.int32, (2, 64): np.int64,
           (3, 32): np.float32, (3, 64): np.float64}


class TiffError(ValueError):
    pass


class GeoTiff:
    def __init__(self, path):
        with open(path, 'rb') as f:
            # mapped, not read: the strip decoder reads the compressed strips where the page cache
            # holds them (a read() copied every 174 MB raster of a c2-size stack once more)
            # (LT_TIFF_MMAP=0: read, for A/B runs)
            try:
                if os.environ.get('LT_TIFF_MMAP', '1') == '0':
                    raise ValueError
                self._d = mmap.mmap(f.fileno(), 0, access=mmap.ACCESS_READ)
            except (ValueError, OSError):  # an empty or unmappable file
                self._d = f.read()
        d = self._d
        if d[:2] == b'II':
            self._bo = '<'
        elif d[:2] == b'MM':
            self._bo = '>'
        else:
            raise TiffError('%s: not a TIFF file' % path)
        magic, off = struct.unpack(self._bo + 'HI', d[2:8])
        if magic != 42:
            raise TiffError('%s: BigTIFF / unknown TIFF version %d' % (path, magic))
        self.tags = self._ifd(off)
        t = self.tags
        self.width = int(t[256][0])
        self.height = int(t[257][0])
        bps = t.get(258, (1,))
        self.bits = int(bps[0])
        if any(int(b) != self.bits for b in bps):
            raise TiffError('mixed bits per sample')
        self.bands = int(t.get(277, (1,))[0])
        fmt = int(t.get(339, (1,))[0])
        self.compression = int(t.get(259, (1,))[0])
        if self.compression not in (1, 5, 8, 32946, 32773):
            raise TiffError('TIFF compression %d is not supported' % self.compression)
        self.predictor = int(t.get(317, (1,))[0])
        if (fmt, self.bits) not in _SAMPLE:
            raise TiffError('sample format %d / %d bits not supported' % (fmt, self.bits))
        self.dtype = np.dtype(_SAMPLE[(fmt, self.bits)]).newbyteorder(self._bo)
        self.planar = int(t.get(284, (1,))[0])
        nd = t.get(42113)
        self.nodata = float(nd.rstrip('\x00')) if nd else None
        self.pixel_scale = t.get(33550)
        self.tiepoint = t.get(33922)
        self.geokeys = t.get(34735)

    def geotransform(self):
        """GDAL's GetGeoTransform() of this file: (top_left_x, pix_width, x_rot, top_left_y,
        y_rot, pix_height), from ModelTransformation (34264) or ModelTiepoint + ModelPixelScale,
        as GDAL's GTiff driver derives it (PixelIsPoint rasters shifted by half a pixel, the
        driver's default). No georeferencing: GDAL's default (0, 1, 0, 0, 0, 1)."""
        point = False
        if self.geokeys:  # GTRasterTypeGeoKey (1025) == RasterPixelIsPoint (2)
            g = self.geokeys
            for k in range(4, 4 + 4 * int(g[3]), 4):
                if g[k] == 1025 and g[k + 1] == 0 and g[k + 3] == 2:
                    point = True
        mt = self.tags.get(34264)
        if mt is not None:
            gt = [mt[3], mt[0], mt[1], mt[7], mt[4], mt[5]]
        elif self.tiepoint and self.pixel_scale:
            i, j, _, x, y, _ = self.tiepoint[:6]
            sx, sy = self.pixel_scale[0], self.pixel_scale[1]
            gt = [x - i * sx, sx, 0.0, y + j * sy, 0.0, -sy]
        else:
            return (0.0, 1.0, 0.0, 0.0, 0.0, 1.0)
        if point:
            gt[0] -= gt[1] * 0.5 + gt[2] * 0.5
            gt[3] -= gt[4] * 0.5 + gt[5] * 0.5
        return tuple(float(v) for v in gt)

    def _ifd(self, off):
        d, bo = self._d, self._bo
        (n,) = struct.unpack(bo + 'H', d[off:off + 2])
        tags = {}
        for i in range(n):
            tag, typ, cnt, val = struct.unpack(bo + 'HHI4s', d[off + 2 + 12 * i:off + 14 + 12 * i])
            if typ not in _TYPES:
                continue
            code, size = _TYPES[typ]
            nbytes = size * cnt
            if nbytes <= 4:
                raw = val[:nbytes]
            else:  # (d[o:][:n] would copy the rest of the file first: 0.14 s per 174 MB raster)
                o = struct.unpack(bo + 'I', val)[0]
                raw = d[o:o + nbytes]
            if typ == 2:
                tags[tag] = raw.decode('latin-1')
            elif typ in (5, 10):
                v = struct.unpack(bo + code[0] * (2 * cnt), raw)
                tags[tag] = tuple(v[k] / v[k + 1] for k in range(0, len(v), 2))
            else:
                tags[tag] = struct.unpack(bo + code * cnt, raw)
        return tags

    def _chunk(self, k, rows, cols, spp):
        """Decoded samples of strip / tile k: [rows, cols * spp] in the file's byte order."""
        t, d = self.tags, self._d
        offs = t[273] if 273 in t else t[324]
        counts = t[279] if 279 in t else t[325]
        size = rows * cols * spp * self.dtype.itemsize
        try:
            raw = tiffcodec.decode(self.compression, d[offs[k]:offs[k] + counts[k]], size)
        except ValueError as e:
            raise TiffError(str(e))
        block = np.frombuffer(raw.tobytes(), self.dtype, rows * cols * spp).reshape(
            rows, cols * spp)
        try:
            return tiffcodec.undo_predictor(block, self.predictor, self.dtype, cols, spp)
        except ValueError as e:
            raise TiffError(str(e))

    def read(self, threads=None, native=True, out=None):
        """All bands as a [bands, rows, cols] array in the sample type (native byte order).
        Strip-organised LZW / uncompressed images with integer predictors are decoded on
        `threads` threads by liblt_io.so (default: the host's share, ingest.host_threads), into
        `out` when given (a C-contiguous array of that shape and type; the other paths copy into
        it); native=False takes the per-strip path (tests compare the two)."""
        if out is not None and not (native and 273 in self.tags and tiffcodec.native_strips(
                self.compression, self.predictor, self.bits) and (
                self.predictor == 1 or self.dtype.kind in 'iu')):
            out[...] = self.read(threads, native)
            return out
        t = self.tags
        W, H, B = self.width, self.height, self.bands
        spp = B if self.planar == 1 else 1
        if native and 273 in t and tiffcodec.native_strips(self.compression, self.predictor, self.bits) and (
                self.predictor == 1 or self.dtype.kind in 'iu'):
            if threads is None:
                from .ingest import host_threads
                threads = host_threads()
            rps = min(int(t.get(278, (H,))[0]), H)
            try:
                return tiffcodec.decode_strips(self._d, t[273], t[279], self.compression,
                                               self.predictor, self.dtype, self._bo == '>', W, H,
                                               B, self.planar, rps, threads, out=out)
            except ValueError as e:
                raise TiffError(str(e))
        if 273 in t:  # strips
            rps = min(int(t.get(278, (H,))[0]), H)
            per_band = -(-H // rps)
            a = np.empty((B, H, W), self.dtype)
            for k in range(len(t[273])):
                b0, r = (0, k) if self.planar == 1 else (k // per_band, k % per_band)
                y0 = r * rps
                rows = min(rps, H - y0)
                if rows <= 0 or b0 >= B:
                    continue
                blk = self._chunk(k, rows, W, spp)
                if self.planar == 1:
                    a[:, y0:y0 + rows, :] = blk.reshape(rows, W, B).transpose(2, 0, 1)
                else:
                    a[b0, y0:y0 + rows, :] = blk
        elif 324 in t:  # tiles
            tw, th = int(t[322][0]), int(t[323][0])
            tx, ty = -(-W // tw), -(-H // th)
            per_band = tx * ty
            a = np.empty((B, ty * th, tx * tw), self.dtype)
            for k in range(len(t[324])):
                b0 = 0 if self.planar == 1 else k // per_band
                r = k % per_band
                yy, xx = (r // tx) * th, (r % tx) * tw
                blk = self._chunk(k, th, tw, spp)
                if self.planar == 1:
                    a[:, yy:yy + th, xx:xx + tw] = blk.reshape(th, tw, spp).transpose(2, 0, 1)
                else:
                    a[b0, yy:yy + th, xx:xx + tw] = blk
            a = a[:, :H, :W]
        else:
            raise TiffError('no strip or tile offsets')
        return np.ascontiguousarray(a).astype(self.dtype.newbyteorder('='), copy=False)


def read_bands(path):
    """[bands, rows, cols] numpy array of a GeoTIFF (GDAL's ReadAsArray per band, stacked)."""
    return GeoTiff(path).read()
