"""Output raster assembly: MRLandTrendrJob.output_reducer
(mr_land_trendr_job.py:128-152) -> utils.data2raster (utils.py:414-440) -> utils.array2raster
(:374-412), for the dense label / trendline planes the GPU produces.

The reference fills, per output key, a holder shaped like the template raster's band 1 with
`np.ones_like(ds2array(template)) * NODATA` (so in the template's dtype), assigns
`float(value)` at each grid point's pixel (numpy's cast into that dtype: truncation toward zero
for integer templates), and writes it with `array2raster(holder, template_fn, out_fn, compress)`
— whose fourth positional parameter is `data_type`, so `compress=True` becomes GDAL type 1,
GDT_Byte. GDAL then saturates every value into 0..255 (-99 -> 0,
1995 -> 255). Two modes:

  * 'reference': that behaviour (uint8 rasters) — parity with what the reference writes, where
    GDAL's saturating Int->Byte/Float->Byte conversion is restated (GDAL absent here: unpinned);
  * 'typed': the corrected output — each field in its own type (int32 class/onset/duration,
    float64 magnitude), NODATA -99 where a rule did not match.

Keys follow the reference: '<rule>_<field>' for labels (mr_land_trendr_job.py:120-126) and
'trendline/<YYYY-MM-DD>-<attr>' per winning acquisition date for the trendline planes
(classes.py:100-116). Files are written by write_geotiff: LZW-compressed GeoTIFF (the reference's
COMPRESS=LZW, utils.py:386) with the template's georeferencing tags copied.
"""
import struct

import numpy as np

from . import _abi
from .geotiff import GeoTiff

NODATA = _abi.LT_NODATA  # settings.py:16
LABEL_KEYS = ('class_val', 'onset_year', 'magnitude', 'duration')
TRENDLINE_ATTRS = ('val_raw', 'val_fit', 'eqn_fit_slope', 'eqn_fit_intercept', 'eqn_right_slope',
                   'eqn_right_intercept', 'spike', 'vertex')
_PLANE_OF_ATTR = {'val_raw': 'val_raw', 'val_fit': 'val_fit', 'eqn_fit_slope': 'fit_m',
                  'eqn_fit_intercept': 'fit_b', 'eqn_right_slope': 'right_m',
                  'eqn_right_intercept': 'right_b', 'spike': 'spike', 'vertex': 'vertex'}


def holder_dtype(template_dtype):
    """dtype of the reference's holder `np.ones_like(template) * NODATA` (utils.py:429) under
    numpy 1.x value-based promotion: the template's own type when it holds -99 (int16 -> int16,
    float32 -> float32), else the smallest signed type that does (uint8 -> int16,
    uint16 -> int32, uint32 -> int64)."""
    from .index_eqn import result_dtype
    return result_dtype(np.dtype(template_dtype), NODATA)


def _holder_cast(values, template_dtype):
    """numpy's assignment of float(value) into the holder's dtype (utils.py:433-438)."""
    v = np.asarray(values, np.float64)
    t = np.dtype(template_dtype)
    if t.kind == 'f':
        return v.astype(t)
    with np.errstate(invalid='ignore'):
        return np.trunc(v).astype(np.int64).astype(t)  # C cast: toward zero, then wrap


def gdal_to_byte(a):
    """GDAL's conversion of a holder into a GDT_Byte band: round (floats) and saturate."""
    a = np.asarray(a)
    if a.dtype.kind == 'f':
        a = np.where(np.isnan(a), 0.0, np.floor(a + 0.5))
    return np.clip(a, 0, 255).astype(np.uint8)


def label_rasters(out, rules, shape, template_dtype=np.int16, mode='reference'):
    """Dense label planes of one analysed tile (Engine.analyze_tile output, host or device
    tensors, [R, P] with P = rows * cols of `shape`) -> {'<rule>_<field>': 2-D array}.
    Pixels whose rule did not match hold NODATA, as the reference's holder does."""
    rows, cols = shape
    res = {}
    matched = _np(out['matched'])
    for r, rule in enumerate(rules):
        m = matched[r, :rows * cols].reshape(rows, cols).astype(bool)
        for key in LABEL_KEYS:
            plane = _np(out[key])[r, :rows * cols].reshape(rows, cols)
            if key == 'class_val':  # the reducer emits rule.val; data2raster takes float(value)
                plane = np.full(plane.shape, float(rule.val))
            if mode == 'typed':
                typ = np.float64 if key == 'magnitude' else np.int32
                res['%s_%s' % (rule.name, key)] = np.where(m, plane, NODATA).astype(typ)
            else:
                hdt = holder_dtype(template_dtype)
                holder = np.full((rows, cols), NODATA, hdt)
                holder[m] = _holder_cast(plane[m], hdt)
                res['%s_%s' % (rule.name, key)] = gdal_to_byte(holder)
    return res


def trendline_rasters(out, scene, dates, shape, template_dtype=np.int16, mode='reference',
                      attrs=TRENDLINE_ATTRS):
    """Per winning acquisition date d and attribute a, the raster 'trendline/<d>-<a>': the pixels
    whose winner in d's year is d carry the attribute, all others NODATA (the reference's
    mr_label_output keys, classes.py:100-116, reduced per key)."""
    rows, cols = shape
    n = rows * cols
    winner = _np(out['winner'])
    res = {}
    for y in range(scene.n_years):
        w = winner[y, :n].reshape(rows, cols)
        for o in np.unique(w[w >= 0]):
            d = dates[int(o)].strftime('%Y-%m-%d')
            sel = w == o
            for a in attrs:
                plane = _np(out[_PLANE_OF_ATTR[a]])[y, :n].reshape(rows, cols)
                if a in ('spike', 'vertex'):
                    plane = plane.astype(np.int64)  # mr_label_output emits 1 / 0 (classes.py:107)
                key = 'trendline/%s-%s' % (d, a)
                if mode == 'typed':
                    typ = np.uint8 if a in ('spike', 'vertex') else np.float64
                    r = np.full((rows, cols), NODATA, np.float64)
                    r[sel] = plane[sel]
                    res[key] = r.astype(typ) if typ != np.uint8 else np.where(sel, plane, 0).astype(
                        np.uint8)
                else:
                    hdt = holder_dtype(template_dtype)
                    holder = np.full((rows, cols), NODATA, hdt)
                    holder[sel] = _holder_cast(plane[sel], hdt)
                    res[key] = gdal_to_byte(holder)
    return res


def _np(t):
    try:
        import torch
        if isinstance(t, torch.Tensor):
            return t.detach().cpu().numpy()
    except ImportError:
        pass
    return np.asarray(t)


# ---- GeoTIFF writer ----------------------------------------------------------------------------
_SAMPLE_FORMAT = {'u': 1, 'i': 2, 'f': 3}
_GEO_TAGS = (33550, 33922, 34264, 34735, 34736, 34737)  # scale, tiepoint, transform, geokeys ...


def write_geotiff(path, array, template=None, nodata=NODATA, geotransform=None, compress='lzw',
                  predictor=1, rows_per_strip=None):
    """Little-endian GeoTIFF of a 2-D array, or of a 3-D [bands, rows, cols] array (planar
    configuration 2: each band's strips in turn, what GeoTiff.read returns as [bands, rows,
    cols]); georeferencing tags copied verbatim from `template` (a GeoTiff or a path), or written
    from a north-up `geotransform` (ModelPixelScale + ModelTiepoint), GDAL_NODATA set to `nodata`.
    compress: 'lzw' (array2raster's COMPRESS=LZW, utils.py:386; the native codec of
    tiffcodec.py), 'deflate' or None; predictor 2 (horizontal differencing) for integer samples.
    Strips of about 8 KB of raw samples, as GDAL's GTiff driver lays them out."""
    from . import tiffcodec
    a = np.ascontiguousarray(array)
    if a.ndim not in (2, 3) or a.dtype.kind not in _SAMPLE_FORMAT:
        raise ValueError('write_geotiff: 2-D or 3-D integer or float array required')
    comp = {None: 1, 'none': 1, 'lzw': 5, 'deflate': 8}[compress]
    if predictor not in (1, 2) or (predictor == 2 and a.dtype.kind == 'f'):
        raise ValueError('write_geotiff: predictor 1, or 2 for integer samples')
    a = a.astype(a.dtype.newbyteorder('<'), copy=False)
    if a.ndim == 2:
        a = a[None]
    nb, rows, cols = a.shape
    tmpl = GeoTiff(template) if isinstance(template, str) else template
    rps = rows_per_strip or max(1, min(rows, 8192 // max(1, cols * a.dtype.itemsize)))
    if tiffcodec.native_strips(comp, predictor, a.dtype.itemsize * 8):
        # every strip on the host's threads (liblt_io.so lt_tiff_encode_strips)
        from .ingest import host_threads
        data, sizes = tiffcodec.encode_strips(a, rps, comp, predictor, host_threads())
        bounds = np.concatenate([[0], np.cumsum(sizes)])
        mv = memoryview(data)
        strips = [mv[bounds[k]:bounds[k + 1]] for k in range(len(sizes))]
    else:
        strips = []
        for b in range(nb):
            for y0 in range(0, rows, rps):
                blk = a[b, y0:y0 + rps]
                if predictor == 2:
                    blk = tiffcodec.apply_predictor2(blk, cols, 1)
                strips.append(tiffcodec.encode(comp, np.ascontiguousarray(blk).tobytes()))

    def layout(data_off):
        entries = []  # (tag, type, count, payload bytes)

        def add(tag, typ, values, fmt):
            payload = struct.pack('<' + fmt * len(values), *values)
            entries.append((tag, typ, len(values), payload))

        offs, o = [], data_off
        for st in strips:
            offs.append(o)
            o += len(st)
        add(256, 4, [cols], 'I')
        add(257, 4, [rows], 'I')
        add(258, 3, [a.dtype.itemsize * 8] * nb, 'H')
        add(259, 3, [comp], 'H')
        add(262, 3, [1], 'H')
        add(273, 4, offs, 'I')
        add(277, 3, [nb], 'H')
        add(278, 4, [rps], 'I')
        add(279, 4, [len(st) for st in strips], 'I')
        add(284, 3, [2 if nb > 1 else 1], 'H')
        if predictor == 2:
            add(317, 3, [2], 'H')
        add(339, 3, [_SAMPLE_FORMAT[a.dtype.kind]] * nb, 'H')
        if tmpl is not None:
            for tag in _GEO_TAGS:
                if tag in tmpl.tags:
                    v = tmpl.tags[tag]
                    if isinstance(v, str):
                        entries.append((tag, 2, len(v), v.encode('latin-1')))
                    elif tag == 34735:
                        add(tag, 3, [int(x) for x in v], 'H')
                    else:
                        add(tag, 12, [float(x) for x in v], 'd')
        elif geotransform is not None:
            x0, sx, rx, y0, ry, sy = (float(v) for v in geotransform)
            if rx != 0.0 or ry != 0.0:
                raise ValueError('write_geotiff: rotated geotransforms are not supported')
            add(33550, 12, [sx, -sy, 0.0], 'd')
            add(33922, 12, [0.0, 0.0, 0.0, x0, y0, 0.0], 'd')
        if nodata is not None:
            s = ('%g' % nodata).encode() + b'\x00'
            entries.append((42113, 2, len(s), s))
        entries.sort(key=lambda e: e[0])
        n = len(entries)
        ifd_off = 8
        extra_off = ifd_off + 2 + 12 * n + 4
        extra = b''
        ifd = struct.pack('<H', n)
        for tag, typ, cnt, payload in entries:
            if len(payload) <= 4:
                ifd += struct.pack('<HHI', tag, typ, cnt) + payload.ljust(4, b'\x00')
            else:
                if len(extra) % 2:
                    extra += b'\x00'
                ifd += struct.pack('<HHII', tag, typ, cnt, extra_off + len(extra))
                extra += payload
        ifd += struct.pack('<I', 0)
        end = extra_off + len(extra)
        return ifd_off, ifd, extra, end + (-end) % 8

    # the header's size does not depend on the offset values: lay out once to find where the
    # pixel data starts, then again with the real strip offsets
    data_off = layout(0)[3]
    ifd_off, ifd, extra, end = layout(data_off)
    assert end == data_off
    if data_off + sum(len(st) for st in strips) >= 1 << 32:
        raise ValueError('write_geotiff: over 4 GiB needs BigTIFF, which is not written')
    with open(path, 'wb') as f:
        f.write(b'II*\x00' + struct.pack('<I', ifd_off))
        f.write(ifd)
        f.write(extra)
        f.write(b'\x00' * (data_off - ifd_off - len(ifd) - len(extra)))
        if strips and isinstance(strips[0], memoryview):  # back to back already
            f.write(strips[0].obj[:sum(len(st) for st in strips)])
        else:
            for st in strips:
                f.write(st)
    return path


def output_reducer(rasters, template, out_dir, job='job', compress='lzw'):
    """The file side of output_reducer (mr_land_trendr_job.py:128-152) without S3: every key's
    raster written as <out_dir>/<job>/output/rasters/<key>.tif (settings.py OUT_RAST_KEYNAME) with
    the template's georeferencing. Yields (key, [path]) like the reducer yields (key, [s3 key])."""
    import os
    tmpl = GeoTiff(template) if isinstance(template, str) else template
    for key in sorted(rasters):
        path = os.path.join(out_dir, '%s/output/rasters/%s.tif' % (job, key))
        os.makedirs(os.path.dirname(path), exist_ok=True)
        write_geotiff(path, rasters[key], template=tmpl, compress=compress)
        yield key, [path]


# ---- the same rasters assembled on the GPU (lt_raster_assemble) --------------------------------
def _job(n_pix, n_out, plane, sel_kind, sel, sel_value, holder_t, const_value, dest, mode,
         out_type, out):
    from . import engine as _eng
    j = _abi.LtRasterJob()
    j.n_pix, j.n_out = n_pix, n_out
    if plane is not None:
        j.plane, j.plane_type = plane.data_ptr(), _eng._LT_T[plane.dtype]
    j.sel_kind, j.sel, j.sel_value = sel_kind, sel.data_ptr() if sel is not None else None, \
        int(sel_value)
    j.holder_type = holder_t
    j.const_value = float(const_value)
    j.dest = dest.data_ptr() if dest is not None else None
    j.mode, j.out_type, j.fill, j.out = mode, out_type, float(NODATA), out.data_ptr()
    return j


def label_rasters_device(engine, planes, rules, shape, dest=None, template_dtype=np.int16,
                         mode='reference'):
    """label_rasters for [R, P] planes in device memory (matched, onset_year, duration,
    magnitude): each '<rule>_<field>' raster is assembled by lt_raster_assemble and only the
    finished raster is copied to the host. dest: None (grid point p is raster pixel p) or a device
    int64 [P] of distinct raster offsets. Same values as label_rasters on the host planes."""
    import torch
    from .index_eqn import DTYPES
    rows, cols = shape
    n_out = rows * cols
    P = planes['matched'].shape[-1]
    ref = mode == 'reference'
    hdt = DTYPES[holder_dtype(template_dtype)] if ref else 0
    jobs, res = [], {}
    for r, rule in enumerate(rules):
        sel = planes['matched'][r]
        for key in LABEL_KEYS:
            typ = torch.uint8 if ref else (torch.float64 if key == 'magnitude' else torch.int32)
            out = torch.empty(n_out, dtype=typ, device=engine.device)
            plane = None if key == 'class_val' else planes[key][r]
            jobs.append(_job(P, n_out, plane, _abi.LT_SEL_NONZERO, sel, 0, hdt,
                             float(rule.val) if key == 'class_val' else 0.0, dest,
                             _abi.LT_RASTER_REFERENCE if ref else _abi.LT_RASTER_TYPED,
                             {torch.uint8: _abi.LT_T_U8, torch.int32: _abi.LT_T_I32,
                              torch.float64: _abi.LT_T_F64}[typ], out))
            res['%s_%s' % (rule.name, key)] = out
    engine.raster_assemble(jobs)
    return {k: v.cpu().numpy().reshape(rows, cols) for k, v in res.items()}


def trendline_rasters_device(engine, planes, scene, dates, shape, dest=None,
                             template_dtype=np.int16, mode='reference', attrs=TRENDLINE_ATTRS,
                             sink=None):
    """trendline_rasters for [Y, P] planes in device memory: the winning acquisition dates come
    from lt_winner_presence, each 'trendline/<date>-<attr>' raster from lt_raster_assemble, one
    year slot at a time; sink(key, array) receives each raster as it reaches the host (default:
    collected into the returned dict). Dates shared by two observations fall back to the host."""
    import ctypes
    import torch
    from .index_eqn import DTYPES
    rows, cols = shape
    n_out = rows * cols
    w = planes['winner']
    Y, P = w.shape
    K = scene.n_obs
    names = [d.strftime('%Y-%m-%d') for d in dates]
    if len(set(names)) != len(names):
        raise ValueError('two observations share an acquisition date: assemble on the host')
    bits = torch.zeros((K + 31) // 32, dtype=torch.int32, device=engine.device)
    st = torch.cuda.current_stream(engine.device)
    engine._check(engine.lib.lt_winner_presence(engine.ctx, w.data_ptr(), w.stride(0), Y, P, K,
                                                bits.data_ptr(), ctypes.c_void_p(st.cuda_stream)),
                  'lt_winner_presence')
    b = bits.cpu().numpy().view(np.uint32)
    present = [o for o in range(K) if (b[o >> 5] >> (o & 31)) & 1]
    slot_of = {}
    for y in range(scene.n_years):
        for k in range(scene.slot_begin[y], scene.slot_begin[y + 1]):
            slot_of[int(scene.order[k])] = y
    ref = mode == 'reference'
    hdt = DTYPES[holder_dtype(template_dtype)] if ref else 0
    res = {}
    for o in present:
        y = slot_of[o]
        jobs, outs = [], []
        for a in attrs:
            plane = planes[_PLANE_OF_ATTR[a]][y]
            if ref:
                typ, ot = torch.uint8, _abi.LT_T_U8
            else:
                typ, ot = ((torch.uint8, _abi.LT_T_U8) if a in ('spike', 'vertex') else
                           (torch.float64, _abi.LT_T_F64))
            out = torch.empty(n_out, dtype=typ, device=engine.device)
            j = _job(P, n_out, plane, _abi.LT_SEL_EQUALS, w[y], o, hdt, 0.0, dest,
                     _abi.LT_RASTER_REFERENCE if ref else _abi.LT_RASTER_TYPED, ot, out)
            if not ref and a in ('spike', 'vertex'):
                j.fill = 0.0
            jobs.append(j)
            outs.append(('trendline/%s-%s' % (names[o], a), out))
        engine.raster_assemble(jobs)
        for key, out in outs:
            arr = out.cpu().numpy().reshape(rows, cols)
            if sink is not None:
                sink(key, arr)
            else:
                res[key] = arr
    return res
