"""Input ingest: the mapper side of the reference pipeline, restated
without GDAL/OGR/S3 over co-registered GeoTIFF stacks.

Reference flow, per analysis raster (MRLandTrendrJob.parse_mapper, mr_land_trendr_job.py:48-81):
  rast_dl -> rast_algebra(index_eqn) -> filename2date -> apply_grid(index raster, grid, mask)
  -> one (pix_ctr_wkt, {'val', 'date'}) pair per grid point whose mask value is not 0.
The reducer then sees, per grid point, the list of its observations.

Here the same data is assembled as planes for the GPU: `ingest_stack` gathers, for every raster k
and grid point p, the band samples bands[k, :, p] and valid[k, p] (1 unless the point is off the
raster or its cloud mask value is 0, exactly the cases apply_grid skips), and the index equation
runs on the GPU over those samples (utils.index_tile — elementwise, so evaluating it at the grid
points equals sampling the evaluated raster). The per-point generators (`serialize_rast`,
`apply_grid`) are kept with the reference's semantics, including its WKT text (Python 2 float
formatting), numpy's negative-index wrap in pt2val and the exceptions it swallows.
"""
import datetime as _dt
import glob
import os
import shutil
import tarfile
import zipfile

import numpy as np

from .geotiff import GeoTiff

RAST_TRIGGER = 'ledaps'      # settings.py:11
MASK_TRIGGER = 'cloudmask'   # settings.py:12


# ---- string parsing (utils.py:189-225) ---------------------------------------------------------
def filename2date(fn):
    """utils.filename2date (utils.py:204-217): 'LE7045029_1999_211_..._cloudmask.tif.tar.gz'
    -> '1999-07-30' (year, day of year from the 2nd and 3rd '_' fields)."""
    chunks = os.path.basename(fn).split('_')
    yr, days = int(chunks[1]), int(chunks[2])
    d = _dt.datetime(year=yr, month=1, day=1) + _dt.timedelta(days=days - 1)
    return d.strftime('%Y-%m-%d')


def py2_float_str(x):
    """Python 2's str(float): repr with 12 significant digits ('%.12g'), '.0' appended when the
    text would read as an integer (what '%s' % x gives in the reference's WKT, utils.py:321)."""
    x = float(x)
    if x != x:
        return 'nan'
    if x in (float('inf'), float('-inf')):
        return 'inf' if x > 0 else '-inf'
    s = '%.12g' % x
    if not any(ch in s for ch in '.en'):
        s += '.0'
    return s


def point_wkt(x, y):
    return 'POINT(%s %s)' % (py2_float_str(x), py2_float_str(y))


def parse_point_wkt(wkt):
    """OGR's CreateGeometryFromWkt(...).GetX()/GetY() for 'POINT(x y)' (and data2raster's own
    split, utils.py:430-431): correctly rounded decimal -> binary64, as float()."""
    clean = wkt.replace('POINT', '').replace('(', '').replace(')', '').strip()
    a, b = clean.split()
    return float(a), float(b)


# ---- compression (utils.py:11-45) --------------------------------------------------------------
def decompress(filename, out_dir='/tmp/decompressed'):
    """utils.decompress: extract a zip or tar(.gz) into out_dir and list its files; an existing
    out_dir is returned as is (the reference's cache); ValueError for any other file type."""
    if os.path.exists(out_dir):
        return glob.glob(os.path.join(out_dir, '*'))
    os.makedirs(out_dir)
    ok = False
    try:
        if zipfile.is_zipfile(filename):
            zipfile.ZipFile(filename, 'r').extractall(out_dir)
        elif tarfile.is_tarfile(filename):
            with tarfile.open(filename, 'r') as tf:
                tf.extractall(out_dir, filter='data')
        else:
            raise ValueError('Invalid file type - must be tar.gz or zip')
        ok = True
    finally:
        if not ok:
            shutil.rmtree(out_dir)
    return [os.path.join(out_dir, f) for f in os.listdir(out_dir)]


def rast_local(fn, work_dir):
    """rast_dl (utils.py:126-135) minus the download: a compressed raster is decompressed into
    work_dir/<name without .tif/.tar.gz/.zip> and its first file returned; a plain .tif as is."""
    if zipfile.is_zipfile(fn) or (os.path.isfile(fn) and tarfile.is_tarfile(fn)):
        name = os.path.basename(fn).replace('.tif', '').replace('.tar.gz', '').replace('.zip', '')
        return sorted(decompress(fn, os.path.join(work_dir, name)))[0]
    return fn


# ---- grid (utils.py:252-370) -------------------------------------------------------------------
def _open(r):
    return r if isinstance(r, GeoTiff) else GeoTiff(r)


def get_pix_offsets_for_point(gt, lng, lat):
    """utils.get_pix_offsets_for_point (utils.py:252-269) on a geotransform tuple: int() of the
    distance over the pixel size, i.e. truncation toward zero."""
    top_left_x, pix_width, _, top_left_y, _, pix_height = gt
    x_offset = int((lng - top_left_x) * 1.0 / pix_width)
    y_offset = int((lat - top_left_y) * 1.0 / pix_height)
    return x_offset, y_offset


def pt2val(gt, pt_wkt, raster_array):
    """utils.pt2val (utils.py:285-297): raster_array[y_off, x_off] with numpy's indexing rules
    (negative offsets wrap, out-of-range ones raise IndexError)."""
    lng, lat = parse_point_wkt(pt_wkt)
    x_off, y_off = get_pix_offsets_for_point(gt, lng, lat)
    return raster_array[y_off, x_off]


def serialize_rast(rast_fn, extra_data={}):
    """utils.serialize_rast (utils.py:300-325): (pixel-centre WKT, {'val': float, **extra}) for
    every pixel of band 1, columns outer, rows inner."""
    ds = _open(rast_fn)
    top_left_x, pix_width, _, top_left_y, _, pix_height = ds.geotransform()
    pixvals = ds.read()[0]
    for xoff in range(ds.width):
        x = top_left_x + (xoff + 0.5) * pix_width
        for yoff in range(ds.height):
            y = top_left_y + (yoff + 0.5) * pix_height
            pt_data = {'val': float(pixvals[yoff, xoff])}
            pt_data.update(extra_data)
            yield point_wkt(x, y), pt_data


def _grid_text(ds):
    """The distinct coordinate texts of rast2grid's grid: one per raster column (x) and row (y),
    the same operations serialize_rast does (utils.py:315-321)."""
    ds = _open(ds)
    top_left_x, pix_width, _, top_left_y, _, pix_height = ds.geotransform()
    xs = top_left_x + (np.arange(ds.width, dtype=np.float64) + 0.5) * pix_width
    ys = top_left_y + (np.arange(ds.height, dtype=np.float64) + 0.5) * pix_height
    return [py2_float_str(v) for v in xs], [py2_float_str(v) for v in ys]


def grid_wkts(ds):
    """The WKT column rast2grid writes, vectorised (same operations, same order)."""
    xt, yt = _grid_text(ds)
    return ['POINT(%s %s)' % (a, b) for a in xt for b in yt]


def grid_axes(ds):
    """The grid's distinct coordinates as grid_coords parses them: (x of each raster column,
    y of each raster row)."""
    xt, yt = _grid_text(ds)
    return (np.array([float(t) for t in xt], np.float64),
            np.array([float(t) for t in yt], np.float64))


def grid_coords(ds):
    """grid_points of the grid rast2grid writes for raster `ds`, without the text round trip per
    point: each distinct coordinate text (one per column and per row) is parsed once, as OGR /
    float() parse it, and laid out in the grid's order (columns outer, rows inner). Equal to
    grid_points(rast2grid(ds)) (tests/test_ingest.py)."""
    xt, yt = _grid_text(ds)
    xv = np.array([float(t) for t in xt], np.float64)
    yv = np.array([float(t) for t in yt], np.float64)
    return np.repeat(xv, len(yv)), np.tile(yv, len(xv))


def rast2grid(rast_fn, out_csv='/tmp/grid.csv'):
    """utils.rast2grid (utils.py:361-370): CSV with a 'pix_ctr_wkt' column, one pixel centre per
    line (pandas to_csv, index=False: no quoting is needed for 'POINT(x y)')."""
    xt, yt = _grid_text(rast_fn)
    with open(out_csv, 'w') as f:
        f.write('pix_ctr_wkt\n')
        for a in xt:  # one column of points (rows inner) per join
            pre = 'POINT(%s ' % a
            f.write(pre + (')\n' + pre).join(yt) + ')\n')
    return out_csv


def read_grid(grid):
    """The 'pix_ctr_wkt' column of a grid CSV (or a list of WKTs, returned as is)."""
    if not isinstance(grid, (str, os.PathLike)):
        return list(grid)
    with open(grid) as f:
        header = f.readline().rstrip('\n').split(',')
        col = header.index('pix_ctr_wkt')
        return [line.rstrip('\n').split(',')[col].strip('"') for line in f if line.strip()]


def grid_points(grid):
    """Grid WKTs -> (lng, lat) float64 arrays."""
    pts = np.array([parse_point_wkt(w) for w in read_grid(grid)], np.float64).reshape(-1, 2)
    return pts[:, 0].copy(), pts[:, 1].copy()


def grid_offsets(gt, shape, lng, lat):
    """Vectorised pt2val addressing for many points: flat pixel index of each point in a raster
    of `shape` and whether pt2val would return a value there (numpy wrap for offsets in
    [-n, 0), IndexError -> False beyond)."""
    rows, cols = shape
    top_left_x, pix_width, _, top_left_y, _, pix_height = gt
    xo = np.trunc((lng - top_left_x) * 1.0 / pix_width)
    yo = np.trunc((lat - top_left_y) * 1.0 / pix_height)
    ok = (xo >= -cols) & (xo < cols) & (yo >= -rows) & (yo < rows)
    xo = np.where(ok, xo, 0).astype(np.int64)
    yo = np.where(ok, yo, 0).astype(np.int64)
    xo = np.where(xo < 0, xo + cols, xo)
    yo = np.where(yo < 0, yo + rows, yo)
    return yo * cols + xo, ok


def mask_name(rast_fn):
    """parse_mapper's mask key (mr_land_trendr_job.py:59): RAST_TRIGGER -> MASK_TRIGGER."""
    return rast_fn.replace(RAST_TRIGGER, MASK_TRIGGER)


def apply_grid(rast_fn, grid_fn, extra_data={}, mask_fn=None):
    """utils.apply_grid (utils.py:328-359), per point: (wkt, {'val': float(v), **extra}) for the
    grid points on the raster whose mask value (when the mask has one there) is not 0."""
    ds = _open(rast_fn)
    gt, arr = ds.geotransform(), ds.read()[0]
    if mask_fn:
        mds = _open(mask_fn)
        mgt, marr = mds.geotransform(), mds.read()[0]
    for wkt in read_grid(grid_fn):
        try:
            val = pt2val(gt, wkt, arr)
        except Exception:  # grid points off the raster
            continue
        if mask_fn:
            try:
                if pt2val(mgt, wkt, marr) == 0:
                    continue
            except Exception:  # an invalid mask is ignored
                pass
        pt_data = {'val': float(val)}
        pt_data.update(extra_data)
        yield wkt, pt_data


def analysis_rasters(paths):
    """setup_mapper's raster list (mr_land_trendr_job.py:29-32): the files whose name holds
    RAST_TRIGGER, in key order (S3 lists keys lexicographically)."""
    return sorted(p for p in paths if RAST_TRIGGER in os.path.basename(p))


def host_threads():
    """CPU threads this process should use: its affinity set, capped by the cgroup CPU quota when
    one is set (a GPU box shows the whole machine's CPUs but grants each job a share)."""
    try:
        n = len(os.sched_getaffinity(0))
    except AttributeError:
        n = os.cpu_count() or 1
    try:
        q, per = open('/sys/fs/cgroup/cpu.max').read().split()[:2]
        if q != 'max':
            n = max(1, min(n, -(-int(q) // int(per))))
    except (OSError, ValueError):
        pass
    return n


class _Offsets:
    """grid_offsets per distinct (geotransform, shape), computed once (a stack's rasters nearly
    all share one), with whether the grid is the raster's own pixels in order (then sampling is
    a plain copy). raster_grid = (geotransform, rows, cols): the caller knows the grid is exactly
    that raster's pixels in raster order (LocalJob._internal_order), so a raster of that
    geotransform and shape is a copy without computing 49 M offsets."""

    def __init__(self, lng, lat, raster_grid=None):
        import threading
        self.lng, self.lat = lng, lat
        self.raster_grid = raster_grid
        self.cache = {}
        self.lock = threading.Lock()

    def __call__(self, ds):
        key = (ds.geotransform(), ds.height, ds.width)
        if self.raster_grid is not None and key == tuple(self.raster_grid):
            return None, None, True
        with self.lock:
            hit = self.cache.get(key)
            if hit is None:
                idx, ok = grid_offsets(key[0], (ds.height, ds.width), self.lng, self.lat)
                ident = bool(ok.all()) and len(idx) == ds.height * ds.width and bool(
                    (idx == np.arange(len(idx))).all())
                hit = self.cache[key] = (idx, ok, ident)
        return hit


def ingest_stack(rast_fns, grid, mask_fns=None, bands=None, threads=None, pixels=None,
                 raster_grid=None, on_raster=None):
    """parse_mapper over every analysis raster, as planes for analysis_reducer_batch.

    rast_fns: the (decompressed) analysis rasters, in the mapper order that becomes each pixel's
    observation order; grid: CSV path, WKT list or (lng, lat) arrays (P points); mask_fns: per
    raster the mask path or None (default: mask_name(fn) when that file exists); bands: the band
    numbers to gather (default: all bands of each raster); threads: decode / gather workers
    (default host_threads(): the codecs and the gathers release the GIL); pixels: None (every
    grid point) or a list of grid-point ranges [(p0, p1), ...] — a rank's tiles of a multi-rank
    job — whose samples alone are gathered, back to back, so a rank holds 1/N of the stack's
    planes (the reference shards parse_mapper per raster, mr_land_trendr_job.py:45-81; here each
    rank keeps the pixel columns its tiles analyse).
    Returns dict(dates=['YYYY-MM-DD'] * K, bands=[K, nb, Q] in the rasters' sample type,
    band_numbers=[nb], valid=[K, Q] uint8, n_pix=P, ranges=[(p0, p1, q0)]) with Q the points
    gathered; grid point p of range (p0, p1, q0) is column q0 + p - p0 (stack_range).
    raster_grid: (geotransform, rows, cols) when grid point p is pixel p of such a raster (the
    job's raster order): rasters of that georeferencing are read by slicing, not by offsets.
    on_raster(k, bands_k [nb, Q], valid_k [Q]): called on the worker thread once raster k's planes
    are complete (the job copies them to the GPU while the other rasters decode)."""
    from concurrent.futures import ThreadPoolExecutor
    lng, lat = grid if isinstance(grid, tuple) else grid_points(grid)
    P = len(lng)
    K = len(rast_fns)
    if pixels is None:
        pixels = [(0, P)] if P else []
    ranges, q = [], 0
    for p0, p1 in pixels:
        if not 0 <= p0 <= p1 <= P:
            raise ValueError('pixel range (%d, %d) outside the grid of %d points' % (p0, p1, P))
        ranges.append((int(p0), int(p1), q))
        q += p1 - p0
    Q = q
    if len(ranges) != 1 or ranges[0][:2] != (0, P):
        sel_pts = (np.concatenate([np.arange(a, b) for a, b, _ in ranges]) if ranges
                   else np.zeros(0, np.int64))
        lng, lat = lng[sel_pts], lat[sel_pts]
    if mask_fns is None:
        mask_fns = [mask_name(f) if os.path.exists(mask_name(f)) and mask_name(f) != f else None
                    for f in rast_fns]
    if K == 0:
        return dict(dates=[], bands=np.zeros((0, 0, Q)), band_numbers=list(bands or []),
                    valid=np.zeros((0, Q), np.uint8), n_pix=P, ranges=ranges)
    first = _open(rast_fns[0])
    numbers = list(bands) if bands is not None else list(range(1, first.bands + 1))
    dtype = first.dtype.newbyteorder('=')
    out_bands = np.empty((K, len(numbers), Q), dtype)
    valid = np.empty((K, Q), np.uint8)
    offsets = _Offsets(lng, lat, raster_grid)
    sel = [b - 1 for b in numbers]
    spans = [(p0, p1, q0) for p0, p1, q0 in ranges]

    def take(flat, idx, ok, ident, out):
        """Samples of the gathered grid points from a raster's flat [..., H*W] samples."""
        if ident and idx is None:  # raster order: the pixel ranges themselves
            if len(spans) == 1 and spans[0][:2] == (0, P) and flat.shape[-1] == P:
                out[...] = flat
            else:
                for p0, p1, q0 in spans:
                    out[..., q0:q0 + p1 - p0] = flat[..., p0:p1]
        elif ident:
            out[...] = flat
        else:
            np.take(flat, idx, axis=-1, out=out)

    def one(k):
        fn = rast_fns[k]
        ds = first if k == 0 else _open(fn)
        if ds.dtype.newbyteorder('=') != dtype:
            raise ValueError('%s: sample type %s differs from the stack\'s %s' % (fn, ds.dtype, dtype))
        if max(numbers) > ds.bands:
            raise Exception('Band %s requested but raster only has %s bands' % (max(numbers),
                                                                                 ds.bands))
        idx, ok, ident = offsets(ds)
        if (ident and idx is None and sel == list(range(ds.bands)) and len(spans) == 1 and
                spans[0][:2] == (0, P) and ds.width * ds.height == P):
            # raster order, every band, one full range: decoded in place (no copy of the planes)
            ds.read(threads=per_file, out=out_bands[k].reshape(ds.bands, ds.height, ds.width))
        else:
            planes = ds.read(threads=per_file).reshape(ds.bands, -1)
            src = planes[sel] if sel != list(range(ds.bands)) else planes
            take(src, idx, ok, ident, out_bands[k])
        if ok is not None and not ident:
            out_bands[k][:, ~ok] = 0
        v = valid[k]
        v[...] = 1 if ok is None else ok
        if mask_fns[k]:
            mds = _open(mask_fns[k])
            midx, mok, mident = offsets(mds)
            m = mds.read(threads=per_file)[0].reshape(-1)
            mval = np.empty(Q, m.dtype)
            take(m, midx, mok, mident, mval)
            drop = (mval == 0) if mok is None else (mok & (mval == 0))
            v &= ~drop
        if on_raster is not None:
            on_raster(k, out_bands[k], valid[k])
        return filename2date(fn)

    total = threads or host_threads()
    # a few files at a time, each file's strips on its share of the threads (lt_tiff_decode_strips
    # balances thousands of strips; one thread per file left half the workers idle in the last
    # round of a 30-file stack): two threads per file, eight files at once on 16 threads (the
    # c2-size job's parse 1.26 s against 1.36-1.38 with four threads per file and 1.29 with one,
    # profiles/r06_run43)
    n = max(1, min(K, total, max(1, total // 2)))
    if os.environ.get('LT_INGEST_FILES'):  # files decoded at once (A/B runs)
        n = max(1, min(K, total, int(os.environ['LT_INGEST_FILES'])))
    per_file = max(1, total // n)
    with ThreadPoolExecutor(n) as pool:
        dates = list(pool.map(one, range(K)))
    return dict(dates=dates, bands=out_bands, band_numbers=numbers, valid=valid, n_pix=P,
                ranges=ranges)


def stack_offset(stack, p0, p1):
    """Where grid points p0..p1 of an ingest_stack result sit in its gathered arrays (the last
    axis): they must lie inside one of the ranges it gathered."""
    for a, b, q0 in stack.get('ranges', [(0, stack['n_pix'], 0)]):
        if a <= p0 and p1 <= b:
            return q0 + p0 - a
    raise KeyError('grid points %d..%d were not gathered by this rank' % (p0, p1))


def stack_range(stack, p0, p1):
    """The (bands [K, nb, n], valid [K, n]) views of grid points p0..p1 of an ingest_stack
    result: they must lie inside one of the ranges it gathered."""
    q = stack_offset(stack, p0, p1)
    return stack['bands'][:, :, q:q + p1 - p0], stack['valid'][:, q:q + p1 - p0]
