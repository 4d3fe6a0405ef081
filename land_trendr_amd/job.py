"""Local job orchestration: MRLandTrendrJob.steps (mr_land_trendr_job.py:154-159)
without mrjob, EMR or S3, over a job directory laid out like the reference's S3 keys
(settings.py:19-25):

    <root>/<job>/input/settings.json             IN_SETTINGS
    <root>/<job>/input/rasters/<...ledaps...>    IN_RASTS (analysis rasters: .tif, .tif.tar.gz, .zip)
    <root>/<job>/input/rasters/<...cloudmask...> optional masks, same name with the trigger swapped
    <root>/<job>/output/pix_grid.csv             OUT_GRID
    <root>/<job>/output/rasters/<key>.tif        OUT_RAST_KEYNAME

Steps, as the reference chains them:
  1. setup    (setup_mapper :20-45)   analysis rasters by RAST_TRIGGER, grid from the first one;
  2. parse    (parse_mapper :47-81)   ingest.ingest_stack: band samples + mask validity per grid
                                      point (index_eqn runs on the GPU in step 3);
  3. analysis (analysis_reducer :83-126) the mosaic path of runner.py over pixel tiles on the GPU
                                      (tiles round-robin over the torchrun ranks; the label planes
                                      go to rank 0 over RCCL, the per-year trendline planes stream
                                      to host memory per tile — a file-backed map shared by the
                                      ranks when there are several — never to one GPU);
  4. output   (output_reducer :128-152) raster.label_rasters / trendline_rasters placed by each
                                      grid point's template offsets, written as GeoTIFFs.

Multi-rank jobs: rank 0 alone extracts the compressed rasters and writes the grid, then every rank
reads them (a barrier between), so no rank sees a partial extraction or a truncated grid.

Errors follow the reference: a pixel the reference's analysis raises for fails the job with the
same exception type (on_error='raise'); on_error='skip' leaves such pixels NODATA instead.
Grid points with no observation at all never reach the reference's reducer; they stay NODATA.

CLI: python -m land_trendr_amd.job --root DIR --job NAME [--tile-pixels N] [--no-trendline]
     (multi-GPU: torchrun --nproc-per-node N -m land_trendr_amd.job ...)
"""
import argparse
import json
import os
import sys
import time

import numpy as np

from . import _abi
from .geotiff import GeoTiff
from .ingest import (analysis_rasters, grid_axes, grid_coords, grid_offsets, ingest_stack,
                     mask_name, rast2grid, rast_local, read_grid, stack_offset, stack_range)

IN_SETTINGS = '%s/input/settings.json'
IN_RASTS = '%s/input/rasters/'
OUT_GRID = '%s/output/pix_grid.csv'
OUT_RASTS = '%s/output/rasters/'


class LocalJob:
    def __init__(self, root, job, device=None, tile_pixels=1 << 22, trendline=True,
                 raster_mode='reference', pre_threshold_mode='reference', on_error='raise',
                 work_dir=None, engine=None):
        """engine: the analysis engine (default: engine.get_engine of `device`, the HIP library);
        tests pass a CPU double (tests/engine_double.py) to run the multi-rank path over gloo."""
        if on_error not in ('raise', 'skip'):
            raise ValueError('on_error must be "raise" or "skip"')
        self.root, self.job, self.device = root, job, device
        self.tile_pixels = int(tile_pixels)
        self.trendline = trendline
        self.raster_mode = raster_mode
        self.pre_threshold_mode = pre_threshold_mode
        self.on_error = on_error
        self.work_dir = work_dir or os.path.join(root, job, 'work')
        self.settings_path = os.path.join(root, IN_SETTINGS % job)
        self._grid_fn = os.path.join(root, OUT_GRID % job)
        self._grid_writer = None  # (thread, [exception]) writing the grid CSV beside parse()
        self.out_dir = os.path.join(root, OUT_RASTS % job)
        self.engine = engine
        self._host = None
        self.host_trendline = None
        self._order = None       # grid point of each internal pixel (None: grid order)
        self._raster_hw = None   # (rows, cols) of the raster order, or None
        self.raster_grid = None  # (geotransform, rows, cols) of the raster order, or None

    @property
    def grid_fn(self):
        """The grid CSV (the reference's grid file): complete once this returns (a one-rank
        job's setup writes it on a thread of its own while parse runs)."""
        self._join_grid()
        return self._grid_fn

    def _join_grid(self):
        w, self._grid_writer = self._grid_writer, None
        if w is not None:
            w[0].join()
            if w[1]:
                raise w[1][0]

    @property
    def order(self):
        """Grid point of each internal pixel (raster order), None in grid order: pixel (row r,
        column c) is grid point c * rows + r, made on first use (49 M entries at c2 size)."""
        if self._order is None and self._raster_hw is not None:
            H, W = self._raster_hw
            self._order = ((np.arange(W, dtype=np.int64) * H)[None, :] +
                           np.arange(H, dtype=np.int64)[:, None]).ravel()
        return self._order

    def _path(self, key):
        return os.path.join(self.root, key)

    @staticmethod
    def _dist():
        """(torch.distributed or None, world size, rank)."""
        try:
            import torch.distributed as dist
            if dist.is_available() and dist.is_initialized():
                return dist, dist.get_world_size(), dist.get_rank()
        except ImportError:
            pass
        return None, 1, 0

    # 1. setup_mapper
    def setup(self):
        """Rank 0 extracts the rasters into work_dir and writes the grid (a temporary file moved
        into place); the other ranks wait for it, then list the same files."""
        rdir = os.path.join(self.root, IN_RASTS % self.job)
        names = sorted(os.listdir(rdir)) if os.path.isdir(rdir) else []
        rasts = analysis_rasters(names)
        if not rasts:
            raise Exception('No analysis rasters specified for job %s' % self.job)
        dist, _, rank = self._dist()
        if rank == 0:
            self._locate(rdir, rasts)
            os.makedirs(os.path.dirname(self._grid_fn), exist_ok=True)
            tmp = '%s.tmp%d' % (self._grid_fn, os.getpid())

            def write_grid(err):
                try:
                    rast2grid(self.rast_fns[0], out_csv=tmp)
                    os.replace(tmp, self._grid_fn)
                except BaseException as e:  # re-raised by the first grid_fn access
                    err.append(e)
            self._join_grid()
            err = []
            if dist is None:  # one rank: no other process waits for the file
                import threading
                th = threading.Thread(target=write_grid, args=(err,), daemon=True)
                th.start()
                self._grid_writer = (th, err)
            else:
                write_grid(err)
                if err:
                    raise err[0]
        if dist is not None:
            dist.barrier()
        if rank != 0:
            self._locate(rdir, rasts)  # every archive is extracted by now: only listed
        # the grid's point coordinates, as parsing the CSV being written gives them (raster
        # order: made from the template's axes)
        self._internal_order()
        if self._raster_hw is None:
            self.grid_xy = grid_coords(self.rast_fns[0])
        with open(self.settings_path) as f:
            self.settings = json.load(f)
        return self.rast_fns

    def _internal_order(self):
        """The job's own pixel order. rast2grid lists the template's pixels column by column
        (utils.py:314-321) while a raster is stored row by row, so gathering every raster at the
        grid points in grid order is a transpose of each band (a random-access gather of 49 M
        samples per band and date). Pixels are independent and the outputs are placed by each
        point's raster offset, so when every grid point lands on its own template pixel (the
        co-registered grid setup() builds from the template) the job runs them in raster order
        instead: internal pixel q is raster pixel q and grid point order[q], and a raster with the
        template's georeferencing is read by slicing (ingest_stack raster_grid). The check is
        pt2val's addressing (grid_offsets' operations) on the grid's distinct coordinates: the
        offsets of a column's points depend on its x alone, a row's on its y. The grid CSV keeps
        the reference's order; grid_wkts() gives the WKTs in the internal order."""
        self._order = self._raster_hw = None
        self.raster_grid = None
        tmpl = GeoTiff(self.rast_fns[0])
        H, W = tmpl.height, tmpl.width
        gt = tmpl.geotransform()
        xv, yv = grid_axes(tmpl)
        xo = np.trunc((xv - gt[0]) * 1.0 / gt[1])
        yo = np.trunc((yv - gt[3]) * 1.0 / gt[5])
        if not (np.array_equal(xo, np.arange(W)) and np.array_equal(yo, np.arange(H))):
            return  # some point not on its own pixel: grid order, offsets per point
        self._raster_hw = (H, W)  # self.order: pixel (row r, column c) is grid point c * H + r
        self.grid_xy = (np.tile(xv, H), np.repeat(yv, W))
        self.raster_grid = (gt, H, W)

    def grid_wkts(self):
        """The grid points' WKTs in the job's internal pixel order (that of the stack and of
        every plane): the grid CSV's order unless _internal_order() chose raster order."""
        w = read_grid(self.grid_fn)
        return w if self.order is None else [w[i] for i in self.order]

    def _locate(self, rdir, rasts):
        os.makedirs(self.work_dir, exist_ok=True)
        self.rast_fns, self.mask_fns = [], []
        for n in rasts:
            self.rast_fns.append(rast_local(os.path.join(rdir, n), self.work_dir))
            m = mask_name(n)
            mp = os.path.join(rdir, m)
            # parse_mapper: a mask that cannot be fetched is ignored (:59-63)
            self.mask_fns.append(rast_local(mp, self.work_dir) if m != n and os.path.exists(mp)
                                 else None)

    # 2. parse_mapper
    def parse(self):
        """Band samples and mask validity of the grid points of this rank's tiles only (the tiles
        of the grid dealt round-robin over the ranks, as analyze runs them): a rank's host planes
        and gathers are 1/N of the job's."""
        from .distributed import Mosaic
        from .index_eqn import parse_eqn_bands
        _, world, rank = self._dist()
        P = len(self.grid_xy[0])
        self.mosaic = Mosaic([P], self.tile_pixels, world, rank, 'round_robin')
        eqn_bands = sorted(parse_eqn_bands(self.settings['index_eqn']))
        # on a GPU (LT_JOB_UPLOAD=whole), each raster's planes cross to the device as soon as they
        # are decoded, on the worker that decoded them, while the other rasters decode: analyze()
        # then starts from the device stack
        self._dev_stack = None
        up = self._stack_uploader(len(self.rast_fns), len(eqn_bands),
                                  sum(t.n for t in self.mosaic.mine))
        self.stack = ingest_stack(self.rast_fns, self.grid_xy, self.mask_fns, bands=eqn_bands,
                                  pixels=[(t.p0, t.p1) for t in self.mosaic.mine],
                                  raster_grid=self.raster_grid, on_raster=up)
        if up is not None and up.bands is not None:
            import torch
            torch.cuda.synchronize(up.device)
            self._dev_stack = (up.bands, up.valid)
        return self.stack

    def _stack_uploader(self, K, nb, Q):
        """The per-raster H2D of parse() (None when the job does not run on a GPU, or
        LT_JOB_UPLOAD is not 'whole')."""
        import threading
        import torch
        if os.environ.get('LT_JOB_UPLOAD', 'whole') != 'whole' or not torch.cuda.is_available():
            return None
        if self.engine is not None and torch.device(self.engine.device).type != 'cuda':
            return None
        dev = torch.device('cuda', self.device if self.device is not None
                           else torch.cuda.current_device())

        class Up:
            def __init__(self):
                self.device, self.bands, self.valid = dev, None, None
                self.lock = threading.Lock()

            def __call__(self, k, b, v):
                with self.lock:  # the device stack made by the first raster (its sample type)
                    if self.bands is None:
                        self.bands = torch.empty((K, nb, Q), dtype=torch.from_numpy(b[:0]).dtype,
                                                 device=dev)
                        self.valid = torch.empty((K, Q), dtype=torch.uint8, device=dev)
                with torch.cuda.device(dev):
                    self.bands[k].copy_(torch.from_numpy(b))
                    self.valid[k].copy_(torch.from_numpy(v))
        return Up()

    # 3. analysis_reducer, batched over pixel tiles: the mosaic path (runner.py) bench.py runs
    def analyze(self):
        """Tiles of the grid dealt round-robin over the torch.distributed ranks (one when not
        initialised), analysed by runner.MosaicRunner. The label planes (and status / n_years) go
        to rank 0, the writer, through the LabelExchange; the per-year trendline planes leave the
        GPU per tile, while the next tile computes, into host planes [Y, P] (file-backed maps in
        work_dir, shared by the ranks, when there are several), from a ring of three tiles'
        device buffers: no GPU ever holds more than three tiles of trendline. Returns the
        writer's label planes (device), None on the other ranks."""
        import torch
        from .distributed import TrendlineStream
        from .engine import _DTYPE, LABELS, TRENDLINE, get_engine, pack_valid_bits
        from .index_eqn import IndexProgram
        from .runner import MosaicRunner, TileInput
        from .scene import build_scene, parse_date
        from .settings import compile_params
        st = self.stack
        P = st['n_pix']
        dist, world, rank = self._dist()
        if self.engine is None:
            self.engine = get_engine(self.device if self.device is not None else
                                     torch.cuda.current_device())
        eng = self.engine
        dev = torch.device(eng.device)
        cuda = dev.type == 'cuda'
        label_fields = LABELS + ('status', 'n_years')
        tl_fields = TRENDLINE if self.trendline else ('winner',)
        self.scene = build_scene(st['dates'], parse_date(self.settings['target_date']))
        params, self.rules = compile_params(self.settings['line_cost'],
                                            self.settings.get('label_rules', ()),
                                            self.pre_threshold_mode)
        numbers = list(st['band_numbers'])
        prog = IndexProgram(self.settings['index_eqn'], band_dtype=st['bands'].dtype,
                            raster_count=max(numbers))
        slots = [numbers.index(b) for b in prog.bands]  # the planes the equation reads
        fn = eng.compile_index(prog)
        m = self.mosaic
        if (m.world, m.rank, m.scene_pixels) != (world, rank, [P]):
            raise RuntimeError('parse() ran under another process group')
        K, Y = self.scene.n_obs, self.scene.n_years
        t_in = time.perf_counter()
        # LT_JOB_UPLOAD 'whole' (default on a GPU): the rank's gathered stack (its tiles' pixel
        # ranges) crosses to the device in one copy per array and each tile's inputs are made from
        # device views of it; 'tile': each tile's bands gathered into a host copy first (a 2 GB
        # single-threaded copy per 16.8 Mpx tile, most of round 6's job analysis time)
        whole = (cuda and os.environ.get('LT_JOB_UPLOAD', 'whole') == 'whole' and
                 st['bands'].flags.c_contiguous and st['valid'].flags.c_contiguous and
                 st['bands'].nbytes + st['valid'].nbytes <= (64 << 30))
        if whole:
            ds = getattr(self, '_dev_stack', None)
            if ds is not None and ds[0].device == dev and ds[0].shape == st['bands'].shape:
                w_bands, w_valid = ds  # uploaded raster by raster during parse()
            else:
                w_bands = torch.from_numpy(st['bands']).to(dev)
                w_valid = torch.from_numpy(st['valid']).to(dev)
            self._dev_stack = None
            if slots != list(range(st['bands'].shape[1])):
                w_bands = w_bands[:, slots]
        items = []
        for t in m.mine:
            if whole:
                q = stack_offset(st, t.p0, t.p1)
                bands = w_bands[:, :, q:q + t.n]
                valid = w_valid[:, q:q + t.n]
            else:
                t_bands, t_valid = stack_range(st, t.p0, t.p1)
                bands = torch.from_numpy(np.ascontiguousarray(t_bands[:, slots])).to(dev)
                valid = torch.from_numpy(np.ascontiguousarray(t_valid)).to(dev)
            if cuda and fn.lin is not None and len(slots) == 2 and bands.dtype == torch.int16:
                # the fused load stage reads a pixel's two int16 bands as one 32-bit word
                inter = torch.empty((K, t.n, 2), dtype=bands.dtype, device=dev).permute(0, 2, 1)
                inter.copy_(bands)
                bands = inter
            elif whole:
                bands = bands.contiguous()
            if whole:
                valid = valid.contiguous()
            if cuda:  # the winner pick reads the mask as bit planes (one word per 32 obs)
                valid = pack_valid_bits(valid)
            # the index raster: allocated by the runner only if the load kernel writes it (the
            # fused load stage never does)
            items.append(TileInput(t, self.scene, None, valid, bands))
        if whole:
            del w_bands, w_valid  # every tile holds its own copies
        if cuda:
            torch.cuda.synchronize(dev)
        self.analyze_s = {'inputs': time.perf_counter() - t_in}
        host = self.host_trendline = self._trendline_planes(tl_fields, Y, P, dist, world, rank)
        # the trendline planes: a ring of three tiles' buffers on the GPU (tile k reuses tile
        # k-3's once its rows have reached the host), so a rank's HBM never holds all its tiles'
        # trendlines
        # LT_JOB_JIT: 'off' (default) — the precompiled kernels (a linear index_eqn fused into
        # them, any other through the load kernel): a scene's analysis is ~1 % of a job's time
        # (tools/job_bench.py: 49 Mpx in ~20 ms of kernels against seconds of decode and IO),
        # while a hiprtc compile takes ~10 s of host time and, left running on its worker thread
        # past the analysis, slowed the output step 13x (profiles/r06_run6d); 'async' — the module
        # compiles on a worker thread while the first tiles run precompiled (same results);
        # 'sync' — compile first (a disk-cached module loads at once)
        jit_mode = os.environ.get('LT_JOB_JIT', 'sync' if os.environ.get('LT_JOB_JIT_SYNC') == '1'
                                  else 'off')
        runner = MosaicRunner(eng, m, params, items, label_fields + tl_fields, fn, dist,
                              exchange_fields=label_fields, ring=3 if cuda else 0,
                              jit=jit_mode != 'off')
        jit_async = cuda and runner.jit is not None and jit_mode == 'async'
        if jit_async:
            eng.set_jit_mode(True)
            runner.prepare_jit(wait=False)

        # a completed year row of tile t, copied from its pinned ring buffer into the host plane
        # in pieces on a pool of host threads (numpy releases the GIL for the copy): one thread
        # copied ~10 GB/s, the bound of a trendline job's analysis (profiles/r06_run33); the ring
        # buffer is reused only after sink() returns
        from concurrent.futures import ThreadPoolExecutor
        from .ingest import host_threads
        n_cp = max(1, min(8, host_threads()))
        pool = ThreadPoolExecutor(n_cp) if cuda and n_cp > 1 else None

        def sink(f, row, view, t):  # one completed year row of tile t
            src = view.numpy().view(host[f].dtype)
            dst = host[f][row, t.p0:t.p1]
            n = src.shape[0]
            if pool is None or n < (1 << 20):
                dst[...] = src
                return
            step = -(-n // n_cp)

            def piece(a):
                dst[a:a + step] = src[a:a + step]
            list(pool.map(piece, range(0, n, step)))

        # the ring's rows sized for the widest plane streamed (the labels-only job's winner rows
        # are 4 bytes a pixel: half the pinned memory to allocate)
        row_b = max(torch.empty(0, dtype=_DTYPE[f]).element_size() for f in tl_fields)
        tls = TrendlineStream(m.tile * row_b, dev, depth=16, sink=sink) if cuda else None
        copied = {}  # tile -> event after its rows' D2H copies

        def push(k):
            t = items[k].tile
            copied[k] = tls.push({f: runner.outs[k][f] for f in tl_fields}, t.n, t)

        # tile k-1's rows are queued behind tile k's kernels, so the copies overlap them
        t_st = time.perf_counter()
        try:
            runner.step(after_tile=(lambda k: push(k - 1) if k > 0 else None) if cuda else None,
                        slab_free=copied.get if cuda else None)
        finally:
            # the engine is cached per device (get_engine): a failed step must not leave later
            # jobs of this process in async-JIT mode
            if jit_async:
                eng.set_jit_mode(False)
        if jit_async:
            self.jit_stats = eng.jit_stats()
        if cuda:
            if items:
                push(len(items) - 1)
            torch.cuda.synchronize(dev)
            self.analyze_s['steps'] = time.perf_counter() - t_st
            t_dr = time.perf_counter()
            tls.drain()
            self.analyze_s['drain'] = time.perf_counter() - t_dr
        if pool is not None:
            pool.shutdown()
        else:  # a CPU engine (tests): its planes are host tensors already
            for o, it in zip(runner.outs, items):
                for f in tl_fields:
                    host[f][:, it.tile.p0:it.tile.p1] = o[f][:, :it.tile.n].numpy()
        for a in host.values():
            if isinstance(a, np.memmap):
                a.flush()
        if dist is not None:
            dist.barrier()  # every rank's trendline rows are in the shared maps
        self._host = None
        if not runner.exchange.is_writer:
            self.dev_planes = None
            return None
        # the writer's label planes stay on the device: the output step assembles each raster
        self.dev_planes = {f: runner.exchange.raster(f) for f in label_fields}
        del runner
        self._check_errors()
        return self.dev_planes

    def _trendline_planes(self, fields, Y, P, dist, world, rank):
        """Host [Y, P] planes the trendline rows stream into: in memory for one rank, else
        file-backed maps in work_dir that rank 0 creates and every rank fills with its tiles."""
        from .engine import _DTYPE
        np_dt = {f: np.dtype(str(_DTYPE[f]).replace('torch.', '')) for f in fields}
        if world == 1:
            return {f: np.empty((Y, P), np_dt[f]) for f in fields}
        d = os.path.join(self.work_dir, 'trendline')
        path = {f: os.path.join(d, f + '.bin') for f in fields}
        if rank == 0:
            os.makedirs(d, exist_ok=True)
            for f in fields:
                np.memmap(path[f], np_dt[f], 'w+', shape=(Y, P)).flush()
        dist.barrier()
        return {f: np.memmap(path[f], np_dt[f], 'r+', shape=(Y, P)) for f in fields}

    @property
    def planes(self):
        """Host copies of the writer's output planes (made on first use): the label planes and
        the trendline planes."""
        if self._host is None and self.dev_planes is not None:
            self._host = {f: t.cpu().numpy() for f, t in self.dev_planes.items()}
            self._host.update({f: np.asarray(a) for f, a in self.host_trendline.items()})
        return self._host

    def _check_errors(self):
        import torch
        from .utils import _raise_for_status
        status = self.dev_planes['status'].cpu().numpy()
        bad = np.flatnonzero(status & ~_abi.LT_ST_EMPTY)
        if len(bad) == 0:
            return
        if self.on_error == 'raise':
            p = int(bad[0])
            wkt = self.grid_wkts()[p]
            s = int(status[p])
            if s & _abi.LT_ST_PRE_THRESHOLD_ATTR:
                raise AttributeError("LabelRule instance has no attribute 'threshold' (pixel %s)"
                                     % wkt)
            try:
                _raise_for_status(s, None)
            except Exception as e:
                raise type(e)('%s (pixel %s)' % (e, wkt)) from e
        else:  # skip: the failing pixels emit nothing
            idx = torch.from_numpy(bad).to(self.dev_planes['matched'].device)
            self.dev_planes['matched'][:, idx] = 0
            self.host_trendline['winner'][:, bad] = -1  # no trendline key either
            self._host = None

    # 4. output_reducer
    def output(self):
        """Every output key's raster, written as LZW GeoTIFF with the template's georeferencing.
        With one grid point per raster pixel (the co-registered grid setup builds) the rasters
        are assembled on the GPU (lt_raster_assemble) and each one reaches the host only as its
        finished GDT_Byte (or typed) array, written at once; a grid that maps two points to one
        pixel (the reference's loop: the last one wins) is assembled on the host."""
        import torch
        from .raster import (label_rasters, label_rasters_device, output_reducer,
                             trendline_rasters, trendline_rasters_device)
        tmpl = GeoTiff(self.rast_fns[0])
        rows, cols = tmpl.height, tmpl.width
        lng, lat = self.grid_xy
        if self._raster_hw is not None:  # raster order: internal pixel q is template pixel q
            dest, ok = np.arange(rows * cols, dtype=np.int64), np.ones(rows * cols, bool)
        else:
            dest, ok = grid_offsets(tmpl.geotransform(), (rows, cols), lng, lat)
        if not ok.all():
            # data2raster assigns holder[y_off, x_off]: an off-template point raises there
            raise IndexError('grid point %s is off the template raster'
                             % self.grid_wkts()[int(np.flatnonzero(~ok)[0])])
        tdt = tmpl.dtype.newbyteorder('=')
        dp = self.dev_planes
        # an EMPTY pixel never reaches the reference's reducer: it emits nothing
        empty = (dp['status'] & _abi.LT_ST_EMPTY) != 0
        dp['matched'].masked_fill_(empty[None, :], 0)
        self._host = None
        names = [d.strftime('%Y-%m-%d') for d in self.scene.dates]
        cuda = torch.device(self.engine.device).type == 'cuda'
        distinct = self._raster_hw is not None or np.bincount(dest, minlength=rows * cols).max() <= 1
        if cuda and distinct and len(set(names)) == len(names):
            ddest = torch.from_numpy(np.ascontiguousarray(dest, np.int64)).to(dp['status'].device)
            out = {}
            # each raster is encoded and written on a writer thread (its LZW strips on the native
            # pool) while the next one is assembled on the GPU and copied back: at most three in
            # flight; written in key order, the first error re-raised
            from collections import deque
            from concurrent.futures import ThreadPoolExecutor
            writer = ThreadPoolExecutor(1)
            inflight = deque()

            def settle(keep):
                while len(inflight) > keep:
                    out.update(inflight.popleft().result())

            def write(key, arr):  # each raster to its file as soon as it is on the host
                inflight.append(writer.submit(
                    lambda r: dict(output_reducer(r, tmpl, self.root, self.job)), {key: arr}))
                settle(2)

            try:
                for k, a in label_rasters_device(self.engine, dp, self.rules, (rows, cols), ddest,
                                                 tdt, self.raster_mode).items():
                    write(k, a)
                if self.trendline:
                    rows_dev = _DeviceRows(self.host_trendline, dp['status'].device)
                    trendline_rasters_device(self.engine, rows_dev, self.scene, self.scene.dates,
                                             (rows, cols), ddest, tdt, self.raster_mode,
                                             sink=write)
                settle(0)
            finally:
                writer.shutdown(wait=True)
            self._join_grid()  # the grid CSV, the job's other output, in place too
            return out
        n = rows * cols
        placed = {}
        for k, a in self.planes.items():
            fill = -1 if k == 'winner' else 0
            b = np.full(a.shape[:-1] + (n,), fill, a.dtype)
            b[..., dest] = a  # repeated offsets: the last grid point wins, as in the loop
            placed[k] = b
        rasters = label_rasters(placed, self.rules, (rows, cols), tdt, self.raster_mode)
        if self.trendline:
            rasters.update(trendline_rasters(placed, self.scene, self.scene.dates, (rows, cols),
                                             tdt, self.raster_mode))
        res = dict(output_reducer(rasters, tmpl, self.root, self.job))
        self._join_grid()
        return res

    def run(self):
        """Every rank runs setup/parse/analysis; the writer (rank 0) also writes the rasters.
        Returns {key: [path]} on the writer, None on the other ranks."""
        self.setup()
        self.parse()
        if self.analyze() is None:
            self._join_grid()
            return None
        out = self.output()
        self._join_grid()
        return out


class _DeviceRows:
    """The host trendline planes as raster.trendline_rasters_device reads them: 'winner' whole on
    the device (it selects the pixels of every key), every other plane one year row at a time,
    uploaded into a buffer of its own when the row is asked for (the rows of one date's rasters
    are assembled together, then the next date's rows overwrite them in stream order)."""

    def __init__(self, host, device):
        import torch
        self.host, self.device = host, device
        self.winner = torch.from_numpy(np.ascontiguousarray(host['winner'])).to(device)
        self.buf = {}

    def __getitem__(self, field):
        if field == 'winner':
            return self.winner
        return _Rows(self, field)


class _Rows:
    def __init__(self, owner, field):
        self.owner, self.field = owner, field

    def __getitem__(self, y):
        import torch
        o = self.owner
        row = torch.from_numpy(np.ascontiguousarray(o.host[self.field][y]))
        b = o.buf.get(self.field)
        if b is None:
            b = o.buf[self.field] = torch.empty(row.shape, dtype=row.dtype, device=o.device)
        b.copy_(row)
        return b


def main(argv=None):
    ap = argparse.ArgumentParser(description='LandTrendr job on the local GPU (steps of '
                                 'MRLandTrendrJob without mrjob/S3)')
    ap.add_argument('--root', required=True, help='directory holding <job>/input/...')
    ap.add_argument('--job', required=True)
    ap.add_argument('--device', type=int, default=None)
    ap.add_argument('--tile-pixels', type=int, default=1 << 22)
    ap.add_argument('--no-trendline', action='store_true')
    ap.add_argument('--raster-mode', choices=('reference', 'typed'), default='reference')
    ap.add_argument('--pre-threshold-mode', choices=('reference', 'documented'),
                    default='reference')
    ap.add_argument('--on-error', choices=('raise', 'skip'), default='raise')
    a = ap.parse_args(argv)
    dist = None
    if int(os.environ.get('WORLD_SIZE', '1')) > 1:
        import torch
        import torch.distributed as dist
        local = int(os.environ.get('LOCAL_RANK', '0'))
        torch.cuda.set_device(local)
        dist.init_process_group('nccl', device_id=torch.device('cuda', local))
        if a.device is None:
            a.device = local
    j = LocalJob(a.root, a.job, a.device, a.tile_pixels, not a.no_trendline, a.raster_mode,
                 a.pre_threshold_mode, a.on_error)
    res = j.run()
    for key in sorted(res or {}):
        print('%s\t%s' % (key, res[key][0]))
    if dist is not None:
        dist.destroy_process_group()
    return 0


if __name__ == '__main__':
    sys.exit(main())
