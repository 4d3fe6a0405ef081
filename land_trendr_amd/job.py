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
                                      (tiles round-robin over the torchrun ranks, every output
                                      plane sent to rank 0);
  4. output   (output_reducer :128-152) raster.label_rasters / trendline_rasters placed by each
                                      grid point's template offsets, written as GeoTIFFs.

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

import numpy as np

from . import _abi
from .ingest import (analysis_rasters, grid_points, grid_offsets, ingest_stack, mask_name,
                     rast2grid, rast_local, read_grid)

IN_SETTINGS = '%s/input/settings.json'
IN_RASTS = '%s/input/rasters/'
OUT_GRID = '%s/output/pix_grid.csv'
OUT_RASTS = '%s/output/rasters/'


class LocalJob:
    def __init__(self, root, job, device=None, tile_pixels=1 << 22, trendline=True,
                 raster_mode='reference', pre_threshold_mode='reference', on_error='raise',
                 work_dir=None):
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
        self.grid_fn = os.path.join(root, OUT_GRID % job)
        self.out_dir = os.path.join(root, OUT_RASTS % job)

    def _path(self, key):
        return os.path.join(self.root, key)

    # 1. setup_mapper
    def setup(self):
        rdir = os.path.join(self.root, IN_RASTS % self.job)
        names = sorted(os.listdir(rdir)) if os.path.isdir(rdir) else []
        rasts = analysis_rasters(names)
        if not rasts:
            raise Exception('No analysis rasters specified for job %s' % self.job)
        os.makedirs(self.work_dir, exist_ok=True)
        self.rast_fns, self.mask_fns = [], []
        for n in rasts:
            self.rast_fns.append(rast_local(os.path.join(rdir, n), self.work_dir))
            m = mask_name(n)
            mp = os.path.join(rdir, m)
            # parse_mapper: a mask that cannot be fetched is ignored (:59-63)
            self.mask_fns.append(rast_local(mp, self.work_dir) if m != n and os.path.exists(mp)
                                 else None)
        os.makedirs(os.path.dirname(self.grid_fn), exist_ok=True)
        rast2grid(self.rast_fns[0], out_csv=self.grid_fn)
        with open(self.settings_path) as f:
            self.settings = json.load(f)
        return self.rast_fns

    # 2. parse_mapper
    def parse(self):
        from .index_eqn import parse_eqn_bands
        eqn_bands = sorted(parse_eqn_bands(self.settings['index_eqn']))
        self.stack = ingest_stack(self.rast_fns, self.grid_fn, self.mask_fns, bands=eqn_bands)
        return self.stack

    # 3. analysis_reducer, batched over pixel tiles: the mosaic path (runner.py) bench.py runs
    def analyze(self):
        """Tiles of the grid dealt round-robin over the torch.distributed ranks (one when not
        initialised), analysed by runner.MosaicRunner; every output plane goes to rank 0 (the
        writer) through the LabelExchange. Returns the host planes on rank 0, None elsewhere."""
        import torch
        from .distributed import Mosaic
        from .engine import LABELS, TRENDLINE, get_engine
        from .index_eqn import IndexProgram
        from .runner import MosaicRunner, TileInput
        from .scene import build_scene, parse_date
        from .settings import compile_params
        st = self.stack
        P = st['n_pix']
        dist, world, rank = None, 1, 0
        if torch.distributed.is_available() and torch.distributed.is_initialized():
            dist = torch.distributed
            world, rank = dist.get_world_size(), dist.get_rank()
        dev = torch.device('cuda', self.device if self.device is not None else
                           torch.cuda.current_device())
        fields = LABELS + ('status', 'n_years') + (TRENDLINE if self.trendline else ('winner',))
        self.scene = build_scene(st['dates'], parse_date(self.settings['target_date']))
        params, self.rules = compile_params(self.settings['line_cost'],
                                            self.settings.get('label_rules', ()),
                                            self.pre_threshold_mode)
        eng = get_engine(dev)
        numbers = list(st['band_numbers'])
        prog = IndexProgram(self.settings['index_eqn'], band_dtype=st['bands'].dtype,
                            raster_count=max(numbers))
        slots = [numbers.index(b) for b in prog.bands]  # the planes the equation reads
        fn = eng.compile_index(prog)
        m = Mosaic([P], self.tile_pixels, world, rank, 'round_robin')
        K = self.scene.n_obs
        items = []
        for t in m.mine:
            bands = torch.from_numpy(np.ascontiguousarray(
                st['bands'][:, slots, t.p0:t.p1])).to(dev)
            valid = torch.from_numpy(np.ascontiguousarray(st['valid'][:, t.p0:t.p1])).to(dev)
            vals = torch.empty((K, t.n), dtype=bands.dtype, device=dev)
            items.append(TileInput(t, self.scene, vals, valid, bands))
        runner = MosaicRunner(eng, m, params, items, fields, fn, dist, exchange_fields=fields)
        runner.step()
        torch.cuda.synchronize(dev)
        self._host = None
        if not runner.exchange.is_writer:
            self.dev_planes = None
            return None
        # the writer's planes stay in HBM: the output step assembles each raster there
        self.dev_planes = {f: runner.exchange.raster(f) for f in fields}
        self.engine = eng
        self._check_errors()
        return self.dev_planes

    @property
    def planes(self):
        """Host copies of the writer's output planes (made on first use)."""
        if self._host is None and self.dev_planes is not None:
            self._host = {f: t.cpu().numpy() for f, t in self.dev_planes.items()}
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
            wkt = read_grid(self.grid_fn)[p]
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
            if 'winner' in self.dev_planes:
                self.dev_planes['winner'][:, idx] = -1
            self._host = None

    # 4. output_reducer
    def output(self):
        """Every output key's raster, written as LZW GeoTIFF with the template's georeferencing.
        With one grid point per raster pixel (the co-registered grid setup builds) the rasters
        are assembled on the GPU (lt_raster_assemble) and each one reaches the host only as its
        finished GDT_Byte (or typed) array, written at once; a grid that maps two points to one
        pixel (the reference's loop: the last one wins) is assembled on the host."""
        import torch
        from .geotiff import GeoTiff
        from .raster import (label_rasters, label_rasters_device, output_reducer,
                             trendline_rasters, trendline_rasters_device)
        tmpl = GeoTiff(self.rast_fns[0])
        rows, cols = tmpl.height, tmpl.width
        lng, lat = grid_points(self.grid_fn)
        dest, ok = grid_offsets(tmpl.geotransform(), (rows, cols), lng, lat)
        if not ok.all():
            # data2raster assigns holder[y_off, x_off]: an off-template point raises there
            raise IndexError('grid point %s is off the template raster'
                             % read_grid(self.grid_fn)[int(np.flatnonzero(~ok)[0])])
        tdt = tmpl.dtype.newbyteorder('=')
        dp = self.dev_planes
        # an EMPTY pixel never reaches the reference's reducer: it emits nothing
        empty = (dp['status'] & _abi.LT_ST_EMPTY) != 0
        dp['matched'].masked_fill_(empty[None, :], 0)
        self._host = None
        names = [d.strftime('%Y-%m-%d') for d in self.scene.dates]
        if len(np.unique(dest)) == len(dest) and len(set(names)) == len(names):
            ddest = torch.from_numpy(np.ascontiguousarray(dest, np.int64)).to(dp['status'].device)
            out = {}

            def write(key, arr):  # each raster to its file as soon as it is on the host
                out.update(output_reducer({key: arr}, tmpl, self.root, self.job))

            for k, a in label_rasters_device(self.engine, dp, self.rules, (rows, cols), ddest,
                                             tdt, self.raster_mode).items():
                write(k, a)
            if self.trendline:
                trendline_rasters_device(self.engine, dp, self.scene, self.scene.dates,
                                         (rows, cols), ddest, tdt, self.raster_mode, sink=write)
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
        return dict(output_reducer(rasters, tmpl, self.root, self.job))

    def run(self):
        """Every rank runs setup/parse/analysis; the writer (rank 0) also writes the rasters.
        Returns {key: [path]} on the writer, None on the other ranks."""
        self.setup()
        self.parse()
        if self.analyze() is None:
            return None
        return self.output()


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
