"""Tile engine: torch device tensors in, lt_analyze_tile (HIP) on the current stream, tensors out.

One Engine per GPU (per process). torch provides device memory and the stream only; all compute
happens in land_trendr_amd/liblt_hip.so. There is no CPU path.
"""
import ctypes

import torch

from . import _abi

TRENDLINE = tuple(f for f, _ in _abi.YEAR_FIELDS)
LABELS = tuple(f for f, _ in _abi.RULE_FIELDS)
ALL_FIELDS = TRENDLINE + LABELS + ('status', 'n_years')
LABEL_FIELDS = ('status', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude')

_DT = {'int16': torch.int16, 'int32': torch.int32, 'uint8': torch.uint8,
       'float64': torch.float64}
# raster element types a tile may carry (index rasters, band planes): torch dtype -> LT_T_*
_LT_T = {torch.float64: _abi.LT_T_F64, torch.int16: _abi.LT_T_I16, torch.uint16: _abi.LT_T_U16,
         torch.int32: _abi.LT_T_I32, torch.float32: _abi.LT_T_F32, torch.uint8: _abi.LT_T_U8,
         torch.uint32: _abi.LT_T_U32, torch.int8: _abi.LT_T_I8, torch.int64: _abi.LT_T_I64}
_TORCH_OF_LT = {v: k for k, v in _LT_T.items()}
_SHAPE_KIND = {**{f: 'year' for f, _ in _abi.YEAR_FIELDS},
               **{f: 'rule' for f, _ in _abi.RULE_FIELDS},
               **{f: 'pix' for f, _ in _abi.PIX_FIELDS}}
_DTYPE = {f: _DT[d] for f, d in _abi.YEAR_FIELDS + _abi.RULE_FIELDS + _abi.PIX_FIELDS}


class LtError(RuntimeError):
    pass


class Engine:
    def __init__(self, device=None):
        if not torch.cuda.is_available():
            raise LtError('land_trendr_amd needs a HIP device (no CPU fallback)')
        self.lib = _abi.load_lib()
        self.device = torch.device('cuda', torch.cuda.current_device() if device is None
                                   else int(device))
        ctx = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            rc = self.lib.lt_ctx_create(self.device.index, ctypes.byref(ctx))
        if rc != 0:
            raise LtError('lt_ctx_create failed (%d)' % rc)
        self.ctx = ctx

    def close(self):
        if self.ctx:
            self.lib.lt_ctx_destroy(self.ctx)
            self.ctx = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc, what):
        if rc != 0:
            raise LtError('%s failed (%d): %s' % (what, rc,
                                                  self.lib.lt_last_error(self.ctx).decode()))

    def alloc_outputs(self, n_years, n_rules, n_pix, fields=ALL_FIELDS):
        out = {}
        for f in fields:
            kind = _SHAPE_KIND[f]
            shape = {'year': (n_years, n_pix), 'rule': (max(n_rules, 1), n_pix),
                     'pix': (n_pix,)}[kind]
            out[f] = torch.empty(shape, dtype=_DTYPE[f], device=self.device)
        return out

    def analyze_tile(self, scene, params, values, valid=None, fields=ALL_FIELDS, out=None,
                     stream=None, lin=None, index=None):
        """values: [K, P] observation values — float64, or an index raster in its stored type
        (int16, uint16, int32, float32, uint8, ...: what index_tile writes) — valid: uint8 [K, P]
        or None. With lin (an IndexFn's linear form, fn.lin): values are the [K, NB, P] band
        planes and the kernel evaluates the index of each winner itself (the fused load stage).
        With index (an IndexFn of any program): the same, with the program inlined into JIT
        analyze / resolve kernels (lt_jit.h; compiled on first use, cached).
        Returns the dict of output tensors ([Y, P], [R, P], [P]); asynchronous on `stream`."""
        tin, tout, out = self._tile_structs(scene, params, values, valid, fields, out, lin, index)
        sc = scene.to_c()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        rc = self.lib.lt_analyze_tile(self.ctx, ctypes.byref(sc), ctypes.byref(params),
                                      ctypes.byref(tin), ctypes.byref(tout),
                                      ctypes.c_void_p(st.cuda_stream))
        self._check(rc, 'lt_analyze_tile')
        return out

    def analyze_tiles(self, scene, params, tiles, fields=ALL_FIELDS, outs=None, stream=None,
                      ready=None, lin=None, index=None, done=None, join=True):
        """analyze_tile over a list of (values, valid) tiles of one scene in one call
        (lt_analyze_tiles: tile t's resolve stage overlaps tile t+1's analyze stage). ready: None
        or one recorded torch.cuda.Event (or None) per tile, which that tile's analyze kernel
        waits on (lt_analyze_tiles_after: the load stage of later tiles may still be running on
        another stream). lin / index: as analyze_tile (every tile's values are then band planes).
        done: None or one torch.cuda.Event (or None) per tile, recorded once every output of that
        tile is complete; join=False: `stream` does not wait for the tiles' last stages
        (lt_analyze_tiles_ev: the caller orders later work on the done events).
        Returns the list of output dicts; asynchronous on `stream`."""
        n = len(tiles)
        tins = (_abi.LtTileIn * max(n, 1))()
        touts = (_abi.LtTileOut * max(n, 1))()
        res = []
        for t, (values, valid) in enumerate(tiles):
            tin, tout, o = self._tile_structs(scene, params, values, valid, fields,
                                              outs[t] if outs is not None else None, lin, index)
            tins[t] = tin
            touts[t] = tout
            res.append(o)
        sc = scene.to_c()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        if done is not None or not join:
            if done is not None and len(done) != n:
                raise LtError('done needs one event (or None) per tile')
            if ready is not None and len(ready) != n:
                raise LtError('ready needs one event (or None) per tile')
            evr = (ctypes.c_void_p * max(n, 1))(
                *[e.cuda_event if e is not None else None for e in (ready or [None] * n)])
            evd = (ctypes.c_void_p * max(n, 1))(
                *[e.cuda_event if e is not None else None for e in (done or [None] * n)])
            rc = self.lib.lt_analyze_tiles_ev(self.ctx, ctypes.byref(sc), ctypes.byref(params), n,
                                              tins, touts, evr, evd, 1 if join else 0,
                                              ctypes.c_void_p(st.cuda_stream))
        elif ready is None:
            rc = self.lib.lt_analyze_tiles(self.ctx, ctypes.byref(sc), ctypes.byref(params), n,
                                           tins, touts, ctypes.c_void_p(st.cuda_stream))
        else:
            if len(ready) != n:
                raise LtError('ready needs one event (or None) per tile')
            evs = (ctypes.c_void_p * max(n, 1))(
                *[e.cuda_event if e is not None else None for e in ready])
            rc = self.lib.lt_analyze_tiles_after(self.ctx, ctypes.byref(sc), ctypes.byref(params),
                                                 n, tins, touts, evs,
                                                 ctypes.c_void_p(st.cuda_stream))
        self._check(rc, 'lt_analyze_tiles')
        return res

    def _tile_structs(self, scene, params, values, valid, fields, out, lin=None, index=None):
        if index is not None:  # any program, JIT kernels: its band type and band count
            nb = len(index.program.bands)
            want = _TORCH_OF_LT[_LT_T_OF_NP(index.program.band_dtype)]
        elif lin is not None:
            nb, want = lin.n_bands, _TORCH_OF_LT.get(lin.band_type)
        if lin is not None or index is not None:  # the fused load stage: [K, NB, P] band planes
            planar = values.dim() == 3 and values.stride(2) == 1
            inter = values.dim() == 3 and values.stride(1) == 1 and values.stride(2) == nb
            if (values.dtype != want or values.device != self.device or values.dim() != 3 or
                    values.shape[1] != nb or not (planar or inter)):
                raise LtError('bands must be a %s [K, %d, P] tensor on %s, planar (unit pixel '
                              'stride) or pixel-interleaved (unit band stride)'
                              % (want, nb, self.device))
            K, _, P = values.shape
        else:
            if values.dtype not in _LT_T or values.device != self.device or values.dim() != 2:
                raise LtError('values must be a [K, P] raster tensor on %s' % self.device)
            if values.stride(1) != 1:
                raise LtError('values must have unit pixel stride')
            K, P = values.shape
        if K != scene.n_obs:
            raise LtError('values has %d obs rows, scene has %d' % (K, scene.n_obs))
        if valid is not None and valid.dtype == torch.int32:  # mask bit planes
            W = (K + 31) // 32
            if (tuple(valid.shape) != (W, P) or valid.stride(1) != 1 or
                    valid.device != self.device):
                raise LtError('valid bit planes must be an int32 [%d, P] tensor with unit pixel '
                              'stride' % W)
            if lin is None and index is None and W > 1 and valid.stride(0) != values.stride(0):
                raise LtError('valid bit planes must share the row stride of values')
        elif valid is not None:
            if lin is not None or index is not None:
                if (valid.dtype != torch.uint8 or tuple(valid.shape) != (K, P) or
                        valid.stride(1) != 1 or valid.device != self.device):
                    raise LtError('valid must be a uint8 [K, P] tensor with unit pixel stride')
            elif (valid.dtype != torch.uint8 or valid.shape != values.shape or
                    valid.stride() != values.stride() or valid.device != self.device):
                raise LtError('valid must be uint8 with the shape/strides of values')
        if out is None:
            out = self.alloc_outputs(scene.n_years, params.n_rules, P, fields)
        ostride = None
        for f, t in out.items():
            kind = _SHAPE_KIND[f]
            if t.device != self.device or t.dtype != _DTYPE[f] or t.shape[-1] < P:
                raise LtError('output %s has wrong device/dtype/shape' % f)
            if kind != 'pix':
                need = scene.n_years if kind == 'year' else params.n_rules
                if t.shape[0] < need or t.stride(1) != 1:
                    raise LtError('output %s too small' % f)
                s = t.stride(0)
                if ostride is None:
                    ostride = s
                elif s != ostride:
                    raise LtError('all [Y|R, P] outputs must share one row stride')
        tin = _abi.LtTileIn()
        tin.n_pix = P
        if lin is not None or index is not None:
            tin.stride = valid.stride(0) if valid is not None and valid.shape[0] > 1 else P
            tin.obs_bands = values.data_ptr()
            tin.band_obs_stride = values.stride(0)
            tin.band_stride = values.stride(1)
            tin.band_pix_stride = values.stride(2)
            if index is not None:
                tin.index = index.handle
            else:
                tin.lin = lin
        elif values.dtype == torch.float64:
            tin.stride = values.stride(0)
            tin.obs_val = ctypes.cast(values.data_ptr(), _abi.c_f64p)
        else:
            tin.stride = values.stride(0)
            tin.obs_index = values.data_ptr()
            tin.index_type = _LT_T[values.dtype]
        if valid is not None and valid.dtype == torch.int32:
            tin.obs_valid_bits = valid.data_ptr()
        else:
            tin.obs_valid = (ctypes.cast(valid.data_ptr(), _abi.c_u8p) if valid is not None
                             else None)
        tout = _abi.LtTileOut()
        tout.stride = ostride if ostride is not None else P
        for f, t in out.items():
            setattr(tout, f, ctypes.cast(t.data_ptr(), type(getattr(tout, f))))
        return tin, tout, out

    # --- load stage: index_eqn (rast_algebra, utils.py:447-484) ---
    def compile_index(self, program):
        """hiprtc-compile an index_eqn.IndexProgram for this device (cached per program). A
        program with an integer linear form is evaluated inside the analyze kernels, so its load
        kernel is compiled only when something asks for an index raster (IndexFn.handle): a
        job's analysis did not need the ~0.1 s."""
        def build():
            fn = ctypes.c_void_p()
            prog = program.to_c()
            with torch.cuda.device(self.device):
                self._check(self.lib.lt_index_compile(self.ctx, ctypes.byref(prog),
                                                      ctypes.byref(fn)), 'lt_index_compile')
            return fn
        lin = linear_form(program)
        if lin is not None:
            return IndexFn(None, program, lin, build=build)
        return IndexFn(build(), program, lin)

    def index_tile(self, fn, bands, out=None, stream=None):
        """bands: [K, NB, P] band planes (NB = the program's band slots; unit pixel stride, or
        pixel-interleaved: band stride 1, pixel stride NB) in the program's band type; returns the
        [K, P] index raster in the program's output type."""
        prog = fn.program
        want = _TORCH_OF_LT[_LT_T_OF_NP(prog.band_dtype)]
        if bands.dim() != 3 or bands.dtype != want or bands.device != self.device:
            raise LtError('bands must be a %s [K, %d, P] tensor on %s' % (want, len(prog.bands),
                                                                         self.device))
        K, NB, P = bands.shape
        if NB != len(prog.bands):
            raise LtError('bands must have %d band planes' % len(prog.bands))
        # planar ([K, NB, P], unit pixel stride) or pixel-interleaved (band stride 1, pixel stride
        # NB: lt_index_kernel4i reads a 4-pixel group's bands with NB vector loads)
        inter = bands.stride(1) == 1 and bands.stride(2) == NB and NB > 1
        if bands.stride(2) != 1 and not inter:
            bands = bands.contiguous()
        odt = _TORCH_OF_LT[_LT_T_OF_NP(prog.out_dtype)]
        if out is None:
            out = torch.empty((K, P), dtype=odt, device=self.device)
        if out.dtype != odt or out.shape[0] < K or out.shape[1] < P or out.stride(1) != 1:
            raise LtError('out must be a %s [K, P] tensor' % odt)
        io = _abi.LtIndexIO()
        io.n_pix, io.n_obs = P, K
        # (one band plane: its band stride is never used; the obs stride stands in)
        io.obs_stride = bands.stride(0)
        io.band_stride = bands.stride(1) if NB > 1 else bands.stride(0)
        io.band_pix_stride = bands.stride(2)
        io.out_stride = out.stride(0)
        io.bands, io.out = bands.data_ptr(), out.data_ptr()
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        self._check(self.lib.lt_index_apply(self.ctx, fn.handle, ctypes.byref(io),
                                            ctypes.c_void_p(st.cuda_stream)), 'lt_index_apply')
        return out

    # --- output raster assembly (output_reducer -> data2raster, lt_raster_assemble) ---
    def raster_assemble(self, jobs, stream=None):
        """jobs: a list of _abi.LtRasterJob (device pointers of this engine's tensors, which the
        caller keeps alive until the stream has run them)."""
        if not jobs:
            return
        arr = (_abi.LtRasterJob * len(jobs))(*jobs)
        st = stream if stream is not None else torch.cuda.current_stream(self.device)
        self._check(self.lib.lt_raster_assemble(self.ctx, arr, len(jobs),
                                                ctypes.c_void_p(st.cuda_stream)),
                    'lt_raster_assemble')

    # --- JIT kernels of tiles carrying a program (lt_jit.h; lt_ctx_set_jit_mode, lt_jit_prepare) ---
    def set_jit_mode(self, asynchronous):
        """False (default): a launch needing a JIT module compiles it first. True: modules compile
        on worker threads and tiles launched before theirs is ready run on the precompiled kernels
        (same results; counted in jit_stats()['fallback_tiles'])."""
        self._check(self.lib.lt_ctx_set_jit_mode(
            self.ctx, _abi.LT_JIT_ASYNC if asynchronous else _abi.LT_JIT_SYNC), 'set_jit_mode')

    def jit_prepare(self, scene, params, bands, valid, fields, index, wait=True):
        """Compile (wait) or start compiling the JIT module lt_analyze_tiles would use for a tile
        of these band planes, mask and output fields, carrying `index` (an IndexFn). Raises
        LtError when a waited-for compile fails (the launches would then fall back)."""
        P = bands.shape[-1]
        tin, _, _ = self._tile_structs(scene, params, bands, valid, (), {}, None, index)
        tout = _abi.LtTileOut()
        tout.stride = P
        for f in fields:  # which planes are requested is all the module depends on (never read)
            setattr(tout, f, ctypes.cast(ctypes.c_void_p(16), type(getattr(tout, f))))
        sc = scene.to_c()
        with torch.cuda.device(self.device):
            self._check(self.lib.lt_jit_prepare(self.ctx, ctypes.byref(sc), ctypes.byref(params),
                                                ctypes.byref(tin), ctypes.byref(tout),
                                                1 if wait else 0), 'lt_jit_prepare')

    def jit_stats(self):
        """The context's JIT counters (lt_jit_stats) and its last JIT failure message."""
        st = _abi.LtJitStats()
        msg = ctypes.create_string_buffer(2048)
        self._check(self.lib.lt_ctx_jit_stats(self.ctx, ctypes.byref(st), msg, len(msg)),
                    'jit_stats')
        d = {f: getattr(st, f) for f, _ in _abi.LtJitStats._fields_}
        d['last_error'] = msg.value.decode(errors='replace')
        return d

    # --- stage timing (HIP events recorded around every launch on the launch stream) ---
    def set_timing(self, enable):
        self._check(self.lib.lt_ctx_set_timing(self.ctx, 1 if enable else 0), 'set_timing')

    def stage_ms(self):
        ms = (ctypes.c_double * 3)()
        n = ctypes.c_int64()
        self._check(self.lib.lt_ctx_stage_ms(self.ctx, ms, 3, ctypes.byref(n)), 'stage_ms')
        return {'analyze': ms[0], 'resolve': ms[1], 'expand': ms[2], 'launches': n.value}

    def last_deferred(self):
        n = ctypes.c_int64()
        self._check(self.lib.lt_ctx_last_deferred(self.ctx, ctypes.byref(n)), 'last_deferred')
        return n.value


def pack_valid_bits(valid):
    """A [K, P] cloud mask (nonzero = valid, utils.py:353) as the bit planes the analyze kernel
    reads (lt_tile_in.obs_valid_bits): int32 [ceil(K/32), P], bit k % 32 of plane k // 32."""
    K, P = valid.shape
    acc = torch.zeros(((K + 31) // 32, P), dtype=torch.int64, device=valid.device)
    for k in range(K):
        acc[k // 32] |= (valid[k] != 0).to(torch.int64) << (k % 32)
    return acc.to(torch.int32)


def valid_bytes(valid, n_obs):
    """The [K, P] uint8 mask of either form (bytes, or pack_valid_bits planes)."""
    if valid is None or valid.dtype == torch.uint8:
        return valid
    return torch.stack([((valid[k // 32] >> (k % 32)) & 1).to(torch.uint8)
                        for k in range(n_obs)])


class IndexFn:
    """A compiled load-stage kernel (owned by the engine's context). lin: the program's integer
    linear form (_abi.LtIndexLin) when it has one: the analyze kernel then evaluates the index of
    each winner from the band planes itself (analyze_tile(..., lin=fn.lin)), and the load kernel
    is needed only to materialise an index raster."""

    def __init__(self, handle, program, lin=None, build=None):
        self._handle = handle
        self._build = build  # makes the handle on first use (Engine.compile_index)
        self.program = program
        self.lin = lin

    @property
    def handle(self):
        if self._handle is None and self._build is not None:
            self._handle, self._build = self._build(), None
        return self._handle


def linear_form(program):
    """lt_index_linearize of an index_eqn.IndexProgram: its _abi.LtIndexLin, or None when the
    program is not an integer linear form (divisions, float nodes, products of band terms, mixed
    node types, more than LT_LIN_MAX_BANDS bands). Host-only: needs the library, not a GPU."""
    lib = _abi.load_lib()
    lin = _abi.LtIndexLin()
    prog = program.to_c()
    if lib.lt_index_linearize(ctypes.byref(prog), ctypes.byref(lin)) != 0:
        return None
    return lin


def _LT_T_OF_NP(np_dtype):
    from .index_eqn import DTYPES
    return DTYPES[np_dtype]


_ENGINES = {}


def get_engine(device=None):
    if isinstance(device, torch.device):
        device = device.index
    idx = torch.cuda.current_device() if device is None else int(device)
    eng = _ENGINES.get(idx)
    if eng is None:
        eng = _ENGINES[idx] = Engine(idx)
    return eng


def label_tile(engine, years, params, val_fit, vertex, present=None, out=None, stream=None):
    """change_labeling alone on trendlines in device memory: val_fit float64 [Y, P],
    vertex / present uint8 [Y, P] (same strides). Returns the rule-plane dict + status."""
    import numpy as np
    # the C ABI reads val_fit, vertex and present with the one lin.stride: check every plane the
    # way _tile_structs checks a tile (a mismatch would be an out-of-bounds device read)
    if (not isinstance(val_fit, torch.Tensor) or val_fit.dim() != 2 or
            val_fit.dtype != torch.float64 or val_fit.device != engine.device or
            val_fit.stride(1) != 1):
        raise LtError('val_fit must be a float64 [Y, P] tensor on %s with unit pixel stride'
                      % engine.device)
    for name, t in (('vertex', vertex), ('present', present)):
        if t is None and name == 'present':
            continue
        if (not isinstance(t, torch.Tensor) or t.dtype != torch.uint8 or
                t.device != engine.device or t.shape != val_fit.shape or
                t.stride() != val_fit.stride()):
            raise LtError('%s must be uint8 with the shape and strides of val_fit' % name)
    Y, P = val_fit.shape
    yrs = np.ascontiguousarray(np.asarray(years, np.int32))
    if len(yrs) != Y:
        raise LtError('years must have one entry per slot')
    if out is None:
        out = engine.alloc_outputs(Y, params.n_rules, P, LABELS + ('status',))
    need = set(LABELS) | {'status'}
    if not need <= set(out):
        raise LtError('out lacks %s' % sorted(need - set(out)))
    rstride = None
    for f, t in out.items():
        kind = _SHAPE_KIND.get(f)
        if kind is None or t.device != engine.device or t.dtype != _DTYPE[f] or t.shape[-1] < P:
            raise LtError('output %s has wrong device/dtype/shape' % f)
        if kind == 'rule':
            if t.dim() != 2 or t.shape[0] < max(params.n_rules, 1) or t.stride(1) != 1:
                raise LtError('output %s too small' % f)
            if rstride is not None and t.stride(0) != rstride:
                raise LtError('all [R, P] outputs must share one row stride')
            rstride = t.stride(0)
        elif kind == 'pix' and t.stride(0) != 1:
            raise LtError('output %s must have unit pixel stride' % f)
    lin = _abi.LtLabelIn()
    lin.n_pix = P
    lin.stride = val_fit.stride(0)
    lin.n_years = Y
    lin.year = yrs.ctypes.data_as(_abi.c_i32p)
    lin.val_fit = ctypes.cast(val_fit.data_ptr(), _abi.c_f64p)
    lin.vertex = ctypes.cast(vertex.data_ptr(), _abi.c_u8p)
    lin.present = ctypes.cast(present.data_ptr(), _abi.c_u8p) if present is not None else None
    tout = _abi.LtTileOut()
    tout.stride = rstride
    for f, t in out.items():
        setattr(tout, f, ctypes.cast(t.data_ptr(), type(getattr(tout, f))))
    st = stream if stream is not None else torch.cuda.current_stream(engine.device)
    rc = engine.lib.lt_label_tile(engine.ctx, ctypes.byref(lin), ctypes.byref(params),
                                  ctypes.byref(tout), ctypes.c_void_p(st.cuda_stream))
    engine._check(rc, 'lt_label_tile')
    return out
