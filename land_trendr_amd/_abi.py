"""ctypes mirror of include/lt_abi.h and the loader of the HIP library.

The library is built in-tree by __graft_entry__.build() (hipcc --offload-arch=gfx950) into
land_trendr_amd/liblt_hip.so. There is no CPU fallback: if the library is missing, load_lib()
raises, so a GPU run can never silently pass on something other than the HIP kernels.
"""
import ctypes
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'liblt_hip.so')

LT_ABI_VERSION = 7
LT_MAX_YEARS = 64
LT_MAX_OBS = 1024
LT_MAX_RULES = 16
LT_NODATA = -99

LT_ST_OK, LT_ST_EMPTY, LT_ST_SINGLE_YEAR = 0, 1, 2
LT_ST_PRE_THRESHOLD_ATTR, LT_ST_FEB29, LT_ST_NUMERIC = 4, 8, 16

LT_CT = {None: 0, 'FD': 1, 'GD': 2, 'LD': 3}
LT_Q_UNSET, LT_Q_EQ, LT_Q_LE, LT_Q_GE, LT_Q_GT, LT_Q_LT, LT_Q_OTHER = 0, 1, 2, 3, 4, 5, 9
LT_PRE_REFERENCE, LT_PRE_DOCUMENTED = 0, 1

c_i32p = ctypes.POINTER(ctypes.c_int32)
c_i16p = ctypes.POINTER(ctypes.c_int16)
c_u8p = ctypes.POINTER(ctypes.c_uint8)
c_f64p = ctypes.POINTER(ctypes.c_double)

# raster element types and the load-stage program (index_eqn)
(LT_T_F64, LT_T_I16, LT_T_U16, LT_T_I32, LT_T_F32, LT_T_U8, LT_T_U32, LT_T_I8,
 LT_T_I64) = range(9)
LT_MAX_PROG = 64
LT_MAX_BANDS = 16
(LT_OP_BAND, LT_OP_CONST_I, LT_OP_CONST_F, LT_OP_ADD, LT_OP_SUB, LT_OP_MUL, LT_OP_DIV,
 LT_OP_FLOORDIV, LT_OP_NEG) = range(1, 10)


class LtRule(ctypes.Structure):
    _fields_ = [('change_type', ctypes.c_int32), ('onset_op', ctypes.c_int32),
                ('duration_op', ctypes.c_int32), ('pre_op', ctypes.c_int32),
                ('onset_val', ctypes.c_double), ('duration_val', ctypes.c_double),
                ('pre_val', ctypes.c_double), ('class_val', ctypes.c_int32),
                ('_pad', ctypes.c_int32)]


class LtParams(ctypes.Structure):
    _fields_ = [('line_cost', ctypes.c_double), ('n_rules', ctypes.c_int32),
                ('pre_threshold_mode', ctypes.c_int32), ('rules', LtRule * LT_MAX_RULES)]


class LtScene(ctypes.Structure):
    _fields_ = [('n_obs', ctypes.c_int32), ('n_years', ctypes.c_int32), ('year', c_i32p),
                ('slot_begin', c_i32p), ('order', c_i32p), ('dist', c_i32p),
                ('feb29_bad', c_u8p)]


def build_hash():
    """Identity of the kernel build: sha256 (first 16 hex digits) over the sources liblt_hip.so
    is compiled from (csrc/*.h, csrc/*.hip, include/lt_abi.h) and the compile flags. bench.py
    records it in its line and profiles/summarize_pmc.py in every PMC summary, so a roofline
    whose counters come from another build is flagged."""
    import hashlib
    csrc = os.path.join(HERE, 'csrc')
    files = sorted(os.path.join(csrc, f) for f in os.listdir(csrc)
                   if f.endswith(('.h', '.hip')))
    files.append(os.path.join(os.path.dirname(HERE), 'include', 'lt_abi.h'))
    h = hashlib.sha256()
    for f in files:
        h.update(os.path.basename(f).encode() + b'\0')
        with open(f, 'rb') as fh:
            h.update(fh.read())
    try:
        import __graft_entry__ as ge  # the flags the library is built with
        h.update(' '.join(ge.HIP_FLAGS).encode())
    except ImportError:
        pass
    # switches that change the code the kernels run (JIT defines, specialisation, another
    # library, override code objects, ...): a run under any of them is another build
    for v in BUILD_ENV:
        if os.environ.get(v):
            h.update(('%s=%s\0' % (v, os.environ[v])).encode())
    return h.hexdigest()[:16]


BUILD_ENV = ('LT_JIT_DEFINES', 'LT_JIT_SPEC', 'LT_JIT_LINEAR', 'LT_JIT_WAVES', 'LT_JIT_SCENE',
             'LT_JIT_INDEX', 'LT_FUSED_INDEX', 'LT_TL_SPLIT', 'LT_JIT_OVERRIDE_DIR', 'LT_SRC_DIR',
             'LT_HIP_LIB', 'LT_DEFER_SETS', 'LT_RESOLVE_PRIORITY', 'LT_EXPAND_PRIORITY')


LT_LIN_MAX_BANDS = 4


class LtIndexLin(ctypes.Structure):
    _fields_ = [('n_bands', ctypes.c_int32), ('band_type', ctypes.c_int32),
                ('wrap_type', ctypes.c_int32), ('out_type', ctypes.c_int32),
                ('c0', ctypes.c_int64), ('coef', ctypes.c_int64 * LT_LIN_MAX_BANDS)]


class LtTileIn(ctypes.Structure):
    _fields_ = [('n_pix', ctypes.c_int64), ('stride', ctypes.c_int64), ('obs_val', c_f64p),
                ('obs_valid', c_u8p), ('obs_index', ctypes.c_void_p),
                ('index_type', ctypes.c_int32), ('_pad', ctypes.c_int32),
                ('obs_bands', ctypes.c_void_p), ('band_obs_stride', ctypes.c_int64),
                ('band_stride', ctypes.c_int64), ('band_pix_stride', ctypes.c_int64),
                ('lin', LtIndexLin), ('obs_valid_bits', ctypes.c_void_p),
                ('index', ctypes.c_void_p)]


class LtIndexOp(ctypes.Structure):
    _fields_ = [('op', ctypes.c_int32), ('type', ctypes.c_int32), ('ival', ctypes.c_int64),
                ('fval', ctypes.c_double)]


class LtIndexProg(ctypes.Structure):
    _fields_ = [('n_ops', ctypes.c_int32), ('n_bands', ctypes.c_int32),
                ('band_type', ctypes.c_int32), ('out_type', ctypes.c_int32),
                ('ops', LtIndexOp * LT_MAX_PROG)]


class LtSettings(ctypes.Structure):
    _fields_ = [('params', LtParams), ('target_year', ctypes.c_int32),
                ('target_month', ctypes.c_int32), ('target_day', ctypes.c_int32),
                ('n_index_bands', ctypes.c_int32), ('index_bands', ctypes.c_int32 * LT_MAX_BANDS),
                ('index', LtIndexProg)]


LT_EXC_NONE, LT_EXC_VALUE, LT_EXC_KEY, LT_EXC_TYPE, LT_EXC_ATTRIBUTE = 0, 1, 2, 3, 4
LT_EXC_ZERO_DIVISION, LT_EXC_OTHER = 5, 6
EXC_TYPES = {LT_EXC_VALUE: ValueError, LT_EXC_KEY: KeyError, LT_EXC_TYPE: TypeError,
             LT_EXC_ATTRIBUTE: AttributeError, LT_EXC_ZERO_DIVISION: ZeroDivisionError,
             LT_EXC_OTHER: Exception}


LT_RASTER_REFERENCE, LT_RASTER_TYPED = 0, 1
LT_SEL_ALL, LT_SEL_NONZERO, LT_SEL_EQUALS = 0, 1, 2


class LtRasterJob(ctypes.Structure):
    _fields_ = [('n_pix', ctypes.c_int64), ('plane', ctypes.c_void_p),
                ('plane_type', ctypes.c_int32), ('sel_kind', ctypes.c_int32),
                ('sel', ctypes.c_void_p), ('sel_value', ctypes.c_int32),
                ('holder_type', ctypes.c_int32), ('const_value', ctypes.c_double),
                ('dest', ctypes.c_void_p), ('n_out', ctypes.c_int64), ('mode', ctypes.c_int32),
                ('out_type', ctypes.c_int32), ('fill', ctypes.c_double), ('out', ctypes.c_void_p)]


class LtIndexIO(ctypes.Structure):
    _fields_ = [('n_pix', ctypes.c_int64), ('n_obs', ctypes.c_int64),
                ('obs_stride', ctypes.c_int64), ('band_stride', ctypes.c_int64),
                ('out_stride', ctypes.c_int64), ('bands', ctypes.c_void_p),
                ('out', ctypes.c_void_p), ('band_pix_stride', ctypes.c_int64)]


class LtTileOut(ctypes.Structure):
    _fields_ = [('stride', ctypes.c_int64), ('status', c_i32p), ('n_years', c_i32p),
                ('winner', c_i16p), ('val_raw', c_f64p), ('val_fit', c_f64p), ('fit_m', c_f64p),
                ('fit_b', c_f64p), ('right_m', c_f64p), ('right_b', c_f64p), ('spike', c_u8p),
                ('vertex', c_u8p), ('matched', c_u8p), ('class_val', c_i32p),
                ('onset_year', c_i32p), ('duration', c_i32p), ('magnitude', c_f64p),
                ('initial_val', c_f64p)]


class LtLabelIn(ctypes.Structure):
    _fields_ = [('n_pix', ctypes.c_int64), ('stride', ctypes.c_int64),
                ('n_years', ctypes.c_int32), ('year', c_i32p), ('val_fit', c_f64p),
                ('vertex', c_u8p), ('present', c_u8p)]


# per-year outputs [Y][stride] and per-rule outputs [R][stride]: (field, numpy dtype)
YEAR_FIELDS = [('winner', 'int16'), ('val_raw', 'float64'), ('val_fit', 'float64'),
               ('fit_m', 'float64'), ('fit_b', 'float64'), ('right_m', 'float64'),
               ('right_b', 'float64'), ('spike', 'uint8'), ('vertex', 'uint8')]
RULE_FIELDS = [('matched', 'uint8'), ('class_val', 'int32'), ('onset_year', 'int32'),
               ('duration', 'int32'), ('magnitude', 'float64'), ('initial_val', 'float64')]
PIX_FIELDS = [('status', 'int32'), ('n_years', 'int32')]

# symbols include/lt_abi.h declares (checked by tests/test_abi.py)
EXPORTS = ['lt_abi_version', 'lt_ctx_create', 'lt_ctx_destroy', 'lt_last_error',
           'lt_analyze_tile', 'lt_analyze_tiles', 'lt_analyze_tiles_after', 'lt_label_tile', 'lt_ctx_set_timing', 'lt_ctx_stage_ms',
           'lt_ctx_last_deferred', 'lt_index_codegen', 'lt_index_compile', 'lt_index_apply',
           'lt_settings_compile', 'lt_raster_assemble', 'lt_winner_presence',
           'lt_index_linearize', 'lt_ctx_set_jit_mode', 'lt_jit_prepare', 'lt_ctx_jit_stats',
           'lt_jit_source', 'lt_analyze_tiles_ev']

LT_JIT_SYNC, LT_JIT_ASYNC = 0, 1
LT_JIT_SRC_SPEC, LT_JIT_SRC_SCENE, LT_JIT_SRC_FIELDS = 1, 2, 4
# the kernels' output-plane bits (lt_pixel.h LT_FIELD_*), for LT_JIT_SRC_FIELDS
LT_FIELD_BITS = {f: 1 << k for k, f in enumerate((
    'status', 'n_years', 'matched', 'class_val', 'onset_year', 'duration', 'magnitude',
    'initial_val', 'winner', 'val_raw', 'val_fit', 'fit_m', 'fit_b', 'right_m', 'right_b',
    'spike', 'vertex'))}


class LtJitStats(ctypes.Structure):
    _fields_ = [(f, ctypes.c_int64) for f in ('jit_tiles', 'fallback_tiles', 'compiles',
                                              'disk_hits', 'failures', 'modules', 'evictions',
                                              'pending')]

_LIB = None


def load_lib(path=None):
    """Load liblt_hip.so and declare its signatures. Raises if the HIP library is absent."""
    global _LIB
    if _LIB is not None and path is None:
        return _LIB
    # LT_HIP_LIB: load another build of the same ABI (kernel ablation / A-B timing builds)
    p = path or os.environ.get('LT_HIP_LIB') or LIB_PATH
    if not os.path.exists(p):
        raise RuntimeError('HIP library %s not built: run __graft_entry__.build() '
                           '(no CPU fallback exists)' % p)
    lib = ctypes.CDLL(p)
    vp = ctypes.c_void_p
    lib.lt_abi_version.restype = ctypes.c_int
    lib.lt_ctx_create.argtypes = [ctypes.c_int, ctypes.POINTER(vp)]
    lib.lt_ctx_destroy.argtypes = [vp]
    lib.lt_last_error.argtypes = [vp]
    lib.lt_last_error.restype = ctypes.c_char_p
    lib.lt_analyze_tile.argtypes = [vp, ctypes.POINTER(LtScene), ctypes.POINTER(LtParams),
                                    ctypes.POINTER(LtTileIn), ctypes.POINTER(LtTileOut), vp]
    lib.lt_analyze_tiles.argtypes = [vp, ctypes.POINTER(LtScene), ctypes.POINTER(LtParams),
                                     ctypes.c_int, ctypes.POINTER(LtTileIn),
                                     ctypes.POINTER(LtTileOut), vp]
    lib.lt_analyze_tiles_after.argtypes = [vp, ctypes.POINTER(LtScene), ctypes.POINTER(LtParams),
                                           ctypes.c_int, ctypes.POINTER(LtTileIn),
                                           ctypes.POINTER(LtTileOut), ctypes.POINTER(vp), vp]
    lib.lt_analyze_tiles_ev.argtypes = [vp, ctypes.POINTER(LtScene), ctypes.POINTER(LtParams),
                                        ctypes.c_int, ctypes.POINTER(LtTileIn),
                                        ctypes.POINTER(LtTileOut), ctypes.POINTER(vp),
                                        ctypes.POINTER(vp), ctypes.c_int32, vp]
    lib.lt_label_tile.argtypes = [vp, ctypes.POINTER(LtLabelIn), ctypes.POINTER(LtParams),
                                  ctypes.POINTER(LtTileOut), vp]
    lib.lt_ctx_set_timing.argtypes = [vp, ctypes.c_int]
    lib.lt_ctx_stage_ms.argtypes = [vp, c_f64p, ctypes.c_int, ctypes.POINTER(ctypes.c_int64)]
    lib.lt_ctx_last_deferred.argtypes = [vp, ctypes.POINTER(ctypes.c_int64)]
    lib.lt_index_codegen.argtypes = [ctypes.POINTER(LtIndexProg), ctypes.c_char_p,
                                     ctypes.c_int64]
    lib.lt_index_codegen.restype = ctypes.c_int
    lib.lt_index_compile.argtypes = [vp, ctypes.POINTER(LtIndexProg), ctypes.POINTER(vp)]
    lib.lt_index_apply.argtypes = [vp, vp, ctypes.POINTER(LtIndexIO), vp]
    lib.lt_index_linearize.argtypes = [ctypes.POINTER(LtIndexProg), ctypes.POINTER(LtIndexLin)]
    lib.lt_raster_assemble.argtypes = [vp, ctypes.POINTER(LtRasterJob), ctypes.c_int, vp]
    lib.lt_winner_presence.argtypes = [vp, vp, ctypes.c_int64, ctypes.c_int32, ctypes.c_int64,
                                       ctypes.c_int32, vp, vp]
    lib.lt_settings_compile.argtypes = [ctypes.c_char_p, ctypes.c_int32, ctypes.c_int32,
                                        ctypes.c_int32, ctypes.c_int32,
                                        ctypes.POINTER(LtSettings),
                                        ctypes.POINTER(ctypes.c_int32), ctypes.c_char_p,
                                        ctypes.c_int64]
    lib.lt_ctx_set_jit_mode.argtypes = [vp, ctypes.c_int32]
    lib.lt_jit_prepare.argtypes = [vp, ctypes.POINTER(LtScene), ctypes.POINTER(LtParams),
                                   ctypes.POINTER(LtTileIn), ctypes.POINTER(LtTileOut),
                                   ctypes.c_int32]
    lib.lt_ctx_jit_stats.argtypes = [vp, ctypes.POINTER(LtJitStats), ctypes.c_char_p,
                                     ctypes.c_int64]
    lib.lt_jit_source.argtypes = [ctypes.POINTER(LtScene), ctypes.POINTER(LtParams),
                                  ctypes.POINTER(LtIndexProg), ctypes.c_int32, ctypes.c_int32,
                                  ctypes.c_int32, ctypes.c_char_p, ctypes.c_int64]
    lib.lt_jit_source.restype = ctypes.c_int
    if lib.lt_abi_version() != LT_ABI_VERSION:
        raise RuntimeError('liblt_hip.so ABI %d != %d' % (lib.lt_abi_version(), LT_ABI_VERSION))
    if path is None:
        _LIB = lib
    return lib
