"""ctypes wrapper of the CPU oracle (oracle/build/liblt_oracle.so). TEST INFRASTRUCTURE ONLY.

Imported only by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg, as the checker
or the timed CPU baseline — never by land_trendr_amd. See lt_oracle.h for what it restates.
"""
import ctypes
import os

import numpy as np

from land_trendr_amd import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, 'build', 'liblt_oracle.so')
_LIB = None


def lib():
    global _LIB
    if _LIB is None:
        if not os.path.exists(LIB_PATH):
            raise RuntimeError('oracle not built: make -C oracle')
        L = ctypes.CDLL(LIB_PATH)
        D = _abi.c_f64p
        L.lto_lstsq.argtypes = [ctypes.c_int, D, D, D, D, D]
        L.lto_std.argtypes = [ctypes.c_int, D]
        L.lto_std.restype = ctypes.c_double
        L.lto_analyze_tile.argtypes = [ctypes.POINTER(_abi.LtScene), ctypes.POINTER(_abi.LtParams),
                                       ctypes.POINTER(_abi.LtTileIn),
                                       ctypes.POINTER(_abi.LtTileOut), ctypes.c_int]
        _LIB = L
    return _LIB


def lstsq(x, y):
    x = np.ascontiguousarray(x, np.float64)
    y = np.ascontiguousarray(y, np.float64)
    o = (ctypes.c_double * 3)()
    p = lambda i: ctypes.cast(ctypes.byref(o, 8 * i), _abi.c_f64p)
    rc = lib().lto_lstsq(len(x), x.ctypes.data_as(_abi.c_f64p), y.ctypes.data_as(_abi.c_f64p),
                         p(0), p(1), p(2))
    return rc, o[0], o[1], o[2]


def alloc_outputs(n_years, n_rules, n_pix):
    out = {}
    for f, dt in _abi.YEAR_FIELDS:
        out[f] = np.empty((n_years, n_pix), dt)
    for f, dt in _abi.RULE_FIELDS:
        out[f] = np.empty((max(n_rules, 1), n_pix), dt)
    for f, dt in _abi.PIX_FIELDS:
        out[f] = np.empty(n_pix, dt)
    return out


def out_struct(out, stride):
    o = _abi.LtTileOut()
    o.stride = stride
    for f, _ in _abi.YEAR_FIELDS + _abi.RULE_FIELDS + _abi.PIX_FIELDS:
        if f in out and out[f] is not None:
            setattr(o, f, out[f].ctypes.data_as(type(getattr(o, f))))
    return o


def analyze_tile(scene_meta, params, values, valid=None, n_threads=1, out=None):
    """Run the oracle over a tile: values [K, P] float64, valid [K, P] uint8 or None."""
    values = np.ascontiguousarray(values, np.float64)
    K, P = values.shape
    if valid is not None:
        valid = np.ascontiguousarray(valid, np.uint8)
    if out is None:
        out = alloc_outputs(scene_meta.n_years, params.n_rules, P)
    tin = _abi.LtTileIn()
    tin.n_pix = P
    tin.stride = P
    tin.obs_val = values.ctypes.data_as(_abi.c_f64p)
    tin.obs_valid = valid.ctypes.data_as(_abi.c_u8p) if valid is not None else None
    sc = scene_meta.to_c()
    o = out_struct(out, P)
    rc = lib().lto_analyze_tile(ctypes.byref(sc), ctypes.byref(params), ctypes.byref(tin),
                                ctypes.byref(o), int(n_threads))
    if rc != 0:
        raise RuntimeError('lto_analyze_tile failed: %d' % rc)
    return out
