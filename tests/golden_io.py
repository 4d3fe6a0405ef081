"""Load the committed golden fixtures (tests/golden/*.npz, made by the reference itself) and
compare engine outputs with them bit for bit."""
import datetime as dt
import glob
import json
import os

import numpy as np

from land_trendr_amd import _abi
from land_trendr_amd.scene import build_scene, parse_date
from land_trendr_amd.settings import compile_params

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), 'golden')


def scene_names():
    return sorted(os.path.basename(p)[6:-4] for p in glob.glob(os.path.join(GOLDEN, 'scene_*.npz')))


class GoldenScene:
    def __init__(self, name):
        z = np.load(os.path.join(GOLDEN, 'scene_%s.npz' % name))  # allow_pickle=False
        self.name = name
        self.meta = json.loads(str(z['meta']))
        self.values = z['values']
        self.valid = z['valid']
        self.err = [str(e) for e in z['err']]
        self.ref = {k: z[k] for k in z.files if k not in ('meta', 'values', 'valid', 'err')}
        self.scene = build_scene(self.meta['dates'], parse_date(self.meta['target']))
        self.params, self.rules = compile_params(self.meta['line_cost'], self.meta['rules'],
                                                 self.meta['mode'])
        assert list(self.scene.years) == self.meta['years']

    @property
    def n_pix(self):
        return self.values.shape[1]


def _bits_equal(a, b):
    """Bitwise float equality, any NaN equal to any NaN."""
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    na, nb = np.isnan(a), np.isnan(b)
    same = (a.view(np.int64) == b.view(np.int64)) | (na & nb)
    return same


def expected_status(err):
    if err == '':
        return 0
    if err == 'IndexError':
        return _abi.LT_ST_EMPTY
    if err == 'ValueError':
        return _abi.LT_ST_SINGLE_YEAR | _abi.LT_ST_FEB29
    if err == 'label:AttributeError':
        return _abi.LT_ST_PRE_THRESHOLD_ATTR
    raise AssertionError('unexpected reference error %r' % err)


def compare(g, out, max_report=5):
    """Return a list of mismatch descriptions (empty = bit-exact parity)."""
    bad = []
    P = g.n_pix
    R = len(g.rules)
    st = out['status']
    for p in range(P):
        exp = expected_status(g.err[p])
        if (exp == 0 and st[p] != 0) or (exp != 0 and not (st[p] & exp)):
            bad.append('pixel %d status %d, reference raised %r' % (p, st[p], g.err[p]))
    ok = np.array([e in ('', 'label:AttributeError') for e in g.err])
    yrs = np.asarray(g.scene.years)
    present = g.ref['winner'] >= 0
    for f, _ in _abi.YEAR_FIELDS:
        ref = g.ref[f]
        got = out[f][:, :P]
        if f in ('winner',):
            m = (ref != got)
        elif f in ('spike', 'vertex'):
            m = (ref != got) & present
        else:
            m = ~_bits_equal(ref, got) & present
        m &= ok[None, :]
        if m.any():
            ys, ps = np.nonzero(m)
            for y, p in list(zip(ys, ps))[:max_report]:
                bad.append('%s[year %d, pixel %d]: got %r want %r' % (f, yrs[y], p, got[y, p],
                                                                       ref[y, p]))
            bad.append('%s: %d mismatches' % (f, m.sum()))
    # index_day = year - first present year (timeseries2int_series, utils.py:552-554)
    first = np.argmax(present, axis=0)
    iday = np.where(present, yrs[:, None] - yrs[first][None, :], -1)
    m = (iday != g.ref['index_day']) & ok[None, :]
    if m.any():
        bad.append('index_day: %d mismatches' % m.sum())
    if out['n_years'] is not None:
        m = (out['n_years'][:P] != present.sum(0)) & ok
        if m.any():
            bad.append('n_years: %d mismatches' % m.sum())
    lab_ok = np.array([e == '' for e in g.err])
    for f in ('matched', 'class_val', 'onset_year', 'duration', 'magnitude'):
        ref = g.ref[f]
        got = out[f][:R, :P]
        if f == 'magnitude':
            m = ~_bits_equal(ref, got)
        else:
            m = ref != got
        m &= lab_ok[None, :]
        if m.any():
            rs, ps = np.nonzero(m)
            for r, p in list(zip(rs, ps))[:max_report]:
                bad.append('%s[rule %d, pixel %d]: got %r want %r' % (f, r, p, got[r, p],
                                                                       ref[r, p]))
            bad.append('%s: %d mismatches' % (f, m.sum()))
    return bad
