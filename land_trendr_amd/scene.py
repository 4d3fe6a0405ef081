"""Host-side observation metadata for a tile: the date half of pick_winners.

pick_winners (/root/reference/utils.py:491-521) groups a pixel's observations by calendar year
and, per year, keeps the first observation (input order) of those closest in days to
target_date's month/day in that year. Everything in it that depends on dates only is shared by
all pixels of a co-registered stack, so it is computed here once per scene:
  - the ascending list of calendar years (one slot each),
  - per slot, the obs ids in input order,
  - per obs, |(target(year) - date).days|,
  - per slot, whether datetime(year, target.month, target.day) raises (Feb-29 target in a
    non-leap year: the reference's ValueError at utils.py:511-513).
The per-pixel half (which obs are valid, the argmin, the value gather) runs on the GPU.
"""
import datetime as _dt
from dataclasses import dataclass

import numpy as np

from . import _abi


def parse_date(date_string):
    """utils.parse_date (utils.py:194-202): strict 'YYYY-MM-DD', ValueError otherwise."""
    try:
        return _dt.datetime.strptime(date_string, '%Y-%m-%d')
    except Exception:
        raise ValueError('date_string must be in "YYYY-MM-DD" format')


def _as_date(d):
    if isinstance(d, _dt.datetime):
        return d.date()
    if isinstance(d, _dt.date):
        return d
    return parse_date(d).date()


@dataclass
class SceneMeta:
    years: np.ndarray       # [Y] int32
    slot_begin: np.ndarray  # [Y+1] int32
    order: np.ndarray       # [K] int32
    dist: np.ndarray        # [K] int32
    feb29_bad: np.ndarray   # [Y] uint8
    dates: list             # [K] datetime.date, input order
    n_obs: int

    @property
    def n_years(self):
        return len(self.years)

    def to_c(self):
        """An LtScene pointing into this object's arrays (keep `self` alive while in use)."""
        s = _abi.LtScene()
        s.n_obs = self.n_obs
        s.n_years = len(self.years)
        s.year = self.years.ctypes.data_as(_abi.c_i32p)
        s.slot_begin = self.slot_begin.ctypes.data_as(_abi.c_i32p)
        s.order = self.order.ctypes.data_as(_abi.c_i32p)
        s.dist = self.dist.ctypes.data_as(_abi.c_i32p)
        s.feb29_bad = self.feb29_bad.ctypes.data_as(_abi.c_u8p)
        return s


def build_scene(dates, target_date):
    """Observation metadata for obs `dates` (input order) and `target_date` (year ignored)."""
    ds = [_as_date(d) for d in dates]
    if len(ds) > _abi.LT_MAX_OBS:
        raise ValueError('at most %d observations per tile' % _abi.LT_MAX_OBS)
    years = sorted({d.year for d in ds})
    if len(years) > _abi.LT_MAX_YEARS:
        raise ValueError('at most %d distinct years per tile' % _abi.LT_MAX_YEARS)
    slot = {y: i for i, y in enumerate(years)}
    groups = [[] for _ in years]
    for k, d in enumerate(ds):
        groups[slot[d.year]].append(k)
    order, dist, begin = [], [], [0]
    feb = np.zeros(len(years), np.uint8)
    for i, y in enumerate(years):
        try:
            target = _dt.date(y, target_date.month, target_date.day)
        except ValueError:
            target = None
            feb[i] = 1
        for k in groups[i]:
            order.append(k)
            dist.append(0 if target is None else abs((target - ds[k]).days))
        begin.append(len(order))
    return SceneMeta(years=np.array(years, np.int32), slot_begin=np.array(begin, np.int32),
                     order=np.array(order, np.int32), dist=np.array(dist, np.int32),
                     feb29_bad=feb, dates=ds, n_obs=len(ds))
