"""Seeded synthetic Landsat-like scenes for tests, goldens and bench.py.

A scene is a co-registered stack: every pixel sees the same acquisition dates (obs), so the
observation metadata is per scene and the values / cloud masks are per pixel, stored obs-major
([K][P], pixel index fastest) — the layout lt_analyze_tile consumes (include/lt_abi.h).

Per pixel (integers, as a `B1 - B2` int16 index would give):
  base ~ U{200..1500}; disturbance year d ~ U{3..T-5}; drop ~ U{100..800};
  recovery slope ~ U{0..drop/10}, recovery capped at drop; noise round(N(0, 40));
  spikes with probability 0.05 of +-U{200..1500}.
Per year K_y ~ U{k_min..k_max} observations with day-of-year ~ U{120..270}; cloud mask 0 with
probability `mask_prob` (masked obs are dropped, as apply_grid does, utils.py:350-354).
Bands: B2 ~ U{100..400}, B1 = B2 + index, so `B1 - B2` reproduces the index exactly in int16.

Everything is generated with torch on `device` (the bench builds 49 Mpx scenes directly in HBM).
"""
import datetime as _dt
from dataclasses import dataclass, field
from typing import List, Optional

import torch


@dataclass
class Scene:
    dates: List[_dt.date]              # [K] acquisition dates, in input (obs) order
    values: torch.Tensor               # [K, P] float64 index values
    valid: Optional[torch.Tensor]      # [K, P] uint8 (1 = keep), None = no cloud mask
    bands: Optional[torch.Tensor] = None  # [K, 2, P] int16 (B1, B2) when requested
    meta: dict = field(default_factory=dict)

    @property
    def n_obs(self):
        return len(self.dates)

    @property
    def n_pix(self):
        return self.values.shape[1]


def make_scene(n_pix, n_years=30, k_min=1, k_max=1, mask_prob=0.0, first_year=1985, seed=0,
               device='cpu', with_bands=False, spike_prob=0.05, chunk=1 << 22,
               band_layout='planar'):
    """Build a seeded synthetic scene. Deterministic for a given (seed, device type).
    band_layout: 'planar' ([K, 2, P] contiguous) or 'pixel' (the same [K, 2, P] view of a
    [K, P, 2] buffer: each pixel's two bands side by side, the fused load stage's layout)."""
    g_cpu = torch.Generator().manual_seed(int(seed))
    # --- per-scene observation dates (obs order = ascending acquisition date) ---
    dates = []
    year_of_obs = []
    for t in range(n_years):
        k_y = int(torch.randint(k_min, k_max + 1, (1,), generator=g_cpu))
        doys = sorted(int(v) for v in torch.randint(120, 271, (k_y,), generator=g_cpu))
        for doy in doys:
            dates.append(_dt.date(first_year + t, 1, 1) + _dt.timedelta(days=doy - 1))
            year_of_obs.append(t)
    K = len(dates)
    dev = torch.device(device)
    gen = torch.Generator(device=dev).manual_seed(int(seed) * 7919 + 17)
    t_obs = torch.tensor(year_of_obs, dtype=torch.int32, device=dev)
    values = torch.empty((K, n_pix), dtype=torch.float64, device=dev)
    valid = torch.empty((K, n_pix), dtype=torch.uint8, device=dev) if mask_prob > 0 else None
    bands = None
    if with_bands:
        bands = (torch.empty((K, n_pix, 2), dtype=torch.int16, device=dev).permute(0, 2, 1)
                 if band_layout == 'pixel' else
                 torch.empty((K, 2, n_pix), dtype=torch.int16, device=dev))
    for p0 in range(0, n_pix, chunk):
        p1 = min(n_pix, p0 + chunk)
        n = p1 - p0
        base = torch.randint(200, 1501, (n,), generator=gen, device=dev, dtype=torch.int32)
        d = torch.randint(3, max(4, n_years - 4), (n,), generator=gen, device=dev,
                          dtype=torch.int32)
        drop = torch.randint(100, 801, (n,), generator=gen, device=dev, dtype=torch.int32)
        u = torch.rand((n,), generator=gen, device=dev, dtype=torch.float64)
        slope = torch.floor(u * (drop // 10 + 1).double()).to(torch.int32)
        rel = t_obs[:, None] - d[None, :]                                  # [K, n]
        rec = torch.minimum(slope[None, :] * rel.clamp(min=0), drop[None, :])
        clean = torch.where(rel < 0, base[None, :], base[None, :] - drop[None, :] + rec)
        noise = torch.round(40.0 * torch.randn((K, n), generator=gen, device=dev,
                                                dtype=torch.float64)).to(torch.int32)
        sp = torch.rand((K, n), generator=gen, device=dev) < spike_prob
        mag = torch.randint(200, 1501, (K, n), generator=gen, device=dev, dtype=torch.int32)
        sign = torch.where(torch.rand((K, n), generator=gen, device=dev) < 0.5, -1, 1)
        idx = clean + noise + torch.where(sp, sign * mag, torch.zeros_like(mag))
        values[:, p0:p1] = idx.double()
        if valid is not None:
            valid[:, p0:p1] = (torch.rand((K, n), generator=gen, device=dev) >= mask_prob).to(
                torch.uint8)
        if bands is not None:
            b2 = torch.randint(100, 401, (K, n), generator=gen, device=dev, dtype=torch.int32)
            bands[:, 0, p0:p1] = (b2 + idx).to(torch.int16)
            bands[:, 1, p0:p1] = b2.to(torch.int16)
    return Scene(dates=dates, values=values, valid=valid, bands=bands,
                 meta=dict(n_years=n_years, k_min=k_min, k_max=k_max, mask_prob=mask_prob,
                           first_year=first_year, seed=seed))


def mosaic_inputs(mosaic, n_years, k_min=1, k_max=1, mask_prob=0.0, seed0=1000, device='cpu',
                  target_date='2014-07-01', band_layout='pixel', mask_format='bits'):
    """runner.TileInput for every tile this rank owns in `mosaic`: scene s is the seeded scene
    make_scene(seed=seed0 + s) as int16 bands (B1, B2) + cloud mask, so a tile's content does not
    depend on the number of ranks. A rank owning a whole scene keeps it in place (tiles are views
    sharing one index raster); otherwise its tiles are copied out and the scene freed. Bands are
    pixel-interleaved by default (make_scene band_layout); cloud masks are bit planes by default
    (engine.pack_valid_bits; mask_format='bytes' keeps the [K, P] uint8 mask)."""
    from .runner import TileInput
    from .scene import build_scene, parse_date
    items = []
    dev = torch.device(device)
    for s in sorted({t.scene for t in mosaic.mine}):
        sc = make_scene(mosaic.scene_pixels[s], n_years=n_years, k_min=k_min, k_max=k_max,
                        mask_prob=mask_prob, seed=seed0 + s, device=dev, with_bands=True,
                        band_layout=band_layout)
        sc.values = None  # only the bands travel (the load stage computes the index raster)
        if sc.valid is not None and mask_format == 'bits':
            from .engine import pack_valid_bits
            sc.valid = pack_valid_bits(sc.valid)
        meta = build_scene(sc.dates, parse_date(target_date))
        mine = [t for t in mosaic.mine if t.scene == s]
        whole = len(mine) == sum(1 for t in mosaic.tiles if t.scene == s)
        K, P = meta.n_obs, mosaic.scene_pixels[s]
        index = torch.empty((K, P), dtype=torch.int16, device=dev) if whole else None
        for t in mine:
            sl = slice(t.p0, t.p1)
            if whole:
                items.append(TileInput(t, meta, index[:, sl],
                                       sc.valid[:, sl] if sc.valid is not None else None,
                                       sc.bands[:, :, sl]))
            else:
                items.append(TileInput(t, meta, torch.empty((K, t.n), dtype=torch.int16,
                                                            device=dev),
                                       sc.valid[:, sl].clone() if sc.valid is not None else None,
                                       sc.bands[:, :, sl].clone()))
        del sc
        if dev.type == 'cuda':
            torch.cuda.empty_cache()
    return items
