"""The per-rank tile pipeline of a mosaic job: load stage -> analyze + label -> label exchange.

For every tile this rank owns (distributed.Mosaic), in tile order:
  1. load stage (parse_mapper's rast_algebra, mr_land_trendr_job.py:67-68 / utils.py:447-484):
     the analyze kernel evaluates the index_eqn program on the winners' band values itself (the
     fused load stage: no index raster, no kernel between tiles) — an integer linear form
     (engine.IndexFn.lin; 'B1 - B2' is one) in the precompiled kernel, any other program in JIT
     kernels with the program inlined (lt_jit.h); with the fusion off (LT_FUSED_INDEX=0 /
     LT_JIT_INDEX=0) the hiprtc-compiled index_eqn kernel turns the tile's band planes into its
     index raster, on a stream of its own, recording an event per tile;
  2. analyze + label (analysis_reducer, mr_land_trendr_job.py:83-126): lt_analyze_tiles_after on
     the current stream, tile t waiting only for tile t's index event, so later tiles' load
     kernels (HBM-bound) run beside earlier tiles' analyze kernels (issue-bound); consecutive
     tiles of one scene share a call (tile t's resolve stage runs beside tile t+1's analyze);
  3. the tile's label rasters go to the writer rank (distributed.LabelExchange) as soon as its
     kernels are queued, so they travel while the next tile computes.
bench.py, the job runner (job.py) and the GPU tests all run this one code path.
"""
import contextlib
import os
from dataclasses import dataclass
from typing import Optional

import torch

from . import _abi
from .distributed import LABEL_GATHER_FIELDS, LabelExchange
from .engine import _DTYPE, _SHAPE_KIND


_nullctx = contextlib.nullcontext


@dataclass
class TileInput:
    tile: object                       # distributed.Tile
    scene: object                      # scene.SceneMeta (lt_scene of the tile's scene)
    # [K, n] index raster: given, or written by the load stage from the bands (None: allocated
    # when the load kernel first writes it — never, on the fused path)
    values: Optional[torch.Tensor]
    valid: Optional[torch.Tensor]      # [K, n] uint8 or None
    bands: Optional[torch.Tensor] = None  # [K, NB, n] band planes, or None (values given)


def label_wire_types(params, fields):
    """The narrower types the label planes travel to the writer in (LabelExchange wire), chosen
    from what the kernels can write (lt_pixel.h RuleState1::write): onset_year a calendar year
    (1-9999, a datetime.date's) or LT_NODATA, duration a year count (<= 255, lt_abi.h limits) or
    LT_NODATA, class_val a rule's class value or LT_NODATA. Every such value fits int16 (class_val:
    when the rules' values do), which narrows c2's 20 bytes per pixel and rule on the wire to 14
    (magnitude stays binary64); the writer's rasters keep the API types. The choice depends on
    the job's rules only, so every rank makes the same one."""
    lo, hi = -(1 << 15), (1 << 15) - 1
    w = {f: torch.int16 for f in ('onset_year', 'duration') if f in fields}
    vals = [int(params.rules[r].class_val) for r in range(params.n_rules)] + [_abi.LT_NODATA]
    if 'class_val' in fields and all(lo <= v <= hi for v in vals):
        w['class_val'] = torch.int16
    return w


class MosaicRunner:
    """One rank's share of a mosaic job on one GPU.

    fields: the output planes the kernels write per tile; label fields in `exchange_fields` live
    in the LabelExchange's slabs (their final place on the writer rank), the others in per-tile
    slabs of this rank. group: tiles per lt_analyze_tiles call (0: every consecutive tile of a
    scene, or 1 when labels are exchanged, so tile t's sends travel while tile t+1 computes).
    ring: 0, every tile has planes of its own for the fields not exchanged (the trendline
    planes); R > 0, tile k writes them into buffer k % R of a ring (one tile per call), and
    step()'s slab_free(j) names the event after which tile j's buffer may be overwritten (its
    D2H copies done): the rank's HBM then holds R tiles' trendline planes, not all of them.
    jit: False keeps the index_eqn program off the JIT kernels (a linear program then runs in
    the precompiled kernels, any other through the load kernel), as LT_JIT_INDEX=0 does."""

    def __init__(self, engine, mosaic, params, items, fields, index_fn=None, dist=None,
                 exchange_fields=LABEL_GATHER_FIELDS, load_stream=True, group=0, dst=0,
                 fused=None, ring=0, jit=True):
        self.eng, self.m, self.params, self.items = engine, mosaic, params, list(items)
        self.fields = tuple(fields)
        self.index_fn = index_fn
        if [it.tile.t for it in self.items] != [t.t for t in mosaic.mine]:
            raise ValueError('items must be this rank\'s tiles, in mosaic order')
        R = max(params.n_rules, 1)
        ys = {it.scene.n_years for it in self.items} or {0}
        Y = max(ys)
        ex = [f for f in exchange_fields if f in self.fields]

        def rows(f):
            k = _SHAPE_KIND[f]
            return None if k == 'pix' else (R if k == 'rule' else Y)

        self.exchange = LabelExchange(mosaic, {f: (rows(f), _DTYPE[f]) for f in ex},
                                      engine.device, dist, dst,
                                      wire=label_wire_types(params, ex))
        W = mosaic.tile
        self.ring = max(0, int(ring))
        self._ring_last = {}  # ring slot -> (slab_free of its step, tile) of its last user

        def planes():
            return {f: torch.empty((W,) if rows(f) is None else (rows(f), W), dtype=_DTYPE[f],
                                   device=engine.device) for f in self.fields if f not in ex}

        shared = [planes() for _ in range(min(self.ring, len(self.items)))]
        self.outs = []
        for k, it in enumerate(self.items):
            o = dict(self.exchange.slab(it.tile))
            o.update(shared[k % self.ring] if self.ring else planes())
            self.outs.append(o)
        # with an exchange, every tile's label send waits for that tile's own completion event
        # (lt_analyze_tiles_ev), not for the caller's stream: the tiles of a scene still share
        # one call, so tile t's resolve stage keeps running beside tile t+1's analyze kernel
        # (one call per tile, each joined to the stream before the next, serialised it)
        self.gathering = mosaic.world > 1 and bool(ex)
        self.group = group if group > 0 else 1 << 30
        if self.ring:
            self.group = 1
        has_bands = any(it.bands is not None for it in self.items)
        # (a CPU engine — the gloo tests' oracle double — has no streams: everything is serial)
        self.cuda = torch.device(engine.device).type == 'cuda'
        if has_bands and index_fn is None:
            raise ValueError('band inputs need a compiled index_eqn (index_fn)')
        # fused load stage: on unless fused=False or LT_FUSED_INDEX=0. An integer linear program
        # (engine.IndexFn.lin) runs in the precompiled analyze kernel; any other program in JIT
        # analyze kernels with the program inlined (lt_jit.h; LT_JIT_INDEX=0 keeps the load
        # kernel and its index raster for those)
        if fused is None:
            fused = os.environ.get('LT_FUSED_INDEX', '1') != '0'
        all_bands = has_bands and all(it.bands is not None for it in self.items)
        jit_ok = (fused and all_bands and self.cuda and jit and
                  os.environ.get('LT_JIT_INDEX', '1') != '0')
        self.lin = getattr(index_fn, 'lin', None) if fused and all_bands else None
        # a linear program too goes to the JIT kernels, specialised for the job's configuration
        # (lt_jit.h Spec), unless LT_JIT_LINEAR=0 keeps it on the precompiled kernels
        if self.lin is not None and jit_ok and os.environ.get('LT_JIT_LINEAR', '1') != '0':
            self.lin = None
        self.jit = index_fn if jit_ok and self.lin is None else None
        self.fused = self.lin is not None or self.jit is not None
        prio = int(os.environ.get('LT_LOAD_PRIORITY', '0'))
        self.load_stream = (torch.cuda.Stream(engine.device, priority=prio)
                            if self.cuda and has_bands and load_stream and not self.fused
                            else None)
        self.index_events = []  # (start, stop) pairs of the timed steps' load kernels
        # pipelined steps (step(overlap=True)): the tiles' completion events not yet joined, the
        # last completion event of every (bank, tile)'s output planes, and the output banks
        self._pending = []
        self._prev_done = {}
        self._inflight = False  # a step left tiles or transfers in flight (finish() joins them)
        self._ex_fields = tuple(ex)
        self._banks = [self.outs]
        self._bank = 0

    def _done_events(self, n):
        """Per-tile completion events for a call whose tiles' labels are exchanged, or whose last
        stages run on past the step (pipelined steps), created by a first record so the library's
        record on its own stream is the one waited for; or None."""
        if not ((self.gathering or getattr(self, '_pipe', False)) and self.cuda):
            return None
        evs = [torch.cuda.Event() for _ in range(n)]
        for e in evs:
            e.record()
        return evs

    @staticmethod
    def _ev_kw(done):
        return {} if done is None else {'done': done, 'join': False}

    def _join(self, pending):
        """The current stream waits for every tile's completion: the step's outputs are complete
        in stream order, as with joined calls."""
        if pending:
            cur = torch.cuda.current_stream(self.eng.device)
            for e in pending:
                cur.wait_event(e)

    def prepare_jit(self, wait=True):
        """Compile (wait) or start compiling the JIT module of every scene this rank's tiles
        belong to before the first step, so no launch waits for hiprtc (a mosaic with several
        scenes compiles them side by side with wait=False under engine.set_jit_mode(True))."""
        if self.jit is None:
            return
        seen = set()
        for it in self.items:
            if it.tile.scene in seen:
                continue
            seen.add(it.tile.scene)
            self.eng.jit_prepare(it.scene, self.params, it.bands, it.valid, self.fields, self.jit,
                                 wait=wait)

    def _groups(self):
        """Consecutive items of one scene, at most self.group per call."""
        g = []
        for k, it in enumerate(self.items):
            if g and (it.tile.scene != self.items[g[0]].tile.scene or len(g) >= self.group):
                yield g
                g = []
            g.append(k)
        if g:
            yield g

    def step(self, timed=False, after_tile=None, stage_in=None, slab_free=None, overlap=False):
        """Queue one pass over this rank's tiles and complete the label exchange.
        after_tile(k): called once tile k's kernels are queued (e.g. to stream its trendline).
        stage_in: an object whose fetch(k) -> (bands, event) supplies tile k's band planes from
        elsewhere (an H2D copy the load kernel waits for) and whose consumed(k, event) learns
        when the load kernel has read them. slab_free(j): with a ring, the event (or None)
        after which tile j's ring buffer is free again; tile j + ring waits for it.
        overlap: the step's work stays in flight past its return, as for a stream of scenes; call
        finish() after the last step. The label exchange (RCCL; not gloo, whose staged copies
        complete in the step): the next step's kernels for tile k wait only for this step's send
        of tile k's slab, so the last tiles' transfers overlap the next step's first tiles. The
        tiles' last stages (resolve, trendline expand; on a GPU with the fused load stage, without
        a ring or stage_in): the current stream does not wait for them at the step's end, so the
        last tile's resolve runs beside the next step's first analyze as consecutive tiles of one
        call do. Safe for inputs that change between steps:
          * tile k's analyze kernel waits (lt_analyze_tiles_ev `ready`) for the completion event
            of the last step that wrote the same output planes, so no resolve of an earlier step
            writes them while a later step's analyze does (a pixel deferred in one step but not
            in the next would otherwise keep the earlier step's value);
          * a runner of ONE tile alternates between two banks of its output planes (self.outs
            names the bank the last step wrote; at world 1 also the label rasters,
            self.exchange.full): its next step writes the other bank, so its analyze still runs
            beside the previous step's resolve;
          * a caller that rewrites tile k's INPUT planes (bands, mask) between pipelined steps
            first makes its stream wait for tile_done(k): the previous step's resolve reads them.
        overlap=False after pipelined steps completes them first (finish())."""
        eng = self.eng
        if not self.cuda:
            timed = False
        if self.ring and self.cuda and slab_free is None:
            raise ValueError('a ring of output buffers needs slab_free')
        if not overlap and self._inflight:
            self.finish()  # a joined step after pipelined ones joins them first
        self._slab_free = slab_free
        self._overlap = bool(overlap) and self.exchange.can_overlap
        # (the unfused load path writes it.values on the load stream while the previous step's
        # resolve may still read them: pipelined steps need the fused load stage)
        self._pipe = (bool(overlap) and self.cuda and not self.ring and stage_in is None and
                      self.fused)
        if self._pipe and len(self.items) == 1:
            self._flip_bank()
        if self.fused:
            return self._step_fused(after_tile, stage_in)
        main = torch.cuda.current_stream(eng.device) if self.cuda else None
        ready = [None] * len(self.items)
        pending = []  # the tiles' completion events (gathering): the stream joins them at the end
        if self.load_stream is not None:  # the previous step's analyze kernels read the rasters
            self.load_stream.wait_stream(main)
        for k, it in enumerate(self.items):
            if it.bands is None:
                continue
            bands = it.bands
            if stage_in is not None:
                bands, ev_in = stage_in.fetch(k)
            with (torch.cuda.stream(self.load_stream if self.load_stream is not None else main)
                  if self.cuda else _nullctx()):
                if stage_in is not None:
                    torch.cuda.current_stream(eng.device).wait_event(ev_in)
                if timed:
                    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(
                        enable_timing=True)
                    e0.record()
                it.values = eng.index_tile(self.index_fn, bands, out=it.values)
                if timed:
                    e1.record()
                    self.index_events.append((e0, e1))
                if self.cuda and (self.load_stream is not None or stage_in is not None):
                    ev = torch.cuda.Event()
                    ev.record()
                    ready[k] = ev
                    if stage_in is not None:
                        stage_in.consumed(k, ev)
        for g in self._groups():
            scene = self.items[g[0]].scene
            n = [self.items[k].tile.n for k in g]
            self._wait_ring(g[0])
            self._wait_sends(g)
            done = self._done_events(len(g))
            eng.analyze_tiles(
                scene, self.params, [(self.items[k].values, self.items[k].valid) for k in g],
                self.fields, outs=[{f: x[..., :nk] for f, x in self.outs[k].items()}
                                   for k, nk in zip(g, n)],
                ready=[ready[k] for k in g] if self.load_stream is not None else None,
                **self._ev_kw(done))
            for j, k in enumerate(g):
                self.exchange.post(k, after=done[j] if done is not None else None)
                if after_tile is not None:
                    after_tile(k)
            pending += done or []
        # rounds past this rank's own tiles: the writer still receives the tiles of ranks that
        # own more (unequal scenes under by_scene, or a writer other than rank 0); a sender has
        # nothing left to post
        for k in range(len(self.items), self.m.rounds):
            self.exchange.post(k)
        self._end_step(pending)

    def _step_fused(self, after_tile, stage_in):
        """step() with the fused load stage: each tile's analyze kernel reads its band planes.
        With stage_in, one tile per call: tile k's analyze waits for its H2D copy, and its slab is
        handed back once the call's work (analyze + resolve) is done."""
        eng = self.eng
        main = torch.cuda.current_stream(eng.device)
        groups = ([[k] for k in range(len(self.items))] if stage_in is not None
                  else list(self._groups()))
        pending = []  # the tiles' completion events (gathering): the stream joins them at the end
        for g in groups:
            scene = self.items[g[0]].scene
            n = [self.items[k].tile.n for k in g]
            tiles, ready = [], None
            for k in g:
                bands = self.items[k].bands
                if stage_in is not None:
                    bands, ev_in = stage_in.fetch(k)
                    ready = [ev_in]
                tiles.append((bands, self.items[k].valid))
            self._wait_ring(g[0])
            self._wait_sends(g)
            done = self._done_events(len(g))
            if self._pipe:  # tile k waits for the last step that wrote its planes (see step)
                ready = [self._prev_done.get((self._bank, k)) for k in g]
                if not any(e is not None for e in ready):
                    ready = None
            eng.analyze_tiles(
                scene, self.params, tiles, self.fields,
                outs=[{f: x[..., :nk] for f, x in self.outs[k].items()} for k, nk in zip(g, n)],
                ready=ready, lin=self.lin, index=self.jit, **self._ev_kw(done))
            if done is not None:
                for j, k in enumerate(g):
                    self._prev_done[(self._bank, k)] = done[j]
            if stage_in is not None:
                ev = torch.cuda.Event()
                ev.record(main)
                stage_in.consumed(g[0], ev)
            for j, k in enumerate(g):
                self.exchange.post(k, after=done[j] if done is not None else None)
                if after_tile is not None:
                    after_tile(k)
            pending += done or []
        for k in range(len(self.items), self.m.rounds):
            self.exchange.post(k)
        self._end_step(pending)

    def _flip_bank(self):
        """A one-tile runner's pipelined step writes the other bank of its output planes. At
        world 1 nothing is sent, so the label rasters alternate too (LabelExchange.rebind): the
        step's analyze waits for nothing the previous step still runs, and its resolve overlaps
        this step's analyze. At world > 1 the exchanged label slabs are shared by the banks: they
        are waited for through the tile's done event."""
        own = self.m.world == 1 and self.exchange.full is not None
        if len(self._banks) == 1:
            o = self._banks[0][0]
            if own:
                full1 = {f: torch.empty_like(x) for f, x in self.exchange.full.items()}
                self._fulls = [self.exchange.full, full1]
                t = self.items[0].tile.t
                self._banks.append([{f: (full1[f][t] if f in self._ex_fields
                                         else torch.empty_like(x)) for f, x in o.items()}])
            else:
                self._banks.append([{f: (x if f in self._ex_fields else torch.empty_like(x))
                                     for f, x in o.items()}])
        self._bank ^= 1
        self.outs = self._banks[self._bank]
        if own:
            self.exchange.rebind(self._fulls[self._bank])
        elif any(f in self._ex_fields for f in self.outs[0]):
            # the shared slabs: the other bank's last writer must be complete as well
            other = self._prev_done.get((self._bank ^ 1, 0))
            if other is not None:
                self._prev_done[(self._bank, 0)] = other

    def tile_done(self, k):
        """The event after which the last step's outputs of tile k are complete and its input
        planes are no longer read (pipelined steps; None: the current stream's order suffices).
        A caller that rewrites tile k's inputs between pipelined steps waits for it first."""
        return self._prev_done.get((self._bank, k)) if self._pending else None

    def _wait_sends(self, g):
        """With overlap: before tiles g are written again, the stream waits for the previous
        step's sends of their slabs (a sender; the writer's receives are ordered on RCCL's
        stream, and its own slabs are not sent)."""
        if getattr(self, '_overlap', False):
            for k in g:
                self.exchange.wait_round(k)

    def _end_step(self, pending):
        """The step's outputs complete in stream order (joined), or, pipelined, left to finish()."""
        if getattr(self, '_pipe', False):
            self._pending = self._pending + pending
            self._inflight = True
        else:
            self._join(pending)
        if not self._overlap:
            self.exchange.wait()
        else:
            self._inflight = True

    def finish(self):
        """Complete every tile and exchange still in flight (after steps run with overlap=True):
        the current stream waits for every tile's last stage."""
        self._join(self._pending)
        self._pending = []
        self._prev_done = {}
        self._inflight = False
        self.exchange.wait()

    def _wait_ring(self, k):
        """Tile k reuses the ring buffer k % ring: the current stream waits until the planes of
        the tile that last used it — tile k - ring of this step, or for k < ring one of the
        previous step's last tiles (a second step() on a ring runner) — have been
        copied out, as the slab_free of that tile's step reports."""
        if not self.ring or not self.cuda:
            return
        slot = k % self.ring
        last = self._ring_last.get(slot)
        self._ring_last[slot] = (self._slab_free, k)
        if last is None:
            return
        free, j = last
        ev = free(j)
        if ev is not None:
            torch.cuda.current_stream(self.eng.device).wait_event(ev)

    def materialise_index(self, k):
        """Tile k's index raster (items[k].values) from its band planes with the load kernel, on
        the current stream — what the fused steps never write; the oracle checks read it."""
        it = self.items[k]
        if self.index_fn is None or it.bands is None:
            return
        it.values = self.eng.index_tile(self.index_fn, it.bands, out=it.values)

    def index_ms(self):
        ev, self.index_events = self.index_events, []
        return sum(a.elapsed_time(b) for a, b in ev) / len(ev) if ev else None
