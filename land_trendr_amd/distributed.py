"""Multi-GPU analysis of a scene mosaic: pixel tiles sharded over ranks, label rasters sent to a
writer rank over RCCL point-to-point (xGMI), trendline planes streamed to the host per tile.

Replaces the reference's MapReduce parallelism (MRLandTrendrJob.steps, mr_land_trendr_job.py:
154-159: one reducer call per pixel key after a Hadoop shuffle by pixel WKT, :83-126, then a second
shuffle by label key into output_reducer, :128-152). Pixels are independent, so:

  * a mosaic is one or more scenes (co-registered stacks, each with its own acquisition dates),
    each cut into fixed-size pixel tiles; the tiles are dealt to ranks round-robin (tile t ->
    rank t % world: per-pixel cost varies with masks and spikes, round-robin balances it) or, for
    one scene per rank (the weak-scaling bench), by scene;
  * each rank analyses its tiles with no communication at all;
  * the only data exchange is the per-rule label rasters (class_val, onset_year, duration,
    magnitude) of every tile to the writer rank. The writer holds them tile-major
    ([n_tiles, R, tile], one contiguous slab per tile and field): its own tiles are analysed
    straight into their slabs, and in round k (the k-th tile of every rank) each other rank sends
    its slab with one point-to-point send per field, which the writer receives into the slab's
    final place — on xGMI every peer has its own link to the writer, so the (world - 1) sends of
    a round arrive in parallel, and no copy or padding follows. The sends are issued right after
    the tile's kernels are queued, on RCCL's stream, so a tile's labels travel while the next
    tile computes;
  * per-year trendline planes (54*T B/px: 106 GB for a 49 Mpx, T = 40 scene) do not fit any one
    GPU, so each rank streams them to pinned host memory per tile (TrendlineStream), overlapped
    with the next tile's kernels, for its host-side writer.

One process per GPU; torch.distributed is initialised by the caller (torchrun env). The same
classes run over gloo on CPU tensors (tests/test_distributed.py).
"""
import contextlib
from dataclasses import dataclass

import torch

LABEL_GATHER_FIELDS = ('class_val', 'onset_year', 'duration', 'magnitude')


@dataclass(frozen=True)
class Tile:
    t: int        # global tile id (mosaic order)
    scene: int    # scene index
    p0: int       # pixel range inside the scene
    p1: int
    g0: int       # first pixel in mosaic order (scenes back to back)

    @property
    def n(self):
        return self.p1 - self.p0


class Mosaic:
    """Scenes of `scene_pixels[s]` pixels cut into tiles of at most `tile` pixels, dealt to
    `world` ranks. assign='round_robin': tile t -> rank t % world; 'by_scene': scene s -> rank
    s % world (one scene per rank)."""

    def __init__(self, scene_pixels, tile, world=1, rank=0, assign='round_robin'):
        if tile <= 0 or world <= 0 or not 0 <= rank < world:
            raise ValueError('bad tile / world / rank')
        if assign not in ('round_robin', 'by_scene'):
            raise ValueError('assign must be round_robin or by_scene')
        self.scene_pixels = [int(n) for n in scene_pixels]
        self.tile, self.world, self.rank, self.assign = int(tile), world, rank, assign
        self.tiles = []
        g = 0
        for s, n in enumerate(self.scene_pixels):
            for p0 in range(0, n, self.tile):
                p1 = min(n, p0 + self.tile)
                self.tiles.append(Tile(len(self.tiles), s, p0, p1, g + p0))
            g += n
        self.n_pix = g

    def owner(self, tile):
        return (tile.t if self.assign == 'round_robin' else tile.scene) % self.world

    def tiles_of(self, rank):
        return [t for t in self.tiles if self.owner(t) == rank]

    @property
    def mine(self):
        return self.tiles_of(self.rank)

    @property
    def rounds(self):
        """Exchange rounds: the largest number of tiles any rank owns."""
        return max(len(self.tiles_of(r)) for r in range(self.world))


def tile_ranges(n_pix, tile):
    return [(t.p0, t.p1) for t in Mosaic([n_pix], tile).tiles]


def my_tiles(n_pix, tile, world, rank):
    """The (p0, p1) tiles of `rank` in a one-scene mosaic: round-robin over the tile list."""
    return [(t.p0, t.p1) for t in Mosaic([n_pix], tile, world, rank).mine]


class LabelExchange:
    """The mosaic's label rasters on the writer rank `dst`, filled by point-to-point sends.

    slab(tile) -> {field: [R, tile] tensor} is where this rank's kernels write tile `tile`'s
    label planes (its final place on the writer, a send buffer elsewhere). post(k) queues round
    k's sends / receives (non-blocking; on NCCL they run on RCCL's stream after the work already
    queued on the current stream), wait() completes every posted one, raster(field) assembles
    the writer's [R, n_pix] raster in mosaic pixel order."""

    def __init__(self, mosaic, spec, device, dist=None, dst=0, wire=None):
        """spec: {field: (rows, torch dtype)}, rows None for a [tile] plane (status) or the
        plane count of a [rows, tile] field (R for label fields, Y for trendline fields).
        wire: {field: torch dtype} a narrower type the field travels in (every value it holds
        must fit: the caller's guarantee, runner.label_wire_types); the writer widens it back."""
        self.m, self.dist, self.dst = mosaic, dist, dst
        self.spec = dict(spec)
        self.wire = {f: (wire or {}).get(f, self.spec[f][1]) for f in self.spec}
        self.fields = tuple(self.spec)
        self.device = torch.device(device)
        self.is_writer = mosaic.rank == dst
        T, W = len(mosaic.tiles), mosaic.tile
        if mosaic.world > 1 and dist is None:
            raise ValueError('world > 1 needs torch.distributed')

        def shape(f, lead=()):
            rows = self.spec[f][0]
            return lead + ((W,) if rows is None else (rows, W))

        self.full = None
        if self.is_writer:  # tile-major: slab t of every field is contiguous
            self.full = {f: torch.empty(shape(f, (T,)), dtype=self.spec[f][1], device=self.device)
                         for f in self.fields}
            self._slabs = {t.t: {f: self.full[f][t.t] for f in self.fields} for t in mosaic.mine}
        else:
            self._slabs = {t.t: {f: torch.empty(shape(f), dtype=self.spec[f][1],
                                                device=self.device) for f in self.fields}
                           for t in mosaic.mine}
        # gloo (the 1-GPU rehearsals and the GPU tests' multi-rank runs) hands a tensor's data
        # pointer to its CPU transport, which for a device tensor would read HBM without waiting
        # for the kernels that write it: device slabs then travel through host copies (the sender
        # copies after its queued work, the writer copies in after the receive). RCCL ops are
        # stream-ordered and take the device slabs directly.
        self._staged = (mosaic.world > 1 and self.device.type == 'cuda' and
                        dist.get_backend() == 'gloo')
        self._staged_in = []   # (host buffer, device slab) pairs to copy in after wait()
        self._staged_out = []  # host copies of sent slabs, kept alive until wait()
        # the writer's receives wait for nothing it computes: they are posted from a stream of
        # their own (an RCCL op first waits for the work queued on the current stream)
        self._recv_stream = (torch.cuda.Stream(self.device)
                             if self.is_writer and self.device.type == 'cuda' and not self._staged
                             else None)
        # a sender's sends wait for their tile's completion event on a stream of their own
        self._send_stream = (torch.cuda.Stream(self.device)
                             if not self.is_writer and self.device.type == 'cuda' and
                             not self._staged and mosaic.world > 1 else None)
        self._works = []   # (round, work) in posting order
        self._widen = []   # (wire buffer, raster slab): receives widened in wait()
        self._wbufs = {}   # (tile, field) -> the writer's wire-type receive buffer

    def slab(self, tile):
        return self._slabs[tile.t]

    def rebind(self, full):
        """World 1 only (nothing is sent): the writer's rasters become `full` (a dict like
        self.full), its slabs views of them. A one-tile runner's pipelined steps alternate two
        such sets (runner._flip_bank), so a step's analyze never waits for the previous step's
        resolve, which still writes the other set."""
        if self.m.world != 1 or not self.is_writer:
            raise ValueError('rebind: world 1 writer only')
        self.full = full
        self._slabs = {t.t: {f: full[f][t.t] for f in self.fields} for t in self.m.mine}

    def post(self, k, after=None):
        """Round k: the k-th tile of every rank goes to the writer. after: an event (this rank's
        tile k complete) the send waits for instead of the work queued on the current stream."""
        if self.m.world == 1:
            return
        d = self.dist
        ops = []
        widen = []  # (wire buffer, raster slab) pairs of this round's narrow receives
        if self.is_writer:
            for r in range(self.m.world):
                if r == self.dst:
                    continue
                mine = self.m.tiles_of(r)
                if k < len(mine):
                    t = mine[k].t
                    for f in self.fields:
                        dst = self.full[f][t]
                        if self._staged:
                            buf = torch.empty(dst.shape, dtype=self.wire[f])
                            self._staged_in.append((buf, dst))
                            dst = buf
                        elif self.wire[f] != dst.dtype:  # widened after the receive
                            buf = self._wire_buf(t, f, dst)
                            widen.append((buf, dst))
                            dst = buf
                        ops.append(d.P2POp(d.irecv, self._bytes(f, dst), r))
        else:
            mine = self.m.mine
            if k < len(mine):
                s = self._slabs[mine[k].t]
                if self._staged and after is not None:  # the host copy below waits for it
                    torch.cuda.current_stream(self.device).wait_event(after)
                narrow = [f for f in self.fields if self.wire[f] != s[f].dtype]
                packed = {}
                if narrow:  # narrowed after the tile's kernels: on the send stream behind `after`
                    # (into buffers kept per tile: this round's previous send of one completed
                    # before the tile's kernels ran again, runner._wait_sends / wait())
                    side = after is not None and self._send_stream is not None
                    with torch.cuda.stream(self._send_stream) if side else contextlib.nullcontext():
                        if side:
                            self._send_stream.wait_event(after)
                        t = mine[k].t
                        packed = {f: self._wire_buf(t, f, s[f]).copy_(s[f]) for f in narrow}
                for f in self.fields:
                    src = packed.get(f, s[f])
                    if self._staged:  # a blocking copy: after the kernels queued so far
                        src = src.cpu()
                        self._staged_out.append(src)
                    ops.append(d.P2POp(d.isend, self._bytes(f, src), self.dst))
        if ops:
            if self._recv_stream is not None:
                with torch.cuda.stream(self._recv_stream):
                    works = d.batch_isend_irecv(ops)
                    if widen:  # stream-ordered: after the receives, before the next round's
                        for w in works:
                            w.wait()
                        for buf, dst in widen:
                            dst.copy_(buf)
                        widen = []
            elif after is not None and self._send_stream is not None:
                # RCCL's stream waits for the send stream, which waits for this tile alone
                with torch.cuda.stream(self._send_stream):
                    self._send_stream.wait_event(after)
                    works = d.batch_isend_irecv(ops)
            else:
                works = d.batch_isend_irecv(ops)
            self._works += [(k, w) for w in works]
            self._widen += widen  # (no receive stream: widened in wait())

    def _bytes(self, f, x):
        """A narrowed field's buffer as the bytes the transport moves: RCCL (NCCL's type list)
        has no 16-bit integer type, and the widening reads the buffer in its own type."""
        return x.view(torch.uint8) if self.wire[f] != self.spec[f][1] else x

    def _wire_buf(self, t, f, like):
        """Tile t's field f in its wire type: the writer's receive buffer (a round's widening copy
        is queued before the next round's receive into it) or a sender's send buffer."""
        b = self._wbufs.get((t, f))
        if b is None:
            b = self._wbufs[(t, f)] = torch.empty(like.shape, dtype=self.wire[f],
                                                   device=like.device)
        return b

    def post_all(self):
        for k in range(self.m.rounds):
            self.post(k)

    def wait(self):
        while self._works:
            self._works.pop(0)[1].wait()
        for buf, dst in self._staged_in:
            dst.copy_(buf)
        for buf, dst in self._widen:
            dst.copy_(buf)
        if self._recv_stream is not None and any(self.wire[f] != self.spec[f][1]
                                                 for f in self.fields):
            # the widening copies ran on the receive stream
            torch.cuda.current_stream(self.device).wait_stream(self._recv_stream)
        self._staged_in, self._staged_out, self._widen = [], [], []

    @property
    def can_overlap(self):
        """Whether a round's ops may stay in flight past the step that posted them (RCCL: ops
        are stream-ordered; gloo's staged host copies need wait() in the step)."""
        return self.m.world > 1 and not self._staged

    def wait_round(self, k):
        """The current stream waits for the ops of round k posted so far (a previous step's send
        of slab k, before this step's kernels write it again); other rounds stay in flight. The
        writer's kernels write only its own slabs, which it never sends: nothing to wait for."""
        if self.is_writer:
            return
        keep = []
        for kk, w in self._works:
            if kk == k:
                w.wait()
            else:
                keep.append((kk, w))
        self._works = keep

    def checksums(self, tiles):
        """Position-weighted byte sums, one per (tile, field), of the slabs of `tiles` as this
        rank holds them: the writer's copies of every tile, a sender's own. Comparing the writer's
        with the owners' checks every exchanged byte landed where it belongs."""
        out = torch.zeros((len(self.m.tiles), len(self.fields)), dtype=torch.int64)
        for t in tiles:
            for j, f in enumerate(self.fields):
                a = (self.full[f][t.t] if self.is_writer else self._slabs[t.t][f])[..., :t.n]
                b = a.contiguous().view(torch.uint8).reshape(-1).to(torch.int64)
                w = torch.arange(b.numel(), device=b.device, dtype=torch.int64) % 251 + 1
                out[t.t, j] = int((b * w).sum().item())
        return out

    def raster(self, field):
        """[rows, n_pix] (or [n_pix]) in mosaic pixel order (writer only): the tile-major slabs
        laid side by side."""
        if not self.is_writer:
            raise ValueError('only the writer rank holds the rasters')
        a = self.full[field]
        out = torch.empty(a.shape[1:-1] + (self.m.n_pix,), dtype=a.dtype, device=a.device)
        for t in self.m.tiles:
            out[..., t.g0:t.g0 + t.n] = a[t.t, ..., :t.n]
        return out


class TrendlineStream:
    """D2H of per-year trendline planes into a ring of pinned host buffers, on a copy stream.

    A tile's [Y, tile] planes are copied one row (one year plane, contiguous) at a time into the
    next ring buffer; a buffer is reused once its previous copy has completed (the host writer
    reads it in between: `sink(field, row, host_view, key)` is called for each completed row when
    its buffer comes round again, and for the rest by drain(); `key` is what push() was given,
    e.g. the tile). The copy stream waits for the work
    queued on the current stream when push() is called, so queue tile t + 1's kernels before
    pushing tile t: its copies then overlap them, and a push that blocks on the ring does not
    hold back the next tile's launches."""

    def __init__(self, row_bytes, device, depth=8, sink=None):
        self.device = torch.device(device)
        self.stream = torch.cuda.Stream(self.device)
        self.ring = [torch.empty(int(row_bytes), dtype=torch.uint8, pin_memory=True)
                     for _ in range(depth)]
        self.pending = [None] * depth  # (event, field, row, nbytes, key) of the buffer's last copy
        self.sink = sink
        self.count = 0
        self.bytes = 0

    def _retire(self, slot):
        p = self.pending[slot]
        if p is None:
            return
        ev, f, row, nb, key = p
        ev.synchronize()
        if self.sink is not None:
            self.sink(f, row, self.ring[slot][:nb], key)
        self.pending[slot] = None

    def push(self, planes, n=None, key=None):
        """Queue the D2H of every row of planes[f] ([rows, W] device tensors; the first n pixels
        of each row, all W by default) after the work queued so far on the current stream.
        Returns an event recorded after the last of these copies: the planes may be overwritten
        once it has completed."""
        ready = torch.cuda.Event()
        ready.record()
        self.stream.wait_event(ready)
        for f, t in planes.items():
            rows = t if t.dim() == 2 else t[None]
            w = rows.shape[1] if n is None else n
            for r in range(rows.shape[0]):
                src = rows[r, :w]
                nb = src.numel() * src.element_size()
                slot = self.count % len(self.ring)
                self._retire(slot)
                dst = self.ring[slot][:nb]
                if nb > self.ring[slot].numel():
                    raise ValueError('row of %d bytes exceeds the ring buffers' % nb)
                with torch.cuda.stream(self.stream):
                    dst.copy_(src.view(torch.uint8), non_blocking=True)
                    ev = torch.cuda.Event()
                    ev.record()
                self.pending[slot] = (ev, f, r, nb, key)
                self.count += 1
                self.bytes += nb
        done = torch.cuda.Event()
        done.record(self.stream)
        return done

    def drain(self):
        for k in range(len(self.ring)):
            self._retire((self.count + k) % len(self.ring))
