"""Multi-GPU scene analysis: pixel tiles sharded over ranks, label rasters gathered to a writer.

Replaces the reference's MapReduce parallelism (MRLandTrendrJob.steps, mr_land_trendr_job.py:
154-159: one reducer call per pixel key, Hadoop shuffle by pixel WKT, then a second shuffle by
label key into output_reducer :128-152). Pixels are independent, so:
  - the scene is cut into fixed-size pixel tiles, dealt round-robin to ranks (tile t -> rank
    t % world: the per-pixel cost varies with masks/spikes, round-robin balances it);
  - each rank analyses its tiles with no communication at all;
  - the only collective is ONE gather of the per-rule label rasters (class_val, onset_year,
    duration, magnitude) to the writer rank, over RCCL (backend "nccl") on a GPU job or gloo on
    CPU tests. Per-year trendline planes are not gathered (54*T B/px: they stay on the rank that
    computed them and are streamed out per tile).
One process per GPU, torch.distributed initialised by the caller (torchrun env).
"""
import torch

LABEL_GATHER_FIELDS = ('class_val', 'onset_year', 'duration', 'magnitude')


def tile_ranges(n_pix, tile):
    return [(p0, min(n_pix, p0 + tile)) for p0 in range(0, n_pix, tile)]


def my_tiles(n_pix, tile, world, rank):
    """The tiles of `rank`: round-robin over the scene's tile list."""
    return tile_ranges(n_pix, tile)[rank::world]


def analyze_shard(n_pix, tile, world, rank, analyze_tile_fn):
    """Run analyze_tile_fn(p0, p1) -> {field: [R|Y, p1-p0] tensor} on this rank's tiles.
    Returns [(p0, p1, outputs), ...] in tile order."""
    return [(p0, p1, analyze_tile_fn(p0, p1)) for p0, p1 in my_tiles(n_pix, tile, world, rank)]


def gather_labels(shard, n_pix, tile, n_rules, world, rank, dist, dst=0,
                  fields=LABEL_GATHER_FIELDS, device=None):
    """Gather this rank's label planes to `dst` and assemble full [n_rules, n_pix] rasters there.

    Each rank packs its tiles back to back into one buffer per field (padded to the largest
    rank's pixel count), so the exchange is a single gather per field — on xGMI every peer has a
    direct link to the writer, so the writer's ingress runs all peers in parallel."""
    counts = [sum(p1 - p0 for p0, p1 in my_tiles(n_pix, tile, world, r)) for r in range(world)]
    cap = max(counts) if counts else 0
    out = {}
    for f in fields:
        ref = shard[0][2][f] if shard else None
        dtype = ref.dtype if ref is not None else (torch.float64 if f == 'magnitude'
                                                   else torch.int32)
        dev = ref.device if ref is not None else device
        buf = torch.zeros((n_rules, cap), dtype=dtype, device=dev)
        off = 0
        for p0, p1, o in shard:
            buf[:, off:off + (p1 - p0)] = o[f][:n_rules, :p1 - p0]
            off += p1 - p0
        bufs = [torch.empty_like(buf) for _ in range(world)] if rank == dst else None
        if world > 1:
            dist.gather(buf, bufs, dst=dst)
        else:
            bufs = [buf]
        if rank != dst:
            continue
        full = torch.empty((n_rules, n_pix), dtype=dtype, device=dev)
        for r in range(world):
            off = 0
            for p0, p1 in my_tiles(n_pix, tile, world, r):
                full[:, p0:p1] = bufs[r][:, off:off + (p1 - p0)]
                off += p1 - p0
        out[f] = full
    return out
