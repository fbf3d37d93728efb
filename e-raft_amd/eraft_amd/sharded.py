"""Query-row sharding of the CorrBlock hot path across the GPUs of one node.

The reference has no multi-GPU CorrBlock; its only parallelism is Lightning DDP data
parallelism over frame pairs (train_dsec.py:197-209).  For high-resolution inputs the volume
is O(N^2) (1920x1280: 5.9 GB per pair), so the build partitions the QUERY pixels by rows:

  * every query owns its volume row C[n, :] and its pyramid slice, so a row partition needs
    no halo and no exchange in build, pyramid, lookup or lookup-backward;
  * rank g owns query rows [h0, h1) of every batch item (row_partition) and needs its fmap1
    rows plus the FULL fmap2 -> one RCCL broadcast of fmap2 per frame pair (over xGMI);
  * lookups produce the rank's output rows; an optional all-gather assembles the full
    [B, L*K, H, W] tensor when a replicated consumer needs it;
  * backward: dfmap1 is row-local; dfmap2 is a sum of per-rank partials -> all-reduce.

Per-query arithmetic is unchanged, so sharded results are bit-identical to one GPU.
The compute goes through libcorr_mi355x.so's *_rows entry points (``HipRows`` below).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib
from .corr import _alloc_pyramid


def row_partition(H: int, world: int, rank: int):
    """Rows [h0, h1) of rank `rank` when H query rows are split over `world` ranks."""
    per = -(-H // world)
    h0 = min(H, rank * per)
    return h0, min(H, h0 + per)


class HipRows:
    """Row-slab compute on the MI355X kernels (the only production backend)."""

    @staticmethod
    def build(f1_rows, f2, num_levels):
        B, _, rows, W = f1_rows.shape
        _, _, H, _ = f2.shape
        levels = _alloc_pyramid_rows(B, rows * W, H, W, num_levels, f2)
        _lib.build(f1_rows, f2, levels)
        return levels

    @staticmethod
    def lookup(levels, coords_rows, radius, H, W):
        B, _, rows, Wc = coords_rows.shape
        K = (2 * radius + 1) ** 2
        out = torch.empty((B, len(levels) * K, rows, Wc), dtype=torch.float32, device=coords_rows.device)
        _lib.lookup(levels, coords_rows, radius, out, H, W)
        return out


def _alloc_pyramid_rows(B, NQ, H, W, num_levels, like):
    shapes = [(H >> l, W >> l) for l in range(num_levels)]
    sizes = [B * NQ * h * w for h, w in shapes]
    offs, tot = [], 0
    for s in sizes:
        offs.append(tot)
        tot += (s + 3) // 4 * 4
    buf = torch.empty(tot, dtype=torch.float32, device=like.device)
    return [buf[o:o + s].view(B * NQ, 1, h, w) for o, s, (h, w) in zip(offs, sizes, shapes)]


class RowShardedCorrBlock:
    """CorrBlock whose query rows are partitioned over the ranks of `group`.

    fmap1: the full query map [B, D, H, W] (each rank slices its rows) or, with
           ``fmap1_is_slab=True``, already this rank's rows [B, D, h1-h0, W].
    fmap2: [B, D, H, W] on every rank; the contents on rank `src` are broadcast to all.
    __call__(coords): coords of this rank's rows [B, 2, h1-h0, W] (or the full [B, 2, H, W],
           sliced) -> this rank's lookup rows [B, L*K, h1-h0, W].
    """

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, group=None, src=0,
                 fmap1_is_slab=False, backend=HipRows, broadcast=True):
        self.num_levels, self.radius = num_levels, radius
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        B, D, H, W = fmap2.shape
        self.B, self.H, self.W = B, H, W
        self.h0, self.h1 = row_partition(H, self.world, self.rank)
        self.backend = backend
        if broadcast and self.world > 1:
            dist.broadcast(fmap2, src=src, group=group)
        f1 = fmap1 if fmap1_is_slab else fmap1[:, :, self.h0:self.h1]
        if f1.shape[2] != self.h1 - self.h0:
            raise ValueError(f"fmap1 slab has {f1.shape[2]} rows, rank {self.rank} owns "
                             f"{self.h1 - self.h0}")
        self.fmap2 = fmap2
        self.corr_pyramid = (backend.build(f1.contiguous(), fmap2, num_levels)
                             if self.h1 > self.h0 else None)

    @property
    def rows(self):
        return self.h1 - self.h0

    def __call__(self, coords):
        if coords.shape[2] == self.H and self.rows != self.H:
            coords = coords[:, :, self.h0:self.h1]
        coords = coords.contiguous()
        K = (2 * self.radius + 1) ** 2
        if self.corr_pyramid is None:
            return coords.new_empty((self.B, self.num_levels * K, 0, self.W))
        return self.backend.lookup(self.corr_pyramid, coords, self.radius, self.H, self.W)

    def gather(self, out_rows):
        """All-gather the ranks' output rows into the full [B, L*K, H, W] tensor."""
        if self.world == 1:
            return out_rows
        per = -(-self.H // self.world)
        B, C, rows, W = out_rows.shape
        pad = out_rows.new_zeros((B, C, per, W))
        pad[:, :, :rows] = out_rows
        parts = [torch.empty_like(pad) for _ in range(self.world)]
        dist.all_gather(parts, pad.contiguous(), group=self.group)
        full = []
        for g, p in enumerate(parts):
            h0, h1 = row_partition(self.H, self.world, g)
            full.append(p[:, :, :h1 - h0])
        return torch.cat(full, dim=2)
