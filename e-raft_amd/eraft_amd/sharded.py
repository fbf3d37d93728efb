"""Query-row sharding of the CorrBlock hot path across the GPUs of one node.

The reference has no multi-GPU CorrBlock; its only parallelism is Lightning DDP data
parallelism over frame pairs (train_dsec.py:197-209).  For high-resolution inputs the volume
is O(N^2) (1920x1280: 5.9 GB per pair), so the build partitions the QUERY pixels by rows:

  * every query owns its volume row C[n, :] and its pyramid slice, so a row partition needs
    no halo and no exchange in build, pyramid, lookup or lookup-backward;
  * rank g owns query rows [h0, h1) of every batch item (row_partition) and needs its fmap1
    rows plus the FULL fmap2 -> one RCCL broadcast of fmap2 per frame pair (over xGMI), sent as
    target-row chunks (chunk_bounds: multiples of the build's 8-row patches) whose broadcasts
    are all issued at once; each rank builds a chunk's pyramid entries (corr_build_region) as
    soon as that chunk has arrived, so the transfer of chunk k+1 overlaps the build of chunk k;
  * lookups produce the rank's output rows; an optional all-gather assembles the full
    [B, L*K, H, W] tensor when a replicated consumer needs it;
  * backward (training): every lookup's backward is stashed and the build's backward runs
    corr_backward on the slab (all lookups' gradients + the pool fold + the two GEMMs), giving
    the slab's dfmap1 rows and a PARTIAL dfmap2 (the slab's queries only).  Gradient rule:
    when every rank holds the FULL fmap1 (a replicated encoder, the default), both gradients
    are SUM-all-reduced (RCCL, B*D*H*W floats each), so every rank ends with the single-GPU
    dfmap1 and dfmap2 — the encoder's parameter gradients are then identical on all ranks and
    equal to the single-GPU ones (DDP's averaging of identical values keeps them).  With
    ``fmap1_is_slab=True`` (a row-sharded fmap1 producer) dfmap1 stays the rank's rows and only
    dfmap2 is all-reduced.

Per-query arithmetic is unchanged, so sharded results are bit-identical to one GPU.
The compute goes through libcorr_mi355x.so's *_rows entry points (``HipRows`` below).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from . import _lib
from .corr import _alloc_grad_pyramid, _alloc_pyramid


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

    # target-row regions of one build (the chunked broadcast): allocate, then build region by region
    @staticmethod
    def export(levels, H, W):
        """The slab's tiled levels -> the reference layout [B*NQ, 1, H_l, W_l]."""
        return _lib.pyramid_export(levels, H, W)

    @staticmethod
    def region_supported(num_levels):
        return _lib.default_algo() == _lib.BUILD_BF16X6 and num_levels <= 4

    @staticmethod
    def region_begin(f1_rows, f2_shape, num_levels):
        B, _, rows, W = f1_rows.shape
        H = f2_shape[2]
        levels = _alloc_pyramid_rows(B, rows * W, H, W, num_levels, f1_rows)
        return levels, _lib.build_workspace(f1_rows, tuple(f2_shape), _lib.BUILD_BF16X6)

    @staticmethod
    def build_region(f1_rows, f2_chunk, y0, y1, H, levels, ws, first):
        _lib.build_region(f1_rows, f2_chunk, y0, y1, H, levels, ws, first)

    @staticmethod
    def lookup(levels, coords_rows, radius, H, W):
        B, _, rows, Wc = coords_rows.shape
        K = (2 * radius + 1) ** 2
        out = torch.empty((B, len(levels) * K, rows, Wc), dtype=torch.float32, device=coords_rows.device)
        _lib.lookup(levels, coords_rows, radius, out, H, W)
        return out

    @staticmethod
    def zero_pyramid(B, NQ, H, W, num_levels, like):
        """A zeroed gradient pyramid of the slab (the reference's row-major layout)."""
        return _alloc_grad_pyramid(B, H, W, num_levels, like, zero=True, NQ=NQ)

    @staticmethod
    def lookup_bwd(coords_rows, grad_rows, radius, grad_levels, H, W):
        _lib.lookup_bwd(coords_rows, grad_rows, radius, grad_levels, H, W)

    @staticmethod
    def pool_bwd(grad_levels, H, W):
        _lib.pool_bwd(grad_levels, H, W)

    @staticmethod
    def build_bwd(grad_c, f1_rows, f2):
        """-> (dfmap1 of the slab, this slab's partial dfmap2)."""
        return _lib.build_bwd(grad_c, f1_rows, f2)

    @staticmethod
    def backward(coords_list, grad_list, radius, f1_rows, f2, num_levels):
        """corr_backward on the slab: every stashed lookup's backward, the pool fold and the GEMMs
        in one call -> (dfmap1 of the slab, this slab's partial dfmap2)."""
        B, _, rows, W = f1_rows.shape
        H = f2.shape[2]
        gl = _alloc_grad_pyramid(B, H, W, num_levels, f2, NQ=rows * W)  # scratch
        return _lib.backward(coords_list, grad_list, radius, gl, f1_rows, f2)


def chunk_bounds(H: int, chunks: int):
    """Target-row chunks [y0, y1) of the chunked fmap2 broadcast: about H / chunks rows each,
    rounded up to a multiple of 8 (the build's patch rows, so each chunk's pyramid rows are
    complete at every level <= 4)."""
    step = max(8, -(-(-(-H // max(1, chunks))) // 8) * 8)
    return [(y, min(H, y + step)) for y in range(0, H, step)]


def _broadcast_build_chunked(backend, f1_rows, fmap2, num_levels, bounds, src, group, rank):
    """Broadcast rank src's fmap2 as target-row chunks (all issued asynchronously, in order) and
    build each chunk's pyramid rows as soon as it has arrived; non-source ranks also assemble the
    chunks into fmap2 (the broadcast's contract: fmap2 ends as rank src's map everywhere).
    Returns the pyramid levels of this rank's query slab."""
    B, D, H, W = fmap2.shape
    with torch.no_grad():
        bufs = [fmap2.new_empty((B, D, y1 - y0, W)) for y0, y1 in bounds]
        if rank == src:
            for buf, (y0, y1) in zip(bufs, bounds):
                buf.copy_(fmap2[:, :, y0:y1])
        works = [dist.broadcast(buf, src=src, group=group, async_op=True) for buf in bufs]
        levels, ws = backend.region_begin(f1_rows, tuple(fmap2.shape), num_levels)
        for k, ((y0, y1), buf, work) in enumerate(zip(bounds, bufs, works)):
            work.wait()  # RCCL: the compute stream waits on chunk k only; chunk k+1 keeps arriving
            if f1_rows.shape[2] > 0:
                backend.build_region(f1_rows, buf, y0, y1, H, levels, ws, k == 0)
            if rank != src:
                fmap2[:, :, y0:y1].copy_(buf)
    return levels


_CHUNKS_AGREED = {}


def _group_key(group):
    """A cache key for a process group that survives the group object: its backend and the
    global ranks it spans (id() of a destroyed group can be reused by a new one)."""
    ranks = tuple(dist.get_process_group_ranks(group)) if group is not None else tuple(range(dist.get_world_size()))
    return (dist.get_backend(group), ranks)


def agree_chunks(H, num_levels, chunks=0, group=None, device=None, region=True):
    """The chunk count RowShardedCorrBlock(..., chunks=chunks) will use for H rows, agreed over
    the group (a blocking all-reduce + host read).  The agreement runs the first time a
    (group, H, levels, chunks) key is seen; call this once, eagerly, before capturing a
    RowShardedCorrBlock construction into a HIP graph, since a capture cannot hold the host
    read (bench.py's eager warm-up pair does the same)."""
    local = chunks if chunks else (4 if region and H >= 32 else 1)
    if not region:
        local = 1
    if dist.get_world_size(group) == 1:
        return local
    return _agreed_chunks(group, (H, num_levels, chunks), local, device)


def _agreed_chunks(group, key, local, device):
    """The broadcast's chunk count, agreed over the group once per (group, key): the MIN of the
    ranks' own choices.  Each rank's choice depends on its environment (ERAFT_AMD_BUILD decides
    whether the region build exists), and ranks that disagreed would issue different numbers of
    broadcasts and hang.  key holds only values every rank shares (H, levels, the requested
    count), so every rank hits or misses the cache together.  The first call for a key runs a
    blocking all-reduce and a host read: it must not happen inside a graph capture (see
    agree_chunks)."""
    k = (_group_key(group), key)
    if k not in _CHUNKS_AGREED:
        t = torch.tensor([local], dtype=torch.int64, device=device)
        dist.all_reduce(t, op=dist.ReduceOp.MIN, group=group)
        _CHUNKS_AGREED[k] = int(t.item())
    return _CHUNKS_AGREED[k]


def _alloc_pyramid_rows(B, NQ, H, W, num_levels, like):
    """The tiled pyramid of a slab of NQ queries per batch item (corr._alloc_pyramid)."""
    return _alloc_pyramid(B, H, W, num_levels, like, NQ=NQ)


class _ShardState:
    __slots__ = ("levels", "grad_levels", "B", "NQ", "H", "W", "backend", "group", "h0", "h1", "full1", "stash",
                 "radius", "chunked")


class _ShardBuildFn(torch.autograd.Function):
    """Build of the rank's slab; backward = pool fold + slab GEMMs + all-reduce of dfmap2 (and,
    when fmap1 is the full replicated map, of the zero-padded dfmap1)."""

    @staticmethod
    def forward(ctx, f1, f2, num_levels, st):
        f1_rows = f1[:, :, st.h0:st.h1].contiguous() if st.full1 else f1
        if st.chunked is not None:  # the chunked broadcast of f2, each chunk built on arrival
            bounds, src, rank = st.chunked
            lv = _broadcast_build_chunked(st.backend, f1_rows, f2, num_levels, bounds, src, st.group, rank)
            st.levels = lv if st.NQ > 0 else None
        else:
            st.levels = st.backend.build(f1_rows, f2, num_levels) if st.NQ > 0 else None
        ctx.save_for_backward(f1_rows, f2)
        ctx.st, ctx.num_levels, ctx.f1_shape = st, num_levels, tuple(f1.shape)
        return f1.new_zeros(())  # autograd anchor of the lookups

    @staticmethod
    def backward(ctx, _):
        f1_rows, f2 = ctx.saved_tensors
        st = ctx.st
        gl, st.grad_levels = st.grad_levels, None
        stash, st.stash = st.stash, []
        if stash and st.NQ > 0:  # fused: every lookup's backward + fold + GEMMs in corr_backward
            df1, df2 = st.backend.backward([c for c, _ in stash], [g for _, g in stash], st.radius, f1_rows, f2,
                                           ctx.num_levels)
        elif st.NQ > 0:
            if gl is None:  # no lookup reached the loss on this rank
                gl = st.backend.zero_pyramid(st.B, st.NQ, st.H, st.W, ctx.num_levels, f2)
            st.backend.pool_bwd(gl, st.H, st.W)
            df1, df2 = st.backend.build_bwd(gl[0], f1_rows, f2)
        else:  # a rank without rows still joins the all-reduces
            df1, df2 = torch.zeros_like(f1_rows), torch.zeros_like(f2)
        if st.full1:
            full = df1.new_zeros(ctx.f1_shape)
            full[:, :, st.h0:st.h1] = df1
            df1 = full
        if dist.get_world_size(st.group) > 1:
            dist.all_reduce(df2, group=st.group)
            if st.full1:
                dist.all_reduce(df1, group=st.group)
        return df1, df2, None, None


class _ShardLookupFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, coords_rows, token, radius, st):
        ctx.save_for_backward(coords_rows)
        ctx.st, ctx.radius = st, radius
        return st.backend.lookup(st.levels, coords_rows, radius, st.H, st.W)

    @staticmethod
    def backward(ctx, grad_rows):
        (coords_rows,) = ctx.saved_tensors
        st = ctx.st
        if hasattr(st.backend, "backward") and _lib.fused_backward():
            st.radius = ctx.radius
            st.stash.append((coords_rows, grad_rows.contiguous()))  # run by the build's backward
        else:
            if st.grad_levels is None:
                st.grad_levels = st.backend.zero_pyramid(st.B, st.NQ, st.H, st.W, len(st.levels), coords_rows)
            st.backend.lookup_bwd(coords_rows, grad_rows.contiguous(), ctx.radius, st.grad_levels, st.H, st.W)
        # no gradient for the token: the engine still runs the build's backward (corr._LookupFn)
        return None, None, None, None


class PendingFmap2:
    """A pair's fmap2 whose broadcast from rank `src` is in flight (RowShardedCorrBlock.prefetch).

    Handing it to RowShardedCorrBlock replaces the constructor's blocking broadcast by a wait on
    this one: with RCCL the compute stream waits for the collective's stream (the host does not
    block), so the broadcast of pair k+1 runs while pair k is built and looked up."""

    __slots__ = ("tensor", "_work")

    def __init__(self, tensor, work):
        self.tensor, self._work = tensor, work

    @property
    def done(self):
        return self._work is None

    def wait(self):
        if self._work is not None:
            self._work.wait()
            self._work = None
        return self.tensor


class Fmap2DoubleBuffer:
    """Two receive buffers for a stream of frame pairs: ``prefetch(next_fmap2)`` starts the
    broadcast of the next pair's fmap2 into the buffer the pair before last used, so pair k's
    build reads one buffer while pair k+1's broadcast fills the other.  On rank `src` the
    argument is that rank's fmap2 (it is copied into the buffer on the compute stream, so the
    caller may reuse its own tensor); the other ranks pass None.  Stream order makes the
    reuse safe: the collective waits for the compute stream's earlier work (pair k-1's build,
    the last reader of the buffer it overwrites) before it starts.

    Inference only: the buffers are detached copies that the prefetch two pairs later
    overwrites, so no gradient could reach the caller's fmap2 through them, and a delayed
    backward would read a later pair's features.  prefetch() therefore runs only with autograd
    disabled (torch.no_grad(), as E-RAFT's eval runs, test.py:84) and raises on EVERY rank
    otherwise — before any collective, on a condition every rank of an SPMD job shares, so no
    rank is left inside a broadcast — and RowShardedCorrBlock raises on every rank when handed a
    PendingFmap2 while its fmap1 requires grad; train with the blocking broadcast
    (RowShardedCorrBlock(fmap1, fmap2))."""

    def __init__(self, shape, device, group=None, src=0, dtype=torch.float32):
        self.group, self.src = group, src
        self.rank = dist.get_rank(group)
        self.bufs = [torch.empty(shape, dtype=dtype, device=device) for _ in range(2)]
        self.k = 0

    def prefetch(self, fmap2=None):
        if torch.is_grad_enabled():
            # the grad mode is the same on every rank, so all ranks refuse together (whereas only
            # the source rank could see its fmap2's requires_grad)
            raise RuntimeError("Fmap2DoubleBuffer is inference-only (its buffers carry no gradient "
                               "back to fmap2): call prefetch under torch.no_grad(), or train with "
                               "RowShardedCorrBlock(fmap1, fmap2)")
        buf = self.bufs[self.k % 2]
        self.k += 1
        if self.rank == self.src:
            if fmap2 is None:
                raise ValueError(f"rank {self.src} is the broadcast source: pass its fmap2")
            buf.copy_(fmap2.detach())
        return RowShardedCorrBlock.prefetch(buf, src=self.src, group=self.group)


class RowShardedCorrBlock:
    """CorrBlock whose query rows are partitioned over the ranks of `group`.

    fmap1: the full query map [B, D, H, W] (each rank slices its rows) or, with
           ``fmap1_is_slab=True``, already this rank's rows [B, D, h1-h0, W].
    fmap2: [B, D, H, W] on every rank; the contents on rank `src` are broadcast to all — in
           ``chunks`` target-row chunks whose builds start as each arrives (0 = automatic:
           4 when the backend builds by region and H >= 32, else one blocking broadcast) — or a
           PendingFmap2 from ``prefetch`` whose broadcast was started earlier and overlapped the
           previous pair's work (see Fmap2DoubleBuffer).
    __call__(coords): coords of this rank's rows [B, 2, h1-h0, W] (or the full [B, 2, H, W],
           sliced) -> this rank's lookup rows [B, L*K, h1-h0, W].
    """

    @staticmethod
    def prefetch(fmap2, src=0, group=None):
        """Start broadcasting rank `src`'s fmap2 into `fmap2` on every rank without waiting;
        returns the PendingFmap2 to construct the block from."""
        if dist.get_world_size(group) == 1:
            return PendingFmap2(fmap2, None)
        with torch.no_grad():
            work = dist.broadcast(fmap2, src=src, group=group, async_op=True)
        return PendingFmap2(fmap2, work)

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4, group=None, src=0,
                 fmap1_is_slab=False, backend=HipRows, broadcast=True, chunks=0):
        self.num_levels, self.radius = num_levels, radius
        self.group = group
        self.world = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        if isinstance(fmap2, PendingFmap2):  # broadcast already issued (prefetch): wait for it
            if torch.is_grad_enabled() and fmap1.requires_grad:
                # every rank sees the same fmap1 flag (SPMD), so all ranks refuse together and
                # none is left waiting in a gradient all-reduce
                raise RuntimeError("a prefetched (double-buffered) fmap2 is inference-only: its buffer "
                                   "carries no gradient and is overwritten two pairs later; train with "
                                   "RowShardedCorrBlock(fmap1, fmap2)")
            fmap2 = fmap2.wait()
            broadcast = False
        B, D, H, W = fmap2.shape
        self.B, self.H, self.W = B, H, W
        self.h0, self.h1 = row_partition(H, self.world, self.rank)
        self.backend = backend
        region = hasattr(backend, "build_region") and backend.region_supported(num_levels)
        asked = chunks
        if chunks == 0:
            chunks = 4 if region and H >= 32 else 1
        if not region:
            chunks = 1
        if broadcast and self.world > 1:
            chunks = _agreed_chunks(group, (H, num_levels, asked), chunks, fmap2.device)
        bounds = chunk_bounds(H, chunks) if chunks > 1 else None
        chunked = broadcast and self.world > 1 and bounds is not None and len(bounds) > 1
        if broadcast and self.world > 1 and not chunked:
            with torch.no_grad():
                dist.broadcast(fmap2, src=src, group=group)
        f1 = fmap1 if fmap1_is_slab else fmap1[:, :, self.h0:self.h1]
        if f1.shape[2] != self.h1 - self.h0:
            raise ValueError(f"fmap1 slab has {f1.shape[2]} rows, rank {self.rank} owns "
                             f"{self.h1 - self.h0}")
        self.fmap2 = fmap2
        self._token = None
        if torch.is_grad_enabled() and (f1.requires_grad or fmap2.requires_grad):
            # training: autograd through the slab; gradients all-reduced over `group` (module doc)
            st = _ShardState()
            st.B, st.NQ, st.H, st.W = B, (self.h1 - self.h0) * W, H, W
            st.backend, st.group, st.grad_levels, st.levels = backend, group, None, None
            st.stash, st.radius = [], radius
            st.h0, st.h1, st.full1 = self.h0, self.h1, not fmap1_is_slab
            st.chunked = (bounds, src, self.rank) if chunked else None
            self._st = st
            src1 = fmap1 if st.full1 else f1.contiguous()
            self._token = _ShardBuildFn.apply(src1, fmap2, num_levels, st)
            self._levels = st.levels if self.h1 > self.h0 else None
            return
        if chunked:
            lv = _broadcast_build_chunked(backend, f1.contiguous(), fmap2, num_levels, bounds, src, group, self.rank)
            self._levels = lv if self.h1 > self.h0 else None
        else:
            self._levels = (backend.build(f1.contiguous(), fmap2, num_levels)
                            if self.h1 > self.h0 else None)

    @property
    def corr_pyramid(self):
        """This rank's slab of the pyramid as the reference holds it (corr.py:16,24,27,36): a list
        of [B*rows*W, 1, H_l, W_l] tensors (None on a rank without rows), exported from the
        backend's internal levels on access as CorrBlock.corr_pyramid does (HipRows keeps them
        tiled, include/corr_mi355x.h).  A read-only export: it carries no gradient."""
        if self._levels is None:
            return None
        export = getattr(self.backend, "export", None)
        return export(self._levels, self.H, self.W) if export is not None else self._levels

    @property
    def rows(self):
        return self.h1 - self.h0

    def __call__(self, coords):
        if coords.shape[2] == self.H and self.rows != self.H:
            coords = coords[:, :, self.h0:self.h1]
        coords = coords.contiguous()
        K = (2 * self.radius + 1) ** 2
        if self._levels is None:
            out = coords.new_empty((self.B, self.num_levels * K, 0, self.W))
            # keep the rank in the autograd graph so its backward joins the all-reduce
            return out + self._token if self._token is not None and torch.is_grad_enabled() else out
        if self._token is not None and torch.is_grad_enabled():
            return _ShardLookupFn.apply(coords.detach(), self._token, self.radius, self._st)
        return self.backend.lookup(self._levels, coords, self.radius, self.H, self.W)

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
