"""Row-sharded CorrBlock (eraft_amd/sharded.py) over a real process group.

CPU tests run world_size 2 and 3 on the gloo backend with an oracle-backed row backend
(tests only — the product backend is HipRows): they check the row partition, the fmap2
broadcast, the all-gather, and that sharded outputs equal the unsharded ones bit for bit.
The GPU tests run the same partition with the HIP *_rows kernels as G logical shards on one
device, and as two real processes sharing the device (gloo carrying the CUDA tensors).
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import prng
from _util import bit_equal
from oracle import oracle


class OracleRows:
    """CPU row-slab backend built on the oracle (test infrastructure)."""

    @staticmethod
    def build(f1_rows, f2, num_levels):
        B, D, rows, W = f1_rows.shape
        H = f2.shape[2]
        # place the slab in a full-size map and compute just its query rows
        full = np.zeros((B, D, H, W), np.float32)
        h0 = OracleRows.h0
        full[:, :, h0:h0 + rows] = f1_rows.numpy()
        c = oracle.corr_rows(full, f2.numpy(), h0 * W, (h0 + rows) * W)
        lv = [c.reshape(B * rows * W, 1, H, W)]
        for _ in range(num_levels - 1):
            lv.append(oracle.avg_pool2x2(lv[-1]))
        return lv

    @staticmethod
    def lookup(levels, coords_rows, radius, H, W):
        return torch.from_numpy(oracle.lookup_rows(levels, np.asarray(coords_rows.detach()), H, W, radius))

    # target-row regions (the chunked broadcast): the chunks are gathered into a full map and
    # the slab's pyramid is computed when the last one has arrived
    chunked_regions = 0  # regions built (test bookkeeping)

    @staticmethod
    def region_supported(num_levels):
        return True

    @staticmethod
    def region_begin(f1_rows, f2_shape, num_levels):
        return [], {"f2": torch.zeros(f2_shape), "rows": 0, "L": num_levels}

    @staticmethod
    def build_region(f1_rows, f2_chunk, y0, y1, H, levels, st, first):
        assert first == (st["rows"] == 0) and y0 % 8 == 0
        st["f2"][:, :, y0:y1] = f2_chunk
        st["rows"] += y1 - y0
        OracleRows.chunked_regions += 1
        if st["rows"] == H:
            levels[:] = OracleRows.build(f1_rows, st["f2"], st["L"])

    # backward: the slab is embedded in a full-size problem whose other query rows carry zero
    # gradient, so the oracle's full-map backward gives exactly the slab's contributions

    @staticmethod
    def zero_pyramid(B, NQ, H, W, num_levels, like):
        return [torch.zeros(B * NQ, 1, H >> l, W >> l) for l in range(num_levels)]

    @staticmethod
    def lookup_bwd(coords_rows, grad_rows, radius, grad_levels, H, W):
        B, _, rows, _ = coords_rows.shape
        h0 = OracleRows.h0
        fc = np.zeros((B, 2, H, W), np.float32)
        fc[:, :, h0:h0 + rows] = coords_rows.numpy()
        fg = np.zeros((B, grad_rows.shape[1], H, W), np.float32)
        fg[:, :, h0:h0 + rows] = grad_rows.numpy()
        gp = [np.zeros((B * H * W, 1, H >> l, W >> l), np.float32) for l in range(len(grad_levels))]
        oracle.lookup_bwd(fc, fg, gp, radius)
        for acc, g in zip(grad_levels, gp):
            part = g.reshape(B, H * W, -1)[:, h0 * W:(h0 + rows) * W].reshape(acc.shape)
            acc += torch.from_numpy(np.ascontiguousarray(part))

    @staticmethod
    def pool_bwd(grad_levels, H, W):
        oracle.pool_bwd([g.numpy() for g in grad_levels], H, W)

    @staticmethod
    def build_bwd(grad_c, f1_rows, f2):
        B, D, rows, W = f1_rows.shape
        H = f2.shape[2]
        h0 = OracleRows.h0
        gc = np.zeros((B, H * W, H * W), np.float32)
        gc[:, h0 * W:(h0 + rows) * W] = grad_c.numpy().reshape(B, rows * W, H * W)
        f1 = np.zeros((B, D, H, W), np.float32)
        f1[:, :, h0:h0 + rows] = f1_rows.detach().numpy()
        df1, df2 = oracle.corr_bwd(gc.reshape(B * H * W, H * W), f1, f2.detach().numpy())
        return torch.from_numpy(np.ascontiguousarray(df1[:, :, h0:h0 + rows])), torch.from_numpy(df2)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, shape, q, chunks=1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from eraft_amd.sharded import RowShardedCorrBlock, row_partition

        B, D, H, W, L, r = shape
        f1 = torch.from_numpy(prng.gauss(1, (B, D, H, W)))
        # only rank 0 holds the real fmap2; the others must receive it by broadcast
        f2 = torch.from_numpy(prng.gauss(2, (B, D, H, W))) if rank == 0 else torch.zeros(B, D, H, W)
        OracleRows.h0 = row_partition(H, world, rank)[0]
        OracleRows.chunked_regions = 0
        blk = RowShardedCorrBlock(f1, f2, L, r, backend=OracleRows, chunks=chunks)
        coords = torch.from_numpy(prng.lookup_coords(3, B, H, W, 3.0))
        out_rows = blk(coords)
        full = blk.gather(out_rows)
        # the broadcast's contract holds with chunks too: every rank's fmap2 is rank 0's
        assert np.array_equal(f2.numpy(), prng.gauss(2, (B, D, H, W)))
        q.put((rank, blk.h0, blk.h1, out_rows.numpy(), full.numpy(), OracleRows.chunked_regions))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,shape,chunks", [(2, (1, 8, 12, 16, 3, 3), 1), (3, (2, 6, 10, 12, 2, 2), 1),
                                                (2, (1, 8, 24, 16, 3, 3), 3), (3, (2, 6, 20, 12, 3, 2), 4)])
def test_row_sharded_matches_unsharded(world, shape, chunks):
    """Row partition + fmap2 broadcast (one blocking broadcast, or target-row chunks each built
    on arrival: SURVEY §8e's overlap) + slab lookups + gather, bit-identical to unsharded."""
    B, D, H, W, L, r = shape
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(g, world, port, shape, q, chunks)) for g in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    f1, f2 = prng.gauss(1, (B, D, H, W)), prng.gauss(2, (B, D, H, W))
    ref = oracle.lookup(oracle.build_pyramid(f1, f2, L), prng.lookup_coords(3, B, H, W, 3.0), r)
    covered = []
    from eraft_amd.sharded import chunk_bounds
    for rank, h0, h1, rows, full, regions in sorted(res, key=lambda t: t[0]):
        covered += list(range(h0, h1))
        assert bit_equal(rows, ref[:, :, h0:h1])
        assert bit_equal(full, ref)
        # the chunked path built every chunk as its own region (ranks with rows)
        assert regions == (len(chunk_bounds(H, chunks)) if chunks > 1 and h1 > h0 else 0)
    assert covered == list(range(H))


def _pipe_worker(rank, world, port, shape, npairs, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from eraft_amd.sharded import Fmap2DoubleBuffer, RowShardedCorrBlock, row_partition

        B, D, H, W, L, r = shape
        OracleRows.h0 = row_partition(H, world, rank)[0]
        dbuf = Fmap2DoubleBuffer((B, D, H, W), "cpu")
        # pair k's fmap2 exists only on rank 0 (seed 100 + k); the next pair's broadcast is
        # issued before the current pair is built
        src = lambda k: torch.from_numpy(prng.gauss(100 + k, (B, D, H, W))) if rank == 0 else None  # noqa: E731
        with torch.no_grad():  # prefetch is inference-only
            pending = dbuf.prefetch(src(0))
        outs = []
        for k in range(npairs):
            with torch.no_grad():
                nxt = dbuf.prefetch(src(k + 1)) if k + 1 < npairs else None
            f1 = torch.from_numpy(prng.gauss(200 + k, (B, D, H, W)))
            blk = RowShardedCorrBlock(f1, pending, L, r, backend=OracleRows)
            coords = torch.from_numpy(prng.lookup_coords(300 + k, B, H, W, 3.0))
            outs.append(blk.gather(blk(coords)).numpy())
            pending = nxt
        q.put((rank, outs))
    finally:
        dist.destroy_process_group()


def test_row_sharded_prefetch_pipeline():
    """The product API for a stream of pairs: Fmap2DoubleBuffer.prefetch issues pair k+1's
    fmap2 broadcast before pair k is built (double-buffered), RowShardedCorrBlock waits on it.
    Every pair's gathered output is bit-identical to the unsharded block."""
    world, npairs = 2, 3
    shape = B, D, H, W, L, r = (1, 8, 12, 16, 3, 3)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_worker, args=(g, world, port, shape, npairs, q)) for g in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for k in range(npairs):
        f1, f2 = prng.gauss(200 + k, (B, D, H, W)), prng.gauss(100 + k, (B, D, H, W))
        ref = oracle.lookup(oracle.build_pyramid(f1, f2, L), prng.lookup_coords(300 + k, B, H, W, 3.0), r)
        for _, outs in res:
            assert bit_equal(outs[k], ref)


def _pipe_train_worker(rank, world, port, q):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from eraft_amd.sharded import Fmap2DoubleBuffer, RowShardedCorrBlock, row_partition

        B, D, H, W, L, r = 1, 4, 8, 8, 2, 1
        OracleRows.h0 = row_partition(H, world, rank)[0]
        dbuf = Fmap2DoubleBuffer((B, D, H, W), "cpu")
        f2 = torch.from_numpy(prng.gauss(5, (B, D, H, W))).requires_grad_(True)
        errs = []
        try:  # every rank refuses a prefetch with autograd enabled (before any collective)
            dbuf.prefetch(f2 if rank == 0 else None).wait()
            errs.append("prefetch accepted")
        except RuntimeError:
            errs.append("prefetch refused")
        with torch.no_grad():
            pending = dbuf.prefetch(f2 if rank == 0 else None)
        f1 = torch.from_numpy(prng.gauss(6, (B, D, H, W))).requires_grad_(True)
        try:  # every rank refuses a prefetched fmap2 for a block that trains
            RowShardedCorrBlock(f1, pending, L, r, backend=OracleRows)
            errs.append("block accepted")
        except RuntimeError:
            errs.append("block refused")
        with torch.no_grad():  # inference through the same pending buffer still works
            blk = RowShardedCorrBlock(f1, pending, L, r, backend=OracleRows)
            out = blk.gather(blk(torch.from_numpy(prng.lookup_coords(7, B, H, W, 1.0))))
        q.put((rank, errs, out.numpy()))
    finally:
        dist.destroy_process_group()


def test_row_sharded_prefetch_rejects_training():
    """Fmap2DoubleBuffer / PendingFmap2 are inference-only: every rank's prefetch refuses while
    autograd is enabled (the same decision on every rank, taken before the collective), every
    rank refuses to build a training block from a prefetched fmap2 (no rank is left waiting in a
    gradient all-reduce), and no-grad use is unaffected."""
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_pipe_train_worker, args=(g, world, port, q)) for g in range(world)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=120) for _ in range(world)], key=lambda t: t[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    assert res[0][1] == ["prefetch refused", "block refused"]
    assert res[1][1] == ["prefetch refused", "block refused"]
    ref = oracle.lookup(oracle.build_pyramid(prng.gauss(6, (1, 4, 8, 8)), prng.gauss(5, (1, 4, 8, 8)), 2),
                        prng.lookup_coords(7, 1, 8, 8, 1.0), 1)
    for _, _, out in res:
        assert bit_equal(out, ref)


def _train_worker(rank, world, port, shape, q, chunks=1):
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from eraft_amd.sharded import RowShardedCorrBlock, row_partition

        B, D, H, W, L, r, T = shape
        f1 = torch.from_numpy(prng.gauss(1, (B, D, H, W))).requires_grad_(True)
        f2 = torch.from_numpy(prng.gauss(2, (B, D, H, W))).requires_grad_(True)
        h0, h1 = row_partition(H, world, rank)
        OracleRows.h0 = h0
        blk = RowShardedCorrBlock(f1, f2, L, r, backend=OracleRows, chunks=chunks)
        loss = 0
        for t in range(T):
            c = torch.from_numpy(prng.lookup_coords(10 + t, B, H, W, 3.0))
            g = torch.from_numpy(prng.gauss(20 + t, (B, L * (2 * r + 1) ** 2, H, W)))
            loss = loss + (blk(c) * g[:, :, h0:h1]).sum()
        loss.backward()
        q.put((rank, h0, h1, f1.grad.numpy(), f2.grad.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,shape,chunks", [(2, (1, 8, 12, 16, 3, 3, 2), 1), (3, (2, 6, 8, 12, 2, 2, 3), 1),
                                                (3, (1, 4, 2, 8, 1, 1, 2), 1),  # rank 2 owns no rows
                                                (2, (1, 8, 24, 16, 3, 3, 2), 3),  # chunked fmap2 broadcast
                                                (3, (1, 4, 17, 8, 2, 1, 2), 2)])
def test_row_sharded_training_grads(world, shape, chunks):
    """dfmap1 rows are rank-local; dfmap2 = all-reduce of the slab partials == unsharded (also
    with the chunked fmap2 broadcast inside the build's autograd forward)."""
    B, D, H, W, L, r, T = shape
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_train_worker, args=(g, world, port, shape, q, chunks)) for g in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    f1, f2 = prng.gauss(1, (B, D, H, W)), prng.gauss(2, (B, D, H, W))
    K = (2 * r + 1) ** 2
    cl = [prng.lookup_coords(10 + t, B, H, W, 3.0) for t in range(T)]
    gl = [prng.gauss(20 + t, (B, L * K, H, W)) for t in range(T)]
    rdf1, rdf2 = oracle.fmap_grads(f1, f2, cl, gl, L, r)
    for rank, h0, h1, g1, g2 in res:
        # full replicated fmap1: every rank holds the all-reduced (single-GPU) dfmap1 and dfmap2
        assert np.abs(g1 - rdf1).max() <= 1e-5 * np.abs(rdf1).max()
        assert np.abs(g2 - rdf2).max() <= 1e-5 * np.abs(rdf2).max()


def _encoder_worker(rank, world, port, shape, q):
    """A shared (replicated) encoder produces both fmaps; after backward through the sharded
    block every rank's parameter gradients must equal the single-GPU ones."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from eraft_amd.sharded import RowShardedCorrBlock, row_partition

        B, D, H, W, L, r, T = shape
        enc = _encoder(D)
        im1, im2 = (torch.from_numpy(prng.gauss(s, (B, 3, H, W))) for s in (31, 32))
        f1, f2 = enc(im1), enc(im2)
        h0, h1 = row_partition(H, world, rank)
        OracleRows.h0 = h0
        blk = RowShardedCorrBlock(f1, f2, L, r, backend=OracleRows, broadcast=False)
        loss = 0
        for t in range(T):
            c = torch.from_numpy(prng.lookup_coords(10 + t, B, H, W, 3.0))
            g = torch.from_numpy(prng.gauss(20 + t, (B, L * (2 * r + 1) ** 2, H, W)))
            loss = loss + (blk(c) * g[:, :, h0:h1]).sum()
        loss.backward()
        q.put((rank, [p.grad.numpy().copy() for p in enc.parameters()]))
    finally:
        dist.destroy_process_group()


def _encoder(D):
    torch.manual_seed(5)
    return torch.nn.Sequential(torch.nn.Conv2d(3, D, 3, padding=1), torch.nn.Tanh())


def test_row_sharded_encoder_param_grads():
    """with fmap1 and fmap2 from one shared encoder, the sharded backward gives every
    rank the single-GPU parameter gradients (dfmap1 and dfmap2 both SUM-all-reduced)."""
    from oracle import torch_ops
    world, shape = 2, (1, 6, 10, 12, 3, 2, 2)
    B, D, H, W, L, r, T = shape
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_encoder_worker, args=(g, world, port, shape, q)) for g in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    enc = _encoder(D)
    im1, im2 = (torch.from_numpy(prng.gauss(s, (B, 3, H, W))) for s in (31, 32))
    lv = torch_ops.cpu_build(enc(im1), enc(im2), L)
    loss = 0
    for t in range(T):
        c = torch.from_numpy(prng.lookup_coords(10 + t, B, H, W, 3.0))
        g = torch.from_numpy(prng.gauss(20 + t, (B, L * (2 * r + 1) ** 2, H, W)))
        loss = loss + (torch_ops.cpu_lookup(lv, c, r) * g).sum()
    loss.backward()
    ref = [p.grad.numpy() for p in enc.parameters()]
    for rank, grads in res:
        for a, b in zip(grads, ref):
            assert np.abs(a - b).max() <= 1e-5 * np.abs(b).max(), rank


def _gpu_worker(rank, world, port, shape, q, chunks=1):
    """HIP row kernels in world processes sharing cuda:0 (gloo carries the CUDA tensors: RCCL
    refuses two ranks on one device): broadcast of fmap2, slab build + lookups, the gather, and
    the training backward with both fmap gradients all-reduced."""
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from eraft_amd.sharded import RowShardedCorrBlock, row_partition

        B, D, H, W, L, r, T = shape
        dev = "cuda:0"
        f1 = torch.from_numpy(prng.gauss(1, (B, D, H, W))).to(dev).requires_grad_(True)
        f2 = (torch.from_numpy(prng.gauss(2, (B, D, H, W))) if rank == 0 else torch.zeros(B, D, H, W)).to(dev)
        f2.requires_grad_(True)
        h0, h1 = row_partition(H, world, rank)
        blk = RowShardedCorrBlock(f1, f2, L, r, chunks=chunks)
        K = (2 * r + 1) ** 2
        loss, outs = 0, []
        for t in range(T):
            c = torch.from_numpy(prng.lookup_coords(40 + t, B, H, W, 2.0)).to(dev)
            g = torch.from_numpy(prng.gauss(50 + t, (B, L * K, H, W))).to(dev)
            o = blk(c)
            outs.append(o.detach().cpu().numpy())
            loss = loss + (o * g[:, :, h0:h1]).sum()
        full = blk.gather(torch.from_numpy(outs[-1]).to(dev)).cpu().numpy()
        loss.backward()
        torch.cuda.synchronize()
        q.put((rank, h0, h1, outs, full, f1.grad.cpu().numpy(), f2.grad.cpu().numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("chunks", [1, 2])
def test_row_sharded_multiprocess_on_gpu(chunks):
    """Two processes on the MI355X through the product backend (HipRows): lookup rows and the
    gathered output bit-identical to the one-process CorrBlock; training gradients (both
    all-reduced) within 1e-5 of it.  chunks = 2: fmap2 broadcast as two target-row chunks, each
    built by corr_build_region as it arrives."""
    from eraft_amd import CorrBlock
    world, shape = 2, (2, 32, 18, 24, 4, 4, 3)
    B, D, H, W, L, r, T = shape
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_gpu_worker, args=(g, world, port, shape, q, chunks)) for g in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    dev = "cuda:0"
    K = (2 * r + 1) ** 2
    t1 = torch.from_numpy(prng.gauss(1, (B, D, H, W))).to(dev).requires_grad_(True)
    t2 = torch.from_numpy(prng.gauss(2, (B, D, H, W))).to(dev).requires_grad_(True)
    cb = CorrBlock(t1, t2, L, r)
    loss, ref = 0, []
    for t in range(T):
        c = torch.from_numpy(prng.lookup_coords(40 + t, B, H, W, 2.0)).to(dev)
        g = torch.from_numpy(prng.gauss(50 + t, (B, L * K, H, W))).to(dev)
        o = cb(c)
        ref.append(o.detach().cpu().numpy())
        loss = loss + (o * g).sum()
    loss.backward()
    d1, d2 = t1.grad.cpu().numpy(), t2.grad.cpu().numpy()
    for rank, h0, h1, outs, full, g1, g2 in res:
        for o, rf in zip(outs, ref):
            assert bit_equal(o, rf[:, :, h0:h1]), rank
        assert bit_equal(full, ref[-1]), rank
        assert np.abs(g1 - d1).max() <= 1e-5 * np.abs(d1).max(), rank
        assert np.abs(g2 - d2).max() <= 1e-5 * np.abs(d2).max(), rank


def test_row_partition_covers_rows():
    from eraft_amd.sharded import row_partition
    for H in (1, 7, 60, 160):
        for world in (1, 2, 3, 4, 8):
            rows = []
            for g in range(world):
                h0, h1 = row_partition(H, world, g)
                assert 0 <= h0 <= h1 <= H
                rows += list(range(h0, h1))
            assert rows == list(range(H))


@pytest.mark.gpu
@pytest.mark.parametrize("algo", ["bf16x6", "f16x3", "fp32"])
@pytest.mark.parametrize("G", [1, 2, 3, 8])
def test_row_slab_kernels_match_full_on_gpu(G, algo, monkeypatch):
    """G logical shards on one device through corr_build_ex / corr_lookup_rows."""
    monkeypatch.setenv("ERAFT_AMD_BUILD", algo)
    from eraft_amd import CorrBlock, _lib
    from eraft_amd.sharded import HipRows, row_partition
    B, D, H, W, L, r = 2, 64, 20, 24, 4, 4
    dev = "cuda:0"
    f1 = torch.from_numpy(prng.gauss(1, (B, D, H, W))).to(dev)
    f2 = torch.from_numpy(prng.gauss(2, (B, D, H, W))).to(dev)
    c = torch.from_numpy(prng.lookup_coords(3, B, H, W, 4.0)).to(dev)
    full_blk = CorrBlock(f1, f2, L, r)
    full = full_blk(c)
    for g in range(G):
        h0, h1 = row_partition(H, G, g)
        if h1 == h0:
            continue
        lv = HipRows.build(f1[:, :, h0:h1].contiguous(), f2, L)
        ex = _lib.pyramid_export(lv, H, W)  # the slab's maps in the reference layout
        for l in range(L):
            ref_l = full_blk.corr_pyramid[l].view(B, H, W, -1)[:, h0:h1].reshape(ex[l].shape)
            assert bit_equal(ex[l].cpu().numpy(), ref_l.cpu().numpy())
        out = HipRows.lookup(lv, c[:, :, h0:h1].contiguous(), r, H, W)
        assert bit_equal(out.cpu().numpy(), full[:, :, h0:h1].cpu().numpy())


@pytest.mark.gpu
@pytest.mark.parametrize("G", [2, 3])
def test_row_slab_backward_on_gpu(G):
    """Slab backward through the HIP *_rows kernels (lookup_bwd_rows, pool_bwd, build_bwd_rows)
    as G logical shards: dfmap1 rows match the unsharded autograd, and the sum of the slab
    partial dfmap2 (what the all-reduce forms) matches its dfmap2."""
    from eraft_amd import CorrBlock
    from eraft_amd.sharded import HipRows, row_partition
    B, D, H, W, L, r, T = 2, 64, 20, 24, 4, 4, 3
    dev = "cuda:0"
    f1 = torch.from_numpy(prng.gauss(1, (B, D, H, W))).to(dev).requires_grad_(True)
    f2 = torch.from_numpy(prng.gauss(2, (B, D, H, W))).to(dev).requires_grad_(True)
    K = (2 * r + 1) ** 2
    cl = [torch.from_numpy(prng.lookup_coords(10 + t, B, H, W, 3.0)).to(dev) for t in range(T)]
    gl = [torch.from_numpy(prng.gauss(20 + t, (B, L * K, H, W))).to(dev) for t in range(T)]
    blk = CorrBlock(f1, f2, L, r)
    loss = sum((blk(c) * g).sum() for c, g in zip(cl, gl))
    loss.backward()
    rdf1, rdf2 = f1.grad.cpu().numpy(), f2.grad.cpu().numpy()
    df1 = np.zeros_like(rdf1)
    df2 = np.zeros_like(rdf2)
    with torch.no_grad():
        for g in range(G):
            h0, h1 = row_partition(H, G, g)
            f1s = f1[:, :, h0:h1].contiguous()
            gp = HipRows.zero_pyramid(B, (h1 - h0) * W, H, W, L, f2)
            for c, go in zip(cl, gl):
                HipRows.lookup_bwd(c[:, :, h0:h1].contiguous(), go[:, :, h0:h1].contiguous(), r, gp, H, W)
            HipRows.pool_bwd(gp, H, W)
            d1, d2 = HipRows.build_bwd(gp[0], f1s, f2)
            df1[:, :, h0:h1] = d1.cpu().numpy()
            df2 += d2.cpu().numpy()
    assert np.abs(df1 - rdf1).max() <= 1e-4 * np.abs(rdf1).max()
    assert np.abs(df2 - rdf2).max() <= 1e-4 * np.abs(rdf2).max()
