"""Row-sharded CorrBlock (eraft_amd/sharded.py) over a real process group.

CPU tests run world_size 2 and 3 on the gloo backend with an oracle-backed row backend
(tests only — the product backend is HipRows): they check the row partition, the fmap2
broadcast, the all-gather, and that sharded outputs equal the unsharded ones bit for bit.
The GPU test runs the same partition with the HIP *_rows kernels as G logical shards on one
device.
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
        return torch.from_numpy(oracle.lookup_rows(levels, coords_rows.numpy(), H, W, radius))


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, shape, q):
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
        blk = RowShardedCorrBlock(f1, f2, L, r, backend=OracleRows)
        coords = torch.from_numpy(prng.lookup_coords(3, B, H, W, 3.0))
        out_rows = blk(coords)
        full = blk.gather(out_rows)
        q.put((rank, blk.h0, blk.h1, out_rows.numpy(), full.numpy()))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,shape", [(2, (1, 8, 12, 16, 3, 3)), (3, (2, 6, 10, 12, 2, 2))])
def test_row_sharded_matches_unsharded(world, shape):
    B, D, H, W, L, r = shape
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(g, world, port, shape, q)) for g in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    f1, f2 = prng.gauss(1, (B, D, H, W)), prng.gauss(2, (B, D, H, W))
    ref = oracle.lookup(oracle.build_pyramid(f1, f2, L), prng.lookup_coords(3, B, H, W, 3.0), r)
    covered = []
    for rank, h0, h1, rows, full in sorted(res, key=lambda t: t[0]):
        covered += list(range(h0, h1))
        assert bit_equal(rows, ref[:, :, h0:h1])
        assert bit_equal(full, ref)
    assert covered == list(range(H))


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
@pytest.mark.parametrize("algo", ["f16x3", "fp32"])
@pytest.mark.parametrize("G", [1, 2, 3, 8])
def test_row_slab_kernels_match_full_on_gpu(G, algo, monkeypatch):
    """G logical shards on one device through corr_build_ex / corr_lookup_rows."""
    monkeypatch.setenv("ERAFT_AMD_BUILD", algo)
    from eraft_amd import CorrBlock
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
        for l in range(L):
            ref_l = full_blk.corr_pyramid[l].view(B, H, W, -1)[:, h0:h1].reshape(lv[l].shape)
            assert bit_equal(lv[l].cpu().numpy(), ref_l.cpu().numpy())
        out = HipRows.lookup(lv, c[:, :, h0:h1].contiguous(), r, H, W)
        assert bit_equal(out.cpu().numpy(), full[:, :, h0:h1].cpu().numpy())
