"""BASELINE.json's configurations 3, 4 and 5 at their real sizes, on the GPU, checked against the
oracle on SAMPLED queries / pixels so the C oracle stays fast:

  config 3  MVSEC 260x346 padded (36x44 fmaps) and the eval's 256x256 centre crop (32x32), B=16
            (loader/loader_mvsec_flow.py:32-40, config/mvsec_20.json): build + 12 lookups;
  config 4  training step, B=8, D=256, 288x384 crops (36x48 fmaps): CorrBlock forward and
            autograd backward through 12 lookups (eraft_train.py:38-53) — dfmap1 on sampled query
            pixels and dfmap2 on sampled target pixels against dC from the oracle's own
            lookup-backward + pool-backward (model/corr.py:26,58 autograd);
  config 5  1920x1280 (160x240 fmaps, 7.8 GB pyramid), B=1: sampled rows, the lookup bit-exact
            on sampled queries, and G = 8 logical row shards bit-identical to the unsharded build.

Bars: level 0 / gradients within REL_TOL (1e-4 norm-relative, north_star); pooled levels and
lookups bit-exact against the oracle applied to the kernel's own level 0 / pyramid rows.
"""
import numpy as np
import pytest
import torch

import prng
from _util import REL_TOL, bit_equal, norm_rel
from oracle import oracle

pytestmark = pytest.mark.gpu
DEV = "cuda:0"


@pytest.fixture(scope="module", autouse=True)
def _native():
    assert torch.cuda.is_available(), "gpu tests need an MI355X"
    from eraft_amd import _lib
    _lib.load()


def _maps(seed, B, D, H, W):
    f1, f2 = prng.gauss(seed, (B, D, H, W)), prng.gauss(seed + 1, (B, D, H, W))
    return f1, f2, torch.from_numpy(f1).to(DEV), torch.from_numpy(f2).to(DEV)


def _rows(pyr, idx):
    """Pyramid rows (query maps) idx of every level, copied to the host."""
    ix = torch.as_tensor(np.asarray(idx), device=DEV)
    return [p.detach()[ix].cpu().numpy() for p in pyr]


def _check_sampled_build(f1, f2, pyr, sel, H, W):
    B = f1.shape[0]
    N = H * W
    rows = _rows(pyr, sel)
    for k, qi in enumerate(sel):
        b, n = divmod(int(qi), N)
        ref = oracle.corr_rows(f1[b:b + 1], f2[b:b + 1], n, n + 1)[0, 0]
        assert norm_rel(rows[0][k, 0].ravel(), ref) < REL_TOL, qi
    for l in range(1, len(pyr)):  # the fused pyramid = avg_pool2d of the kernel's own rows
        assert bit_equal(oracle.avg_pool2x2(rows[l - 1]), rows[l]), l
    return rows


@pytest.mark.parametrize("H,W", [(36, 44), (32, 32)])
def test_config3_mvsec_b16(H, W):
    from eraft_amd import CorrBlock
    B, D, L, r = 16, 256, 4, 4
    f1, f2, t1, t2 = _maps(301, B, D, H, W)
    cb = CorrBlock(t1, t2, num_levels=L, radius=r)
    N = H * W
    # 32 queries over all 16 batch items, first and last pixels included
    sel = np.unique(np.concatenate([np.linspace(0, B * N - 1, 30).astype(int), [N - 1, N]]))
    _check_sampled_build(f1, f2, cb.corr_pyramid, sel, H, W)
    pyr = [p.cpu().numpy() for p in cb.corr_pyramid]  # 212 MB: the whole pyramid, lookups bit-exact
    for l in range(1, L):
        assert bit_equal(oracle.avg_pool2x2(pyr[l - 1]), pyr[l]), l
    for t in range(12):
        c = prng.lookup_coords(310 + t, B, H, W, 0.5 * t)
        out = cb(torch.from_numpy(c).to(DEV)).cpu().numpy()
        assert bit_equal(out, oracle.lookup(pyr, c, r)), t


def test_config4_train_b8_d256_forward_backward():
    from eraft_amd import CorrBlock
    B, D, H, W, L, r, T = 8, 256, 36, 48, 4, 4, 12
    K = (2 * r + 1) ** 2
    N = H * W
    f1, f2, t1, t2 = _maps(401, B, D, H, W)
    t1.requires_grad_(True)
    t2.requires_grad_(True)
    cb = CorrBlock(t1, t2, num_levels=L, radius=r)
    coords = [prng.lookup_coords(410 + t, B, H, W, 2.0 + t) for t in range(T)]
    grads = [prng.gauss(430 + t, (B, L * K, H, W)) for t in range(T)]
    outs = [cb(torch.from_numpy(c).to(DEV)) for c in coords]
    sel = np.unique(np.linspace(0, B * N - 1, 24).astype(int))
    _check_sampled_build(f1, f2, cb.corr_pyramid, sel, H, W)
    pyr = [p.detach().cpu().numpy() for p in cb.corr_pyramid]
    for t in (0, 5, 11):  # forward lookups of the training step, bit-exact
        assert bit_equal(outs[t].detach().cpu().numpy(), oracle.lookup(pyr, coords[t], r)), t
    torch.autograd.backward(outs, [torch.from_numpy(g).to(DEV) for g in grads])
    df1, df2 = t1.grad.cpu().numpy(), t2.grad.cpu().numpy()
    # dC = d loss / d corr from the oracle (12 lookup-backwards + the pool-backward fold)
    gp = [np.zeros((B * N, 1, H >> l, W >> l), np.float32) for l in range(L)]
    for c, g in zip(coords, grads):
        oracle.lookup_bwd(c, g, gp, r)
    oracle.pool_bwd(gp, H, W)
    dC = gp[0].reshape(B, N, N).astype(np.float64)
    F1 = f1.reshape(B, D, N).astype(np.float64)
    F2 = f2.reshape(B, D, N).astype(np.float64)
    s = np.sqrt(D)
    sc1 = np.abs(df1).max()
    sc2 = np.abs(df2).max()
    for qi in np.unique(np.linspace(0, B * N - 1, 40).astype(int)):
        b, n = divmod(int(qi), N)
        ref1 = F2[b] @ dC[b, n] / s                      # dF1[b][:, n]
        assert np.abs(df1.reshape(B, D, N)[b, :, n] - ref1).max() <= REL_TOL * sc1, qi
        ref2 = F1[b] @ dC[b, :, n] / s                   # dF2[b][:, m = n]
        assert np.abs(df2.reshape(B, D, N)[b, :, n] - ref2).max() <= REL_TOL * sc2, qi


def test_config5_1920x1280_rows_lookup_and_shards():
    from eraft_amd import CorrBlock, _lib
    from eraft_amd.sharded import HipRows, row_partition
    B, D, H, W, L, r = 1, 256, 160, 240, 4, 4
    N = H * W
    f1, f2, t1, t2 = _maps(501, B, D, H, W)
    cb = CorrBlock(t1, t2, num_levels=L, radius=r)
    sel = np.unique(np.concatenate([np.linspace(0, N - 1, 20).astype(int), [W - 1, W, N - W]]))
    rows = _check_sampled_build(f1, f2, cb.corr_pyramid, sel, H, W)
    c = prng.lookup_coords(510, B, H, W, 6.0)
    out = cb(torch.from_numpy(c).to(DEV)).cpu().numpy().reshape(B, L * (2 * r + 1) ** 2, N)
    csel = c.reshape(B, 2, N)[:, :, sel][..., None]          # [1, 2, nsel, 1]
    ref = oracle.lookup_rows(rows, csel, H, W, r)[..., 0]    # the sampled queries' own maps
    assert bit_equal(out[:, :, sel], ref)
    # G = 8 logical row shards (the 8-GPU partition on one device): slab pyramids and lookups
    # bit-identical to the unsharded block on every sampled query of the slab
    tc = torch.from_numpy(c).to(DEV)
    for g in range(8):
        h0, h1 = row_partition(H, 8, g)
        lv = HipRows.build(t1[:, :, h0:h1].contiguous(), t2, L)
        mine = [int(q) for q in sel if h0 * W <= q < h1 * W]
        if mine:
            loc = _rows(_lib.pyramid_export(lv, H, W), [q - h0 * W for q in mine])
            full = _rows(cb.corr_pyramid, mine)
            for l in range(L):
                assert bit_equal(loc[l], full[l]), (g, l)
        o = HipRows.lookup(lv, tc[:, :, h0:h1].contiguous(), r, H, W).cpu().numpy()
        assert bit_equal(o.reshape(B, -1, (h1 - h0) * W), out[:, :, h0 * W:h1 * W]), g
        del lv
        torch.cuda.empty_cache()
