"""Generate the golden fixtures in tests/golden/*.npz FROM THE REFERENCE ITSELF.

Run in the survey container only (needs /root/reference, never present on the GPU box):

    PYTHONDONTWRITEBYTECODE=1 python tests/golden/make_golden.py

It imports the reference's own CorrBlock (model/corr.py:12-60) and coords_grid
(model/utils.py:24-27), feeds it inputs from tests/golden/prng.py (portable; only seeds are
stored) and records its outputs.  The fixtures are data (inputs' seeds + reference outputs),
never reference source.  Backward goldens come from the reference under torch autograd.
"""
from __future__ import annotations

import os
import sys
import warnings

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import prng  # noqa: E402

REF = "/root/reference"
sys.dont_write_bytecode = True
sys.path.insert(0, REF)
warnings.filterwarnings("ignore")
from model.corr import CorrBlock  # noqa: E402  (reference)

torch.set_num_threads(8)


def fmaps(seed, B, D, H, W):
    return prng.gauss(seed, (B, D, H, W)), prng.gauss(seed + 1, (B, D, H, W))


def ref_build(f1, f2, L, r):
    return CorrBlock(torch.from_numpy(f1), torch.from_numpy(f2), num_levels=L, radius=r)


def save(name, **arrs):
    path = os.path.join(HERE, name + ".npz")
    np.savez_compressed(path, **arrs)
    print(f"{name}: {os.path.getsize(path) / 1e6:.2f} MB")


def case_build_lookup(name, seed, B, D, H, W, L, r, sigmas, store_pyramid=True):
    f1, f2 = fmaps(seed, B, D, H, W)
    cb = ref_build(f1, f2, L, r)
    out = {"meta": np.array([seed, B, D, H, W, L, r], np.int64),
           "sigmas": np.array(sigmas, np.float32)}
    if store_pyramid:
        for l, p in enumerate(cb.corr_pyramid):
            out[f"pyr{l}"] = p.numpy()
    corr6 = CorrBlock.corr(torch.from_numpy(f1), torch.from_numpy(f2))
    out["corr_shape"] = np.array(corr6.shape, np.int64)
    for k, s in enumerate(sigmas):
        c = prng.lookup_coords(seed + 100 + k, B, H, W, s)
        out[f"coords{k}"] = c
        out[f"look{k}"] = cb(torch.from_numpy(c)).numpy()
    c = prng.special_coords(B, H, W)
    out["coords_special"] = c
    out["look_special"] = cb(torch.from_numpy(c)).numpy()
    save(name, **out)


def case_backward(name, seed, B, D, H, W, L, r, iters):
    f1, f2 = fmaps(seed, B, D, H, W)
    t1 = torch.from_numpy(f1).requires_grad_(True)
    t2 = torch.from_numpy(f2).requires_grad_(True)
    cb = CorrBlock(t1, t2, num_levels=L, radius=r)
    K = (2 * r + 1) ** 2
    loss = 0.0
    for t in range(iters):
        c = prng.lookup_coords(seed + 200 + t, B, H, W, 2.0 + t)
        g = prng.gauss(seed + 300 + t, (B, L * K, H, W))
        o = cb(torch.from_numpy(c))
        loss = loss + (o * torch.from_numpy(g)).sum()
    loss.backward()
    save(name, meta=np.array([seed, B, D, H, W, L, r, iters], np.int64),
         df1=t1.grad.numpy(), df2=t2.grad.numpy())


def case_dsec_spot(name, seed):
    """DSEC shape (B=1, 60x80, D=256): slices + fp64 checksums only (full pyramid is 122 MB)."""
    B, D, H, W, L, r = 1, 256, 60, 80, 4, 4
    f1, f2 = fmaps(seed, B, D, H, W)
    cb = ref_build(f1, f2, L, r)
    q = np.array([0, 1, 79, 80, 2399, 2400, 4719, 4799, 1234, 3000, 4321, 17, 555, 2048, 3333, 4000])
    out = {"meta": np.array([seed, B, D, H, W, L, r], np.int64), "q": q}
    for l, p in enumerate(cb.corr_pyramid):
        p = p.numpy()
        out[f"pyr{l}_rows"] = p[q]
        out[f"pyr{l}_sum"] = np.array([p.astype(np.float64).sum(), np.abs(p).astype(np.float64).sum()])
    c = prng.lookup_coords(seed + 100, B, H, W, 8.0)
    o = cb(torch.from_numpy(c)).numpy()
    out["look_q"] = o.reshape(B, -1, H * W)[:, :, q]
    out["look_sum"] = np.array([o.astype(np.float64).sum(), np.abs(o).astype(np.float64).sum()])
    save(name, **out)


def init_model(model):
    sd = model.state_dict()
    with torch.no_grad():
        for name, t in sd.items():
            v = prng.param_init(name, tuple(t.shape))
            if v is not None:
                t.copy_(torch.from_numpy(v))


def case_e2e(name, seed, H=480, W=640, bins=15, iters=12):
    """Full reference E-RAFT forward (model/eraft.py:89-146), random weights from
    prng.param_init, cold call then warm-start call with the reference's own forward splat
    (utils/image_utils.py:52-83, test.py:209).  flow_up is stored every 4th pixel."""
    from model.eraft import ERAFT
    from utils.image_utils import forward_interpolate_pytorch
    model = ERAFT({"subtype": "warm_start"}, n_first_channels=bins).eval()
    init_model(model)
    im1 = torch.from_numpy(prng.voxel_grid(seed, (1, bins, H, W)))
    im2 = torch.from_numpy(prng.voxel_grid(seed + 2, (1, bins, H, W)))
    with torch.no_grad():
        low, ups = model(im1, im2, iters=iters)
        finit = forward_interpolate_pytorch(low)
        model2 = ERAFT({"subtype": "warm_start"}, n_first_channels=bins).eval()
        init_model(model2)
        low_w, ups_w = model2(im1, im2, iters=iters, flow_init=finit)
    keys = [f"{k}:{tuple(v.shape)}" for k, v in model.state_dict().items()]
    save(name, meta=np.array([seed, H, W, bins, iters], np.int64), state_keys=np.array(keys),
         low=low.numpy(), up_sub=ups[-1][..., ::4, ::4].numpy(),
         up_mean_abs=np.array([ups[-1].abs().mean().item()]),
         flow_init=finit.numpy(), low_warm=low_w.numpy(), up_warm_sub=ups_w[-1][..., ::4, ::4].numpy())


def case_splat(name, seed):
    """Warm-start forward splat (utils/image_utils.py:10-83, forward_interpolate_pytorch):
    flows with fractional, exactly-integer (floor == ceil: the reference counts that corner
    twice), out-of-bounds and colliding targets; B = 2 at 17 x 23 and B = 1 at 60 x 80."""
    from utils.image_utils import forward_interpolate_pytorch
    out = {}
    cases = [("a", 2, 17, 23, 3.0), ("b", 1, 60, 80, 6.0)]
    for tag, B, H, W, sig in cases:
        f = prng.gauss(seed, (B, 2, H, W), sig)
        f[:, :, ::4, ::3] = np.round(f[:, :, ::4, ::3])          # integer displacements
        f[0, 0, 1, :5] = [40.0, -40.0, 0.0, -0.5, 1e4]           # far out / exact / half
        f[0, 1, 2, :4] = [0.0, 0.0, -3.0, 2.5]
        f[0, :, 3, :6] = 0.0                                     # several sources, one target
        out[f"flow_{tag}"] = f
        out[f"splat_{tag}"] = forward_interpolate_pytorch(torch.from_numpy(f)).numpy()
        seed += 1
    save(name, **out)


def case_voxel(name, seed):
    """DSEC event -> voxel grid (utils/dsec_utils.py:19-64 VoxelGrid.convert, normalize=True
    and False) on events shaped as loader_dsec.py:245-257 makes them: float32 rectified x, y
    (fractional, some out of the frame), t normalised to [0, 1], p in {0, 1}; repeated pixels
    collide.  Inputs from prng; outputs from the reference, run single-threaded as its own
    entry point pins it (main.py:2-5): put_(accumulate=True) on CPU is chunked over threads,
    so its summation order (and the low bits) depend on the thread count; one thread = the
    sequential event order."""
    from utils.dsec_utils import VoxelGrid
    torch.set_num_threads(1)
    out = {}
    for tag, M, C, H, W in (("a", 3000, 5, 12, 16), ("b", 40000, 15, 48, 64)):
        u = prng.uniform(seed, (4, M))
        x = (u[0] * (W + 2) - 1.0).astype(np.float32)
        y = (u[1] * (H + 2) - 1.0).astype(np.float32)
        x[::7] = np.floor(x[::7])                       # integer coordinates
        t = np.sort(u[2]).astype(np.float32)
        t = (t - t[0]) / (t[-1] - t[0])
        p = (u[3] > 0.5).astype(np.float32)
        ev = {k: torch.from_numpy(v.copy()) for k, v in (("x", x), ("y", y), ("t", t), ("p", p))}
        out[f"ev_{tag}"] = np.stack([x, y, t, p])
        out[f"meta_{tag}"] = np.array([M, C, H, W], np.int64)
        out[f"raw_{tag}"] = VoxelGrid((C, H, W), normalize=False).convert(ev).numpy()
        out[f"norm_{tag}"] = VoxelGrid((C, H, W), normalize=True).convert(ev).numpy()
        seed += 1
    save(name, **out)


def case_voxel_mvsec(name, seed):
    """MVSEC event -> voxel grid (utils/transformers.py:18-126 EventSequenceToVoxelGrid_Pytorch,
    the representation of loader/loader_mvsec_flow.py:35), normalize=True and False.  Events
    as the MVSEC loader holds them: [M, 4] float64 rows (t, x, y, p) with integer pixel
    coordinates, t ascending relative microsecond stamps, p in {0, 1}; duplicated stamps, the
    first/last bins and colliding pixels are included, and case "c" has all stamps equal
    (deltaT = 0 -> 1).  index_add_ on CPU adds sequentially in index order, so the thread
    count does not matter; run single-threaded anyway as main.py:2-5 does."""
    import types
    from utils.transformers import EventSequenceToVoxelGrid_Pytorch
    torch.set_num_threads(1)
    out = {}
    for tag, M, C, H, W in (("a", 3000, 5, 12, 16), ("b", 60000, 15, 260, 346), ("c", 500, 3, 8, 8)):
        u = prng.uniform(seed, (4, M)).astype(np.float64)
        x = np.floor(u[0] * W)
        y = np.floor(u[1] * H)
        t = np.sort(u[2] * 50000.0)          # relative microseconds (loader_mvsec_flow.py:170-172)
        t[::5] = np.floor(t[::5])             # some integer stamps
        t[10:20] = t[10]                      # repeated stamps
        if tag == "c":
            t[:] = 12345.0
        p = (u[3] > 0.5).astype(np.float64)
        ev = np.ascontiguousarray(np.stack([t, x, y, p], axis=1))
        seq = types.SimpleNamespace(features=ev, image_width=W, image_height=H)
        out[f"ev_{tag}"] = ev
        out[f"meta_{tag}"] = np.array([M, C, H, W], np.int64)
        for norm, key in ((False, "raw"), (True, "norm")):
            conv = EventSequenceToVoxelGrid_Pytorch(C, gpu=False, normalize=norm, forkserver=False)
            out[f"{key}_{tag}"] = conv(seq).numpy()
        seed += 1
    save(name, **out)


if __name__ == "__main__":
    if len(sys.argv) > 1 and sys.argv[1] == "voxel_mvsec":
        case_voxel_mvsec("g_voxel_mvsec", 51)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "voxel":
        case_voxel("g_voxel", 41)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "splat":
        case_splat("g_splat", 31)
        sys.exit(0)
    if len(sys.argv) > 1 and sys.argv[1] == "e2e":
        case_e2e("g_e2e_dsec", 21)
        sys.exit(0)
    case_build_lookup("g_b1_d32_16x16", 11, 1, 32, 16, 16, 4, 4, [0.0, 3.0, 20.0])
    case_build_lookup("g_b2_d256_17x23", 12, 2, 256, 17, 23, 4, 4, [8.0])
    case_build_lookup("g_b2_d64_16x20_L2r3", 13, 2, 64, 16, 20, 2, 3, [5.0])
    case_build_lookup("g_degenerate_b1_d32_12x16", 14, 1, 32, 12, 16, 4, 4, [3.0])
    case_build_lookup("g_degenerate_b1_d16_15x21", 15, 1, 16, 15, 21, 4, 4, [3.0])
    case_backward("g_bwd_b2_d16_18x24", 16, 2, 16, 18, 24, 4, 4, 12)
    case_backward("g_bwd_b1_d32_17x23_L2r3", 17, 1, 32, 17, 23, 2, 3, 3)
    case_dsec_spot("g_dsec_spot", 18)
