"""Shared helpers for the test-suite (fixture loading, parity metrics)."""
import os

import numpy as np

GOLDEN = os.path.join(os.path.dirname(os.path.abspath(__file__)), "golden")

# north_star: "fp32 correlation and lookup within 1e-4 relative", defined as the
# norm-relative error ||a - b||_inf / ||b||_inf.
REL_TOL = 1e-4


def load(name):
    return dict(np.load(os.path.join(GOLDEN, name + ".npz"), allow_pickle=False))


def golden_names(prefix="g_"):
    return sorted(f[:-4] for f in os.listdir(GOLDEN) if f.startswith(prefix) and f.endswith(".npz"))


def norm_rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    fin = np.isfinite(b)
    assert np.array_equal(np.isfinite(a), fin), "non-finite pattern differs"
    d = np.abs(a[fin] - b[fin]).max(initial=0.0)
    s = np.abs(b[fin]).max(initial=0.0)
    return d / s if s > 0 else d


def bit_equal(a, b):
    """Bitwise equality, treating every NaN as equal to every NaN."""
    a = np.ascontiguousarray(a, np.float32)
    b = np.ascontiguousarray(b, np.float32)
    if a.shape != b.shape:
        return False
    na, nb = np.isnan(a), np.isnan(b)
    if not np.array_equal(na, nb):
        return False
    return np.array_equal(a.view(np.uint32)[~na], b.view(np.uint32)[~nb])


def tiled_levels(B, H, W, L, device, fill=None, NQ=None):
    """Separate tiled level tensors [B*NQ, map_floats(H_l, W_l)] (the library's value pyramid,
    include/corr_mi355x.h), optionally filled with `fill`."""
    import torch
    from eraft_amd.corr import map_floats
    BN = B * (H * W if NQ is None else NQ)
    out = []
    for l in range(L):
        t = torch.empty(BN, map_floats(H >> l, W >> l), dtype=torch.float32, device=device)
        if fill is not None:
            t.fill_(fill)
        out.append(t)
    return out


def export_levels(levels, H, W):
    """The tiled levels in the reference's layout, as numpy [BN, 1, H_l, W_l] arrays."""
    from eraft_amd import _lib
    return [p.cpu().numpy() for p in _lib.pyramid_export(levels, H, W)]


def build_level0(t1, t2, algo, ws=None):
    """Level 0 of one build (corr_build_ex), row-major numpy [B*N, H*W]."""
    from eraft_amd import _lib
    B, _, H, W = t2.shape
    lv = tiled_levels(B, H, W, 1, t1.device, NQ=t1.shape[2] * t1.shape[3])
    _lib.build(t1, t2, lv, algo, ws)
    return export_levels(lv, H, W)[0].reshape(-1, H * W)
