"""ORACLE — test infrastructure only (see oracle/corr_oracle.c header).

numpy front-end over ``oracle/_build/libcorr_oracle.so``, the plain-C restatement of the
reference CorrBlock (model/corr.py:12-60, model/utils.py:7-21).  Imported only by tests/,
``__graft_entry__.smoke()`` and bench.py's ``cpu_baseline`` leg; the product package
``eraft_amd`` never imports it.

All arrays are float32, C-contiguous, in the reference's layouts:
  fmaps  [B, D, H, W]           (corr.py:53-56)
  pyramid level l  [B*H*W, 1, H>>l, W>>l]   (corr.py:21-27)
  coords [B, 2, H, W], ch0 = x, ch1 = y     (utils.py:24-27)
  lookup out [B, L*(2r+1)^2, H, W]          (corr.py:49-50)
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "_build", "libcorr_oracle.so")
_lib = None

_f32p = ctypes.POINTER(ctypes.c_float)


def build() -> str:
    """Compile the C restatement (make -C oracle).  Returns the .so path."""
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _SO


def _load():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            build()
        lib = ctypes.CDLL(_SO)
        i, l, vp = ctypes.c_int, ctypes.c_long, ctypes.c_void_p
        lib.oracle_corr_rows.argtypes = [vp, vp, i, i, i, i, i, vp]
        lib.oracle_avg_pool2x2.argtypes = [vp, l, i, i, vp]
        lib.oracle_lookup.argtypes = [vp, vp, i, i, i, i, i, vp]
        lib.oracle_lookup_rows.argtypes = [vp, vp, i, i, i, i, i, i, vp]
        lib.oracle_lookup_rows.restype = None
        lib.oracle_lookup_bwd.argtypes = [vp, vp, i, i, i, i, i, vp]
        lib.oracle_pool_bwd.argtypes = [vp, l, i, i, i]
        lib.oracle_corr_bwd.argtypes = [vp, vp, vp, i, i, i, vp, vp]
        lib.oracle_forward_splat.argtypes = [vp, i, i, i, vp]
        lib.oracle_voxel_grid.argtypes = [vp, vp, vp, vp, l, i, i, i, i, vp]
        lib.oracle_voxel_grid_tbilinear.argtypes = [vp, l, i, i, i, i, vp]
        for f in ("oracle_corr_rows", "oracle_avg_pool2x2", "oracle_lookup",
                  "oracle_lookup_bwd", "oracle_pool_bwd", "oracle_corr_bwd", "oracle_forward_splat",
                  "oracle_voxel_grid", "oracle_voxel_grid_tbilinear"):
            getattr(lib, f).restype = None
        _lib = lib
    return _lib


def _c(a: np.ndarray) -> np.ndarray:
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a


def _p(a: np.ndarray):
    return a.ctypes.data_as(ctypes.c_void_p)


def _ptr_array(arrs):
    return (ctypes.c_void_p * len(arrs))(*[a.ctypes.data for a in arrs])


def level_shapes(H: int, W: int, L: int):
    """Floor-halving level sizes of avg_pool2d(2, stride 2) (corr.py:25-27)."""
    return [(H >> l, W >> l) for l in range(L)]


def corr_rows(f1, f2, q0=0, q1=None) -> np.ndarray:
    """corr.py:52-60 for query rows [q0, q1): returns [B, q1-q0, H*W]."""
    f1, f2 = _c(f1), _c(f2)
    B, D, H, W = f1.shape
    N = H * W
    q1 = N if q1 is None else q1
    out = np.empty((B, q1 - q0, N), np.float32)
    _load().oracle_corr_rows(_p(f1), _p(f2), B, D, N, q0, q1, _p(out))
    return out


def avg_pool2x2(level: np.ndarray) -> np.ndarray:
    """corr.py:26 on [BN, 1, H, W] -> [BN, 1, H//2, W//2]."""
    level = _c(level)
    BN, _, H, W = level.shape
    out = np.empty((BN, 1, H // 2, W // 2), np.float32)
    _load().oracle_avg_pool2x2(_p(level), BN, H, W, _p(out))
    return out


def build_pyramid(f1, f2, num_levels=4):
    """corr.py:13-27: list of levels [B*H*W, 1, H>>l, W>>l]."""
    B, D, H, W = f1.shape
    c = corr_rows(f1, f2).reshape(B * H * W, 1, H, W)
    pyr = [c]
    for _ in range(num_levels - 1):
        pyr.append(avg_pool2x2(pyr[-1]))
    return pyr


def lookup(pyr, coords, radius=4) -> np.ndarray:
    """corr.py:29-50: [B, L*(2r+1)^2, H, W]."""
    coords = _c(coords)
    B, _, H, W = coords.shape
    L = len(pyr)
    pyr = [_c(p) for p in pyr]
    K = (2 * radius + 1) ** 2
    out = np.empty((B, L * K, H, W), np.float32)
    _load().oracle_lookup(_ptr_array(pyr), _p(coords), B, H, W, L, radius, _p(out))
    return out


def lookup_rows(pyr, coords_rows, H, W, radius=4) -> np.ndarray:
    """Lookup for a query-row slab: coords [B, 2, rows, Wq] against a pyramid of the
    (H, W) target map whose levels are [B*rows*Wq, 1, H>>l, W>>l]."""
    coords_rows = _c(coords_rows)
    B = coords_rows.shape[0]
    NQ = int(np.prod(coords_rows.shape[2:]))
    L = len(pyr)
    pyr = [_c(p) for p in pyr]
    K = (2 * radius + 1) ** 2
    out = np.empty((B, L * K) + coords_rows.shape[2:], np.float32)
    _load().oracle_lookup_rows(_ptr_array(pyr), _p(coords_rows), B, NQ, H, W, L, radius, _p(out))
    return out


def lookup_bwd(coords, grad_out, grad_pyr, radius=4):
    """Input-gradient of corr.py:45, accumulated into grad_pyr (list, modified in place)."""
    coords, grad_out = _c(coords), _c(grad_out)
    B, _, H, W = coords.shape
    for g in grad_pyr:
        assert g.dtype == np.float32 and g.flags.c_contiguous
    _load().oracle_lookup_bwd(_p(coords), _p(grad_out), B, H, W, len(grad_pyr), radius,
                              _ptr_array(grad_pyr))
    return grad_pyr


def pool_bwd(grad_pyr, H, W):
    """avg_pool2d backward chain (corr.py:25-27), in place; grad_pyr[0] = dL/dC."""
    BN = grad_pyr[0].shape[0]
    _load().oracle_pool_bwd(_ptr_array(grad_pyr), BN, H, W, len(grad_pyr))
    return grad_pyr


def corr_bwd(grad_c, f1, f2):
    """bmm + 1/sqrt(D) backward (corr.py:58-60): returns (df1, df2) [B, D, H, W]."""
    grad_c, f1, f2 = _c(grad_c), _c(f1), _c(f2)
    B, D, H, W = f1.shape
    df1 = np.empty_like(f1)
    df2 = np.empty_like(f2)
    _load().oracle_corr_bwd(_p(grad_c), _p(f1), _p(f2), B, D, H * W, _p(df1), _p(df2))
    return df1, df2


def fmap_grads(f1, f2, coords_list, grads_list, num_levels=4, radius=4):
    """Full backward of one build + len(coords_list) lookups w.r.t. fmap1, fmap2."""
    B, D, H, W = f1.shape
    gp = [np.zeros((B * H * W, 1, h, w), np.float32) for h, w in level_shapes(H, W, num_levels)]
    for c, g in zip(coords_list, grads_list):
        lookup_bwd(c, g, gp, radius)
    pool_bwd(gp, H, W)
    return corr_bwd(gp[0], f1, f2)


def forward_splat(flow) -> np.ndarray:
    """utils/image_utils.py:52-83 forward_interpolate_pytorch: [B, 2, H, W] -> [B, 2, H, W]."""
    flow = _c(flow)
    B, _, H, W = flow.shape
    out = np.empty_like(flow)
    _load().oracle_forward_splat(_p(flow), B, H, W, _p(out))
    return out


def voxel_grid(ev, C, H, W, normalize) -> np.ndarray:
    """utils/dsec_utils.py:26-64 VoxelGrid.convert: ev = [4, M] rows x, y, t, p -> [C, H, W]."""
    ev = _c(ev)
    M = ev.shape[1]
    out = np.empty((C, H, W), np.float32)
    rows = [np.ascontiguousarray(ev[k]) for k in range(4)]
    _load().oracle_voxel_grid(*[_p(r) for r in rows], M, C, H, W, int(bool(normalize)), _p(out))
    return out


def voxel_grid_tbilinear(events, C, H, W, normalize) -> np.ndarray:
    """utils/transformers.py:36-126 EventSequenceToVoxelGrid_Pytorch: events [M, 4] float64
    rows (t, x, y, p) -> [C, H, W] float32."""
    ev = np.ascontiguousarray(events, dtype=np.float64)
    M = ev.shape[0]
    out = np.empty((C, H, W), np.float32)
    _load().oracle_voxel_grid_tbilinear(_p(ev), M, C, H, W, int(bool(normalize)), _p(out))
    return out
