"""Portable, counter-based PRNG for golden inputs (test infrastructure).

Golden fixtures store only seeds for their inputs; the inputs are regenerated bit-identically
on any machine / numpy version because every step is exact integer arithmetic or exact fp64
arithmetic (sums of 24-bit fractions) followed by one IEEE rounding:

  u64   = splitmix64(seed * 2^32 + index)
  unif  = (u64 >> 40) * 2^-24                        in [0, 1), exact in fp32
  gauss = (u1 + u2 + u3 + u4 - 2) * sqrt(3)          Irwin-Hall(4), unit variance, fp32
"""
from __future__ import annotations

import numpy as np

_M = np.uint64(0xFFFFFFFFFFFFFFFF)


def _splitmix64(x: np.ndarray) -> np.ndarray:
    with np.errstate(over="ignore"):
        z = x + np.uint64(0x9E3779B97F4A7C15)
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _counters(seed: int, n: int, stream: int = 0) -> np.ndarray:
    base = (np.uint64(seed) << np.uint64(32)) + np.uint64(stream) * np.uint64(1 << 58)
    return np.arange(n, dtype=np.uint64) + base


def uniform(seed: int, shape, lo: float = 0.0, hi: float = 1.0, stream: int = 0) -> np.ndarray:
    n = int(np.prod(shape))
    u = (_splitmix64(_counters(seed, n, stream)) >> np.uint64(40)).astype(np.float64) * 2.0 ** -24
    return (lo + (hi - lo) * u).astype(np.float32).reshape(shape)


def gauss(seed: int, shape, sigma: float = 1.0) -> np.ndarray:
    n = int(np.prod(shape))
    acc = np.zeros(n, np.float64)
    for s in range(4):
        acc += (_splitmix64(_counters(seed, n, s + 1)) >> np.uint64(40)).astype(np.float64) * 2.0 ** -24
    g = (acc - 2.0) * np.sqrt(3.0)
    return (g * sigma).astype(np.float32).reshape(shape)


def param_init(name: str, shape) -> np.ndarray | None:
    """Deterministic random-init value of a model parameter / buffer, keyed by its
    state_dict name (so two independent implementations with the reference's parameter
    names get identical weights).  None for integer bookkeeping buffers."""
    import zlib
    if name.endswith("num_batches_tracked"):
        return None
    seed = zlib.crc32(name.encode()) & 0x3FFFFFFF
    g = gauss(seed, shape).astype(np.float64)
    if name.endswith("running_var"):
        v = 1.0 + 0.1 * np.abs(g)
    elif name.endswith("running_mean"):
        v = 0.1 * g
    elif name.endswith("weight") and len(shape) == 4:
        fan_in = shape[1] * shape[2] * shape[3]
        v = g * np.sqrt(2.0 / fan_in)
    elif name.endswith("weight"):
        v = 1.0 + 0.1 * g
    else:  # bias
        v = 0.05 * g
    return v.astype(np.float32)


def voxel_grid(seed: int, shape, density: float = 0.15) -> np.ndarray:
    """Sparse event-voxel-like input: N(0,1) on ~`density` of the cells, 0 elsewhere."""
    mask = uniform(seed, shape, stream=7) < density
    return np.where(mask, gauss(seed + 1, shape), 0.0).astype(np.float32)


def coords_grid(B: int, H: int, W: int) -> np.ndarray:
    """Pixel grid [B, 2, H, W], ch0 = x (column), ch1 = y (row) — model/utils.py:24-27."""
    y, x = np.meshgrid(np.arange(H, dtype=np.float32), np.arange(W, dtype=np.float32), indexing="ij")
    return np.broadcast_to(np.stack([x, y])[None], (B, 2, H, W)).copy()


def lookup_coords(seed: int, B: int, H: int, W: int, sigma: float) -> np.ndarray:
    """coords_grid + N(0, sigma) flow at fmap scale (eraft.py:121-124 + :136)."""
    c = coords_grid(B, H, W)
    if sigma > 0:
        c = c + gauss(seed, (B, 2, H, W), sigma)
    return c.astype(np.float32)


def special_coords(B: int, H: int, W: int) -> np.ndarray:
    """Edge cases for the lookup: exact integers, exact last index, negatives, far outside,
    half-pixel and tiny offsets around the border (zero-padding semantics, utils.py:15)."""
    c = coords_grid(B, H, W)
    flat = c.reshape(B, 2, -1)
    n = flat.shape[-1]
    vals_x = np.array([0.0, W - 1, -0.5, -4.0, -9.25, W + 7.5, 1e4, -1e4, 0.5, W - 1.5,
                       2.999999, 3.000001, -1e-7, (W - 1) * 1.0000001, 1234.567, 7.0], np.float32)
    vals_y = np.array([0.0, H - 1, H + 3.5, -0.5, 2.0, -3.75, 1e4, 0.25, -1e4, H - 0.5,
                       1.000001, 0.999999, H - 1 + 1e-6, -2.0, -1234.5, 3.0], np.float32)
    k = min(n, len(vals_x))
    flat[:, 0, :k] = vals_x[:k]
    flat[:, 1, :k] = vals_y[:k]
    return flat.reshape(B, 2, H, W).astype(np.float32)
