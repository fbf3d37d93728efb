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
