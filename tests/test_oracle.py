"""Pin the oracle (oracle/corr_oracle.c, oracle/torch_ops.py) to the reference's own outputs.

The golden vectors were produced by the reference CorrBlock (model/corr.py:12-60) — see
tests/golden/make_golden.py.  CPU only, no GPU needed.
"""
import numpy as np
import pytest
import torch

import prng
from _util import REL_TOL, bit_equal, golden_names, load, norm_rel
from oracle import oracle, torch_ops

BUILD_CASES = [n for n in golden_names() if not n.startswith(("g_bwd", "g_dsec", "g_e2e", "g_splat", "g_voxel"))]


def _inputs(meta):
    seed, B, D, H, W = (int(v) for v in meta[:5])
    return prng.gauss(seed, (B, D, H, W)), prng.gauss(seed + 1, (B, D, H, W))


@pytest.mark.parametrize("name", BUILD_CASES)
def test_build_within_tolerance(name):
    g = load(name)
    f1, f2 = _inputs(g["meta"])
    L = int(g["meta"][5])
    pyr = oracle.build_pyramid(f1, f2, L)
    for l in range(L):
        assert pyr[l].shape == g[f"pyr{l}"].shape
        assert norm_rel(pyr[l], g[f"pyr{l}"]) < 1e-6


@pytest.mark.parametrize("name", BUILD_CASES)
def test_pool_bitexact(name):
    """avg_pool2d restatement is bit-identical to the reference on the reference's level 0."""
    g = load(name)
    L = int(g["meta"][5])
    for l in range(1, L):
        assert bit_equal(oracle.avg_pool2x2(g[f"pyr{l - 1}"]), g[f"pyr{l}"])


@pytest.mark.parametrize("name", BUILD_CASES)
def test_lookup_bitexact(name):
    """Lookup restatement on the reference pyramid is bit-identical (NaN levels included)."""
    g = load(name)
    r = int(g["meta"][6])
    L = int(g["meta"][5])
    pyr = [g[f"pyr{l}"] for l in range(L)]
    keys = [k[len("coords"):] for k in g if k.startswith("coords")]
    assert keys
    for k in keys:
        out = oracle.lookup(pyr, g["coords" + k], r)
        assert bit_equal(out, g["look" + k]), k


def test_degenerate_level_is_nan():
    """12x16 fmaps: level 3 is 1x2 -> the reference returns NaN for that level (utils.py:11-12)."""
    g = load("g_degenerate_b1_d32_12x16")
    ref = g["look0"]
    assert np.isnan(ref[:, 3 * 81:]).all()
    assert np.isfinite(ref[:, :3 * 81]).all()


@pytest.mark.parametrize("name", [n for n in golden_names("g_bwd")])
def test_backward_within_tolerance(name):
    g = load(name)
    seed, B, D, H, W, L, r, iters = (int(v) for v in g["meta"])
    f1, f2 = prng.gauss(seed, (B, D, H, W)), prng.gauss(seed + 1, (B, D, H, W))
    K = (2 * r + 1) ** 2
    coords = [prng.lookup_coords(seed + 200 + t, B, H, W, 2.0 + t) for t in range(iters)]
    grads = [prng.gauss(seed + 300 + t, (B, L * K, H, W)) for t in range(iters)]
    df1, df2 = oracle.fmap_grads(f1, f2, coords, grads, L, r)
    assert norm_rel(df1, g["df1"]) < 1e-5
    assert norm_rel(df2, g["df2"]) < 1e-5


def test_dsec_spot_rows():
    g = load("g_dsec_spot")
    seed, B, D, H, W, L, r = (int(v) for v in g["meta"])
    f1, f2 = prng.gauss(seed, (B, D, H, W)), prng.gauss(seed + 1, (B, D, H, W))
    q = g["q"]
    for qi in q[:4]:
        row = oracle.corr_rows(f1, f2, int(qi), int(qi) + 1)[0, 0]
        assert norm_rel(row, g["pyr0_rows"][list(q).index(qi), 0].ravel()) < 1e-6


def test_torch_ops_restatement_matches_reference():
    """The CPU baseline path (oracle/torch_ops.py) reproduces the reference outputs."""
    for name in ("g_b1_d32_16x16", "g_b2_d64_16x20_L2r3"):
        g = load(name)
        f1, f2 = _inputs(g["meta"])
        L, r = int(g["meta"][5]), int(g["meta"][6])
        lv = torch_ops.cpu_build(torch.from_numpy(f1), torch.from_numpy(f2), L)
        for l in range(L):
            assert norm_rel(lv[l].numpy(), g[f"pyr{l}"]) < 1e-6
        ref_lv = [torch.from_numpy(g[f"pyr{l}"]) for l in range(L)]
        out = torch_ops.cpu_lookup(ref_lv, torch.from_numpy(g["coords_special"]), r)
        assert bit_equal(out.numpy(), g["look_special"])


def test_prng_is_stable():
    """Golden inputs are regenerated from seeds: pin a few values of the PRNG stream."""
    u = prng.uniform(7, (4,))
    g = prng.gauss(7, (3,))
    assert u.dtype == np.float32 and g.dtype == np.float32
    assert np.all((u >= 0) & (u < 1))
    # regenerating gives identical bits
    assert bit_equal(u, prng.uniform(7, (4,)))
    assert bit_equal(g, prng.gauss(7, (3,)))
    assert abs(float(prng.gauss(3, (200000,)).std()) - 1.0) < 0.01


def test_oracle_grad_matches_finite_difference():
    """Independent check of the backward restatement: directional derivative vs autograd-free
    finite difference through the oracle forward (double-checked sign/orientation)."""
    B, D, H, W, L, r = 1, 4, 8, 8, 2, 2
    f1, f2 = prng.gauss(1, (B, D, H, W)), prng.gauss(2, (B, D, H, W))
    c = prng.lookup_coords(3, B, H, W, 1.3)
    K = (2 * r + 1) ** 2
    g = prng.gauss(4, (B, L * K, H, W))
    df1, df2 = oracle.fmap_grads(f1, f2, [c], [g], L, r)
    v1, v2 = prng.gauss(5, f1.shape), prng.gauss(6, f2.shape)

    def J(a, b):
        pyr = oracle.build_pyramid(a.astype(np.float32), b.astype(np.float32), L)
        return float((oracle.lookup(pyr, c, r).astype(np.float64) * g).sum())

    eps = 1e-3
    fd = (J(f1 + eps * v1, f2 + eps * v2) - J(f1 - eps * v1, f2 - eps * v2)) / (2 * eps)
    an = float((df1.astype(np.float64) * v1).sum() + (df2.astype(np.float64) * v2).sum())
    assert abs(fd - an) <= 2e-2 * max(1.0, abs(an))


def test_oracle_forward_splat_matches_reference_golden():
    """Warm-start splat (utils/image_utils.py:52-83) restated in C: bit-identical to the
    reference on the splat fixtures (fractional, integer, far-out and colliding flows) and on
    the E2E golden's own flow_init = forward_interpolate_pytorch(cold low-res flow)."""
    from oracle import oracle
    g = load("g_splat")
    for t in "ab":
        assert bit_equal(oracle.forward_splat(g[f"flow_{t}"]), g[f"splat_{t}"]), t
    e = load("g_e2e_dsec")
    assert bit_equal(oracle.forward_splat(e["low"]), e["flow_init"])


def test_oracle_voxel_grid_tbilinear_matches_reference_golden():
    """MVSEC event -> voxel grid (utils/transformers.py:36-126) restated in C: the raw grid is
    bit-identical to the reference (left then right index_add_ passes, event order), including
    the all-equal-stamps case (deltaT = 0 -> 1); the normalised grid within 1e-6 of max|v|."""
    g = load("g_voxel_mvsec")
    for t in "abc":
        M, C, H, W = (int(v) for v in g[f"meta_{t}"])
        assert bit_equal(oracle.voxel_grid_tbilinear(g[f"ev_{t}"], C, H, W, False), g[f"raw_{t}"]), t
        n, ref = oracle.voxel_grid_tbilinear(g[f"ev_{t}"], C, H, W, True), g[f"norm_{t}"]
        assert np.abs(n - ref).max() <= 1e-6 * np.abs(ref).max(), t


def test_oracle_voxel_grid_matches_reference_golden():
    """DSEC event -> voxel grid (utils/dsec_utils.py:26-64) restated in C: the raw grid is
    bit-identical to the reference (single-threaded, as main.py:2-5 runs it); the normalised
    grid is within 1e-6 of max|v| (mean / std reductions: fp64 here, ATen's order there)."""
    from oracle import oracle
    g = load("g_voxel")
    for t in "ab":
        M, C, H, W = (int(v) for v in g[f"meta_{t}"])
        assert bit_equal(oracle.voxel_grid(g[f"ev_{t}"], C, H, W, False), g[f"raw_{t}"]), t
        n, ref = oracle.voxel_grid(g[f"ev_{t}"], C, H, W, True), g[f"norm_{t}"]
        assert np.abs(n - ref).max() <= 1e-6 * np.abs(ref).max(), t
