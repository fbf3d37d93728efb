"""C-ABI checks that need no GPU: the library builds, loads, exports every symbol declared in
include/corr_mi355x.h, and rejects bad arguments before any HIP call."""
import ctypes
import os
import re

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HEADER = os.path.join(ROOT, "include", "corr_mi355x.h")


def _declared():
    src = open(HEADER).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(corr_[a-z_]+)\s*\(", src)))


@pytest.fixture(scope="module")
def lib():
    from eraft_amd.build import build_library
    from eraft_amd import _lib
    build_library()
    return _lib.load()


def test_header_declares_the_python_exports():
    from eraft_amd import _lib
    assert sorted(_lib.EXPORTS) == _declared()


def test_every_declared_symbol_is_exported(lib):
    for name in _declared():
        assert hasattr(lib, name), name


def test_version_and_workspace(lib):
    assert lib.corr_version() == 202
    # DSEC: 256 x 4800 slabs; at least one slab, deterministic plan
    ws = lib.corr_build_bwd_workspace(1, 256, 60, 80)
    assert ws >= 256 * 4800 * 4 and ws % (256 * 4800 * 4) == 0
    assert lib.corr_build_bwd_workspace(0, 256, 60, 80) == 0


@pytest.mark.parametrize("args,msg", [
    ((8, 8, 1, 256, 60, 80, 4, None, None), "pyr is NULL"),
    ((None, 8, 1, 256, 60, 80, 4, None, None), "fmap1 is NULL"),
    ((8, 8, 0, 256, 60, 80, 4, None, None), "B, H, W"),
    ((8, 8, 1, 0, 60, 80, 4, None, None), "D must be"),
    ((8, 8, 1, 256, 60, 80, 9, None, None), "levels must be"),
    ((8, 8, 1, 256, 4, 80, 4, None, None), "too small"),
    ((6, 8, 1, 256, 60, 80, 4, None, None), "aligned"),
])
def test_build_rejects_bad_arguments(lib, args, msg):
    rc = lib.corr_build(*args)
    assert rc == -1
    assert msg in lib.corr_last_error().decode()


def test_lookup_rejects_bad_radius(lib):
    pyr = (ctypes.c_void_p * 4)(16, 16, 16, 16)
    rc = lib.corr_lookup(pyr, 16, 1, 60, 80, 4, 8, 16, None)
    assert rc == -1 and "radius" in lib.corr_last_error().decode()


def test_build_bwd_rejects_small_workspace(lib):
    rc = lib.corr_build_bwd(16, 16, 16, 1, 256, 60, 80, 16, 16, 16, 4, None)
    assert rc == -1 and "workspace" in lib.corr_last_error().decode()


def test_python_front_end_refuses_cpu_tensors():
    import torch
    from eraft_amd import CorrBlock
    f = torch.zeros(1, 8, 16, 16)
    with pytest.raises(RuntimeError, match="MI355X"):
        CorrBlock(f, f)


def test_build_ex_workspace_and_validation(lib):
    # F16X3 workspace: hi/lo f16 operands (4 B per padded channel per pixel) + int32 exponents
    n = lib.corr_build_workspace(1, 1, 256, 4800, 60, 80)
    assert n >= 2 * 4800 * 256 * 4 + 2 * 4800 * 4
    assert lib.corr_build_workspace(0, 1, 256, 4800, 60, 80) == 0  # fp32 needs none
    assert lib.corr_build_workspace(1, 1, 10 ** 6, 4800, 60, 80) == ctypes.c_size_t(-1).value
    # BF16X6 workspace: hi/mid/lo bf16 operands (6 B per padded channel per pixel), any D
    n = lib.corr_build_workspace(2, 1, 256, 4800, 60, 80)
    assert n >= 2 * 4800 * 256 * 6
    assert lib.corr_build_workspace(2, 1, 1000, 4800, 60, 80) >= 2 * 4800 * 1000 * 6
    assert lib.corr_build_workspace(9, 1, 256, 4800, 60, 80) == ctypes.c_size_t(-1).value
    rc = lib.corr_build_ex(2, 256, 4800, 256, 1, 256, 60, 80, 4, pyr := (ctypes.c_void_p * 4)(256, 256, 256, 256),
                           256, 16, None)
    assert rc == -1 and "workspace" in lib.corr_last_error().decode()
    pyr = (ctypes.c_void_p * 4)(256, 256, 256, 256)
    rc = lib.corr_build_ex(1, 256, 4800, 256, 1, 256, 60, 80, 4, pyr, 256, 16, None)
    assert rc == -1 and "workspace" in lib.corr_last_error().decode()
    rc = lib.corr_build_ex(1, 256, 4800, 256, 1, 10 ** 6, 60, 80, 4, pyr, 256, 1 << 40, None)
    assert rc == -2 and "too large" in lib.corr_last_error().decode()
    rc = lib.corr_build_ex(7, 256, 4800, 256, 1, 256, 60, 80, 4, pyr, 256, 1 << 40, None)
    assert rc == -1 and "unknown algorithm" in lib.corr_last_error().decode()
    rc = lib.corr_build_ex(1, 256, 4800, 256, 1, 256, 60, 80, 4, pyr, 260, 1 << 40, None)
    assert rc == -1 and "256-byte aligned" in lib.corr_last_error().decode()
    # measurement phase flags: one at a time, and only on the split builds
    for algo in (0x100 | 0x200 | 1, 0x100 | 0x200 | 2, 0x100 | 0, 0x200 | 0):
        rc = lib.corr_build_ex(algo, 256, 4800, 256, 1, 256, 60, 80, 4, pyr, 256, 1 << 40, None)
        assert rc == -1 and "unknown algorithm" in lib.corr_last_error().decode(), hex(algo)


def test_build_region_validation(lib):
    """corr_build_region: bf16x6 only, region rows on 8-row patch boundaries, <= 4 levels, a
    workspace as corr_build_ex's — all refused before any HIP call."""
    pyr = (ctypes.c_void_p * 4)(256, 256, 256, 256)
    ws = 1 << 40
    call = lambda algo, y0, y1, L=4, H=60, wsb=ws, wsp=256: lib.corr_build_region(  # noqa: E731
        algo, 256, 4800, 256, y0, y1, 1, 256, H, 80, L, pyr, wsp, wsb, 1, None)
    assert call(1, 0, 16) == -2 and "BF16X6" in lib.corr_last_error().decode()
    assert call(0, 0, 16) == -2
    for y0, y1 in ((4, 16), (0, 12), (16, 16), (-8, 8), (48, 64)):
        assert call(2, y0, y1) == -1 and "y0" in lib.corr_last_error().decode(), (y0, y1)
    assert call(2, 0, 16, L=5) == -2 and "levels" in lib.corr_last_error().decode()
    assert call(2, 0, 16, wsb=16) == -1 and "workspace" in lib.corr_last_error().decode()
    assert call(2, 0, 16, wsp=260) == -1 and "aligned" in lib.corr_last_error().decode()


def test_build_algo_env(monkeypatch):
    from eraft_amd import _lib
    monkeypatch.delenv("ERAFT_AMD_BUILD", raising=False)
    assert _lib.default_algo() == _lib.BUILD_BF16X6
    assert _lib.backward_algo() == _lib.BUILD_BF16X6
    monkeypatch.setenv("ERAFT_AMD_BUILD", "fp32")
    assert _lib.default_algo() == _lib.BUILD_FP32
    assert _lib.backward_algo() == _lib.BUILD_FP32
    monkeypatch.setenv("ERAFT_AMD_BUILD", "f16x3")
    assert _lib.default_algo() == _lib.BUILD_F16X3
    monkeypatch.setenv("ERAFT_AMD_BUILD", "bf16")
    with pytest.raises(ValueError):
        _lib.default_algo()


def test_backward_workspace_and_validation(lib):
    """corr_backward: the workspace covers the GEMM slabs plus the per-workgroup column maxima
    (r = 4: 4 queries per workgroup), and a short workspace or a missing pointer is refused
    before any HIP call."""
    B, D, H, W, r = 8, 256, 36, 48, 4
    N = H * W
    ws = lib.corr_backward_workspace(1, B, D, N, H, W, r)
    assert ws >= lib.corr_build_bwd_ex_workspace(1, B, D, N, H, W) + B * (N // 4) * N * 4
    assert lib.corr_backward_workspace(0, B, D, N, H, W, r) == lib.corr_build_bwd_ex_workspace(0, B, D, N, H, W)
    assert lib.corr_backward_workspace(1, 0, D, N, H, W, r) == 0
    # bf16x6 (algo 2): the GEMM slabs only (no maxima partials), as corr_build_bwd_ex's
    assert lib.corr_backward_workspace(2, B, D, N, H, W, r) == lib.corr_build_bwd_ex_workspace(2, B, D, N, H, W)
    assert lib.corr_backward_workspace(2, B, D, N, H, W, r) < ws
    assert lib.corr_build_bwd_ex_workspace(3, B, D, N, H, W) == ctypes.c_size_t(-1).value
    # CORR_BACKWARD_EXACT_FOLD (0x400) selects the fold's arithmetic only: same workspace
    for a in (0, 1, 2):
        assert lib.corr_backward_workspace(a | 0x400, B, D, N, H, W, r) == lib.corr_backward_workspace(a, B, D, N, H, W, r)
    ptrs = (ctypes.c_void_p * 1)(16)
    gp = (ctypes.c_void_p * 4)(16, 16, 16, 16)
    rc = lib.corr_backward(1, ptrs, ptrs, 1, 16, N, 16, B, D, H, W, 4, r, gp, 16, 16, 16, 4, None)
    assert rc == -1 and "workspace" in lib.corr_last_error().decode()
    rc = lib.corr_backward(1, ptrs, ptrs, 1, None, N, 16, B, D, H, W, 4, r, gp, 16, 16, 16, ws, None)
    assert rc == -1
    rc = lib.corr_backward(3 | 0x400, ptrs, ptrs, 1, 16, N, 16, B, D, H, W, 4, r, gp, 16, 16, 16, ws, None)
    assert rc == -2 and "unknown algorithm" in lib.corr_last_error().decode()


def test_lookup_conv_validation(lib):
    assert lib.corr_lookup_conv_weights_bytes() >= 256 * 352 * 4
    rc = lib.corr_lookup_conv_weights(16, 128, 324, 16, None)  # 128 output channels: not convc1
    assert rc != 0 and "256" in lib.corr_last_error().decode()
    rc = lib.corr_lookup_conv_weights(None, 256, 324, 16, None)
    assert rc == -1
    pyr = (ctypes.c_void_p * 4)(16, 16, 16, 16)
    rc = lib.corr_lookup_conv(pyr, 16, 1, 60, 80, 4, 3, 16, 16, 1, 16, None)  # radius 3
    assert rc != 0 and "radius 4" in lib.corr_last_error().decode()


def test_lookup_conv_bwd_validation(lib):
    """corr_lookup_conv_bwd rejects what it cannot run before touching the GPU: radius != 4,
    a missing `out` under ReLU, a short workspace for dW / bias; with no output requested it is
    a no-op (no workspace needed)."""
    pyr = (ctypes.c_void_p * 4)(16, 16, 16, 16)
    ws_need = lib.corr_lookup_conv_bwd_workspace(8, 36, 48, 4)
    assert ws_need >= 64 * 256 * 324 * 4
    rc = lib.corr_lookup_conv_bwd(pyr, 16, 1, 60, 80, 4, 3, 16, 16, 1, 16, 16, 16, 16, 16, ws_need, None)
    assert rc == -2 and "radius 4" in lib.corr_last_error().decode()
    rc = lib.corr_lookup_conv_bwd(pyr, 16, 1, 60, 80, 4, 4, 16, None, 1, 16, 16, 16, 16, 16, ws_need, None)
    assert rc == -1 and "out" in lib.corr_last_error().decode()
    rc = lib.corr_lookup_conv_bwd(pyr, 16, 8, 36, 48, 4, 4, 16, 16, 1, 16, 16, None, None, 16, ws_need - 4, None)
    assert rc == -1 and "workspace" in lib.corr_last_error().decode()
    rc = lib.corr_lookup_conv_bwd(pyr, 16, 8, 36, 48, 4, 4, 16, 16, 1, 16, None, None, None, None, 0, None)
    assert rc == 0


def test_tiled_map_size_and_layout_validation(lib):
    """The value pyramid is tiled (include/corr_mi355x.h): ceil(H_l/4) * ceil(W_l/4) 4x4 tiles
    per query map, the Python allocator agrees, and level pointers that are not 16-B aligned are
    refused by the build, the lookup and the export / import before any HIP call."""
    from eraft_amd.corr import map_floats
    for h, w in ((60, 80), (7, 10), (15, 20), (1, 2), (17, 23), (160, 240), (4, 5)):
        assert lib.corr_map_floats(h, w) == map_floats(h, w) == ((h + 3) // 4) * ((w + 3) // 4) * 16
    assert lib.corr_map_floats(0, 5) == 0
    bad = (ctypes.c_void_p * 4)(256, 264, 256, 256)  # level 1 only 8-B aligned
    rc = lib.corr_build(256, 256, 1, 32, 60, 80, 4, bad, None)
    assert rc == -1 and "16-byte aligned" in lib.corr_last_error().decode()
    rc = lib.corr_lookup(bad, 256, 1, 60, 80, 4, 4, 256, None)
    assert rc == -1 and "16-byte aligned" in lib.corr_last_error().decode()
    ok = (ctypes.c_void_p * 4)(256, 256, 256, 256)
    rc = lib.corr_pyramid_export(bad, 4800, 60, 80, 4, ok, None)
    assert rc == -1 and "16-byte aligned" in lib.corr_last_error().decode()
    rc = lib.corr_pyramid_import(ok, 4800, 60, 80, 4, bad, None)
    assert rc == -1 and "16-byte aligned" in lib.corr_last_error().decode()
    rc = lib.corr_pyramid_export(ok, 0, 60, 80, 4, ok, None)
    assert rc == -1 and "BN" in lib.corr_last_error().decode()
    rc = lib.corr_pyramid_import(ok, 4800, 4, 80, 4, ok, None)
    assert rc == -1 and "too small" in lib.corr_last_error().decode()


def test_python_level_size_check():
    """the ctypes front-end refuses level buffers smaller than the maps the library
    will touch (the C-ABI takes bare pointers): tiled value levels need BN * map_floats per
    level, row-major gradient / export levels BN * H_l * W_l (exactly, for the export's out)."""
    import torch
    from eraft_amd import _lib
    BN, H, W = 6, 30, 40
    tiled = [torch.empty(BN * _lib.map_floats(H >> l, W >> l)) for l in range(3)]
    _lib._check_levels(tiled, BN, H, W, "pyr")
    rowmajor = [torch.empty(BN, 1, H >> l, W >> l) for l in range(3)]  # ABI-104 value levels: too small
    with pytest.raises(ValueError, match=r"pyr\[0\] has 7200 floats, needs 7680"):
        _lib._check_levels(rowmajor, BN, H, W, "pyr")
    _lib._check_levels(rowmajor, BN, H, W, "out", tiled=False, exact=True)
    with pytest.raises(ValueError, match="exactly"):
        _lib._check_levels(tiled, BN, H, W, "out", tiled=False, exact=True)
    with pytest.raises(ValueError, match="levels"):
        _lib._check_levels(rowmajor * 3, BN, H, W, "pyr", tiled=False)
