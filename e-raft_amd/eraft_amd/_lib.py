"""ctypes binding of libcorr_mi355x.so (C-ABI: include/corr_mi355x.h).

This is the ONLY path to the kernels: there is no CPU or eager-PyTorch fallback.  If the
library is missing, or a tensor is not on a HIP device, calls raise.
torch is imported first so that the library binds to the HIP runtime torch already loaded
(both carry the SONAME libamdhip64.so.7), i.e. one runtime, one set of device pointers.
"""
from __future__ import annotations

import ctypes
import os

import torch

from .build import SO_PATH

CORR_OK = 0
CORR_EINVAL = -1
CORR_EUNSUPPORTED = -2
CORR_EHIP = -3
MAX_LEVELS = 8
MAX_RADIUS = 7

EXPORTS = ("corr_version", "corr_last_error", "corr_build", "corr_lookup", "corr_lookup_bwd",
           "corr_pool_bwd", "corr_build_bwd_workspace", "corr_build_bwd", "corr_build_rows",
           "corr_lookup_rows", "corr_lookup_bwd_rows", "corr_build_bwd_rows_workspace",
           "corr_build_bwd_rows", "corr_build_workspace", "corr_build_ex",
           "corr_build_bwd_ex_workspace", "corr_build_bwd_ex", "corr_forward_splat_workspace",
           "corr_forward_splat", "corr_convex_upsample", "corr_voxel_grid_workspace",
           "corr_voxel_grid", "corr_lookup_conv", "corr_lookup_conv_weights", "corr_lookup_conv_weights_bytes", "corr_voxel_grid_tbilinear_workspace",
           "corr_voxel_grid_tbilinear", "corr_lookup_bwd_multi", "corr_pool_fold", "corr_backward_workspace",
           "corr_backward", "corr_convex_upsample_bwd_workspace", "corr_convex_upsample_bwd", "corr_build_region",
           "corr_lookup_conv_bwd_workspace", "corr_lookup_conv_bwd", "corr_map_floats", "corr_pyramid_export",
           "corr_pyramid_import")
ABI_VERSION = 202  # include/corr_mi355x.h: tiled value pyramid, separable fold, fp32 non-finite rule (bf16x6 bwd)

# Build algorithms (include/corr_mi355x.h).  BF16X6 is the default: every fp32 feature split
# exactly into three bf16 pieces, the six largest piece products on the bf16 MFMA, fp32
# accumulate — no narrower than the exact-fp32 MFMA build (test_build_bf16x6_not_narrower_than_fp32).
# ERAFT_AMD_BUILD=fp32 selects the fp32-operand MFMA build, =f16x3 the two-piece f16 split
# (~2^-22 per feature, narrower than fp32).
BUILD_FP32 = 0
BUILD_F16X3 = 1
BUILD_BF16X6 = 2
BUILD_ONLY_PACK = 0x100  # measurement: OR into BUILD_F16X3 / _BF16X6 to run only the operand pack
BUILD_ONLY_MFMA = 0x200  # ... or only the MFMA kernel (the workspace holds this pair's pack)
BACKWARD_EXACT_FOLD = 0x400  # OR into corr_backward's algo: the bit-exact fold (exact_fold())
_ALGOS = {"fp32": BUILD_FP32, "f16x3": BUILD_F16X3, "bf16x6": BUILD_BF16X6}


def default_algo() -> int:
    name = os.environ.get("ERAFT_AMD_BUILD", "bf16x6").lower()
    if name not in _ALGOS:
        raise ValueError(f"ERAFT_AMD_BUILD must be one of {sorted(_ALGOS)} (got {name!r})")
    return _ALGOS[name]


def backward_algo(algo=None) -> int:
    """The backward GEMMs' algorithm for a build algorithm: each build's own arithmetic (bf16x6:
    the exact three-piece bf16 split GEMMs, smaller worst / mean row error than fp32's; f16x3: the
    two-piece f16 split;
    fp32: the fp32-operand MFMA GEMMs)."""
    return default_algo() if algo is None else algo

_lib = None


class CorrError(RuntimeError):
    """A libcorr_mi355x call returned a negative status."""

    def __init__(self, code: int, msg: str):
        super().__init__(f"[corr {code}] {msg}")
        self.code = code


def load(path: str | None = None) -> ctypes.CDLL:
    """Load (once) and type the library.  Raises if it has not been built."""
    global _lib
    if _lib is not None and path is None:
        return _lib
    so = path or SO_PATH
    if not os.path.exists(so):
        raise RuntimeError(
            f"{so} is missing: build it with `python -c 'import __graft_entry__ as g; g.build()'` "
            "(eraft_amd has no CPU fallback)")
    lib = ctypes.CDLL(so)
    vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
    lib.corr_version.argtypes, lib.corr_version.restype = [], i
    lib.corr_last_error.argtypes, lib.corr_last_error.restype = [], ctypes.c_char_p
    lib.corr_map_floats.argtypes, lib.corr_map_floats.restype = [i, i], sz
    lib.corr_pyramid_export.argtypes = [vp, i, i, i, i, vp, vp]
    lib.corr_pyramid_import.argtypes = [vp, i, i, i, i, vp, vp]
    lib.corr_build.argtypes = [vp, vp, i, i, i, i, i, vp, vp]
    lib.corr_lookup.argtypes = [vp, vp, i, i, i, i, i, vp, vp]
    lib.corr_lookup_bwd.argtypes = [vp, vp, i, i, i, i, i, vp, vp]
    lib.corr_pool_bwd.argtypes = [vp, i, i, i, i, vp]
    lib.corr_build_bwd_workspace.argtypes = [i, i, i, i]
    lib.corr_build_bwd_workspace.restype = sz
    lib.corr_build_bwd.argtypes = [vp, vp, vp, i, i, i, i, vp, vp, vp, sz, vp]
    lib.corr_build_rows.argtypes = [vp, i, vp, i, i, i, i, i, vp, vp]
    lib.corr_lookup_rows.argtypes = [vp, vp, i, i, i, i, i, i, vp, vp]
    lib.corr_lookup_bwd_rows.argtypes = [vp, vp, i, i, i, i, i, i, vp, vp]
    lib.corr_build_bwd_rows_workspace.argtypes = [i, i, i, i, i]
    lib.corr_build_bwd_rows_workspace.restype = sz
    lib.corr_build_bwd_rows.argtypes = [vp, vp, i, vp, i, i, i, i, vp, vp, vp, sz, vp]
    lib.corr_build_workspace.argtypes = [i, i, i, i, i, i]
    lib.corr_build_workspace.restype = sz
    lib.corr_build_ex.argtypes = [i, vp, i, vp, i, i, i, i, i, vp, vp, sz, vp]
    lib.corr_build_bwd_ex_workspace.argtypes = [i, i, i, i, i, i]
    lib.corr_build_bwd_ex_workspace.restype = sz
    lib.corr_build_bwd_ex.argtypes = [i, vp, vp, i, vp, i, i, i, i, vp, vp, vp, sz, vp]
    lib.corr_forward_splat_workspace.argtypes = [i, i, i]
    lib.corr_forward_splat_workspace.restype = sz
    lib.corr_forward_splat.argtypes = [vp, i, i, i, vp, vp, sz, vp]
    lib.corr_convex_upsample.argtypes = [vp, vp, i, i, i, vp, vp]
    lib.corr_convex_upsample_bwd_workspace.argtypes = [i, i, i]
    lib.corr_convex_upsample_bwd_workspace.restype = sz
    lib.corr_convex_upsample_bwd.argtypes = [vp, vp, vp, i, i, i, vp, vp, vp, sz, vp]
    lib.corr_lookup_conv.argtypes = [vp, vp, i, i, i, i, i, vp, vp, i, vp, vp]
    lib.corr_lookup_conv_weights.argtypes = [vp, i, i, vp, vp]
    lib.corr_lookup_conv_weights_bytes.argtypes = []
    lib.corr_lookup_conv_weights_bytes.restype = sz
    lib.corr_voxel_grid_workspace.argtypes = [i, i, i, i]
    lib.corr_voxel_grid_workspace.restype = sz
    lib.corr_voxel_grid.argtypes = [vp, vp, vp, vp, i, i, i, i, i, vp, vp, sz, vp]
    lib.corr_voxel_grid_tbilinear_workspace.argtypes = [i, i, i, i]
    lib.corr_voxel_grid_tbilinear_workspace.restype = sz
    lib.corr_voxel_grid_tbilinear.argtypes = [vp, i, i, i, i, i, vp, vp, sz, vp]
    lib.corr_lookup_bwd_multi.argtypes = [vp, vp, i, i, i, i, i, i, i, vp, vp]
    lib.corr_pool_fold.argtypes = [vp, i, i, i, i, i, vp]
    lib.corr_backward_workspace.argtypes = [i, i, i, i, i, i, i]
    lib.corr_backward_workspace.restype = sz
    lib.corr_backward.argtypes = [i, vp, vp, i, vp, i, vp, i, i, i, i, i, i, vp, vp, vp, vp, sz, vp]
    lib.corr_build_region.argtypes = [i, vp, i, vp, i, i, i, i, i, i, i, vp, vp, sz, i, vp]
    lib.corr_lookup_conv_bwd_workspace.argtypes = [i, i, i, i]
    lib.corr_lookup_conv_bwd_workspace.restype = sz
    lib.corr_lookup_conv_bwd.argtypes = [vp, vp, i, i, i, i, i, vp, vp, i, vp, vp, vp, vp, vp, sz, vp]
    for f in ("corr_build_region", "corr_build", "corr_lookup", "corr_lookup_bwd", "corr_pool_bwd", "corr_build_bwd",
              "corr_build_rows", "corr_lookup_rows", "corr_lookup_bwd_rows", "corr_build_bwd_rows",
              "corr_build_ex", "corr_build_bwd_ex", "corr_forward_splat",
              "corr_convex_upsample", "corr_voxel_grid", "corr_lookup_conv", "corr_lookup_conv_weights",
              "corr_voxel_grid_tbilinear", "corr_lookup_bwd_multi", "corr_pool_fold", "corr_backward_workspace",
              "corr_backward", "corr_convex_upsample_bwd", "corr_lookup_conv_bwd", "corr_pyramid_export",
              "corr_pyramid_import"):
        getattr(lib, f).restype = i
    if lib.corr_version() != ABI_VERSION:
        raise RuntimeError(f"{so} has ABI {lib.corr_version()}, eraft_amd needs {ABI_VERSION}: rebuild it")
    if path is None:
        _lib = lib
    return lib


def _check(rc: int):
    if rc != CORR_OK:
        raise CorrError(rc, load().corr_last_error().decode(errors="replace"))


def _dev(t: torch.Tensor, name: str) -> int:
    if not isinstance(t, torch.Tensor):
        raise TypeError(f"{name} must be a torch.Tensor")
    if t.device.type != "cuda":
        raise RuntimeError(f"{name} is on {t.device}: eraft_amd runs only on an MI355X (HIP) device")
    if t.dtype != torch.float32:
        raise TypeError(f"{name} must be float32 (got {t.dtype})")
    if not t.is_contiguous():
        raise ValueError(f"{name} must be contiguous")
    return t.data_ptr()


def _ptrs(ts, name):
    arr = (ctypes.c_void_p * len(ts))()
    for k, t in enumerate(ts):
        arr[k] = _dev(t, f"{name}[{k}]")
    return arr


TILE_W = 4  # cells per tile row (include/corr_mi355x.h): tiles of 4 rows x TILE_W cells


def map_floats(Hl: int, Wl: int) -> int:
    """Floats of one query's tiled level map (include/corr_mi355x.h, corr_map_floats)."""
    return ((Hl + 3) // 4) * ((Wl + TILE_W - 1) // TILE_W) * 4 * TILE_W


def _check_levels(levels, BN: int, H: int, W: int, name: str, tiled: bool = True, exact: bool = False):
    """Every level tensor must hold the BN maps the library will read or write: BN * map_floats
    of the level for the tiled value pyramid, BN * H_l * W_l for the row-major ones (gradient
    pyramids, the reference-layout export).  The C-ABI takes bare pointers, so a short buffer
    (e.g. a caller still allocating the ABI-104 row-major [B*N, 1, H_l, W_l] value levels, which
    are smaller than the tiled maps whenever H_l or W_l is not a multiple of 4) would be an
    out-of-bounds device access: refuse it here."""
    if not 1 <= len(levels) <= MAX_LEVELS:
        raise ValueError(f"{name}: {len(levels)} levels (1..{MAX_LEVELS} supported)")
    for l, t in enumerate(levels):
        h, w = H >> l, W >> l
        need = BN * (map_floats(h, w) if tiled else h * w)
        n = t.numel()
        if n < need or (exact and n != need):
            what = f"{BN} maps of {'map_floats' if tiled else 'H_l*W_l'}({h}, {w})"
            raise ValueError(f"{name}[{l}] has {n} floats, needs {'exactly ' if exact else ''}{need} ({what})")


def _stream(t: torch.Tensor) -> int:
    return torch.cuda.current_stream(t.device).cuda_stream


def _nq(t):
    """Query pixels per batch item of a [B, C, rows, W] (or [B, C, NQ]) tensor."""
    n = 1
    for d in t.shape[2:]:
        n *= d
    return n


def pyramid_export(levels, H, W, out=None):
    """corr_pyramid_export: the tiled levels ([BN, map_floats]) -> the reference's layout, a list
    of [BN, 1, H_l, W_l] tensors (allocated unless `out` is given)."""
    BN = levels[0].shape[0]
    _check_levels(levels, BN, H, W, "pyr")
    if out is None:
        out = [torch.empty((BN, 1, H >> l, W >> l), dtype=torch.float32, device=levels[0].device)
               for l in range(len(levels))]
    elif len(out) != len(levels):
        raise ValueError(f"out has {len(out)} levels, the pyramid {len(levels)}")
    _check_levels(out, BN, H, W, "out", tiled=False, exact=True)
    with torch.cuda.device(levels[0].device):
        _check(load().corr_pyramid_export(_ptrs(levels, "pyr"), BN, H, W, len(levels), _ptrs(out, "out"),
                                          _stream(levels[0])))
    return out


def pyramid_import(src, levels, H, W):
    """corr_pyramid_import: reference-layout levels [BN, 1, H_l, W_l] (any contiguous view) ->
    the tiled `levels` (padding cells zeroed)."""
    BN = levels[0].shape[0]
    src = [t.contiguous() for t in src]
    if len(src) != len(levels):
        raise ValueError(f"src has {len(src)} levels, the pyramid {len(levels)}")
    for l, t in enumerate(src):
        if t.numel() != BN * (H >> l) * (W >> l):
            raise ValueError(f"level {l} has {t.numel()} values, expected {BN}x{H >> l}x{W >> l}")
    _check_levels(levels, BN, H, W, "pyr")
    with torch.cuda.device(levels[0].device):
        _check(load().corr_pyramid_import(_ptrs(src, "src"), BN, H, W, len(levels), _ptrs(levels, "pyr"),
                                          _stream(levels[0])))


def build_workspace(fmap1, fmap2, algo=None):
    """A device workspace for corr_build_ex (None when the algorithm needs none).  fmap2: the
    target map or just its shape [B, D, H, W]."""
    algo = default_algo() if algo is None else algo
    B, D, H, W = fmap2 if isinstance(fmap2, (tuple, list, torch.Size)) else fmap2.shape
    n = load().corr_build_workspace(algo, B, D, _nq(fmap1), H, W)
    if n == ctypes.c_size_t(-1).value:
        raise CorrError(CORR_EUNSUPPORTED, f"build algorithm {algo} does not support D = {D}")
    if n == 0:
        return None
    return torch.empty(n, dtype=torch.uint8, device=fmap1.device)


def build(fmap1, fmap2, levels, algo=None, workspace=None):
    """corr_build_ex into caller-allocated tiled levels (corr._alloc_pyramid).  fmap1 may be a row
    slab [B, D, rows, W] of the query map; fmap2 is the full target map [B, D, H, W].
    algo: BUILD_BF16X6 (default, see default_algo), BUILD_F16X3 or BUILD_FP32."""
    algo = default_algo() if algo is None else algo
    B, D, H, W = fmap2.shape
    a, b, pp = _dev(fmap1, "fmap1"), _dev(fmap2, "fmap2"), _ptrs(levels, "pyr")
    _check_levels(levels, B * _nq(fmap1), H, W, "pyr")
    if workspace is None:
        workspace = build_workspace(fmap1, fmap2, algo & 0xff)
    wp = 0 if workspace is None else workspace.data_ptr()
    wn = 0 if workspace is None else workspace.numel() * workspace.element_size()
    with torch.cuda.device(fmap1.device):
        _check(load().corr_build_ex(algo, a, _nq(fmap1), b, B, D, H, W, len(levels), pp, wp, wn,
                                    _stream(fmap1)))


REGION_PACK_QUERIES = 1


def build_region(fmap1, fmap2_rows, y0, y1, H, levels, workspace, pack_queries, algo=BUILD_BF16X6):
    """corr_build_region: the pyramid entries of target rows [y0, y1) (tiled levels, corr._alloc_pyramid)
    from fmap2_rows [B, D, y1 - y0, W]; workspace from build_workspace(fmap1, <full fmap2 shape>)."""
    B, D, rows, W = fmap2_rows.shape
    if rows != y1 - y0:
        raise ValueError(f"fmap2_rows has {rows} rows for the region [{y0}, {y1})")
    a, b, pp = _dev(fmap1, "fmap1"), _dev(fmap2_rows, "fmap2_rows"), _ptrs(levels, "pyr")
    _check_levels(levels, B * _nq(fmap1), H, W, "pyr")
    with torch.cuda.device(fmap1.device):
        _check(load().corr_build_region(algo, a, _nq(fmap1), b, y0, y1, B, D, H, W, len(levels), pp,
                                        workspace.data_ptr(), workspace.numel() * workspace.element_size(),
                                        REGION_PACK_QUERIES if pack_queries else 0, _stream(fmap1)))


def lookup(levels, coords, radius, out, H=None, W=None):
    """corr_lookup_rows: coords [B, 2, rows, W] -> out [B, L*K, rows, W].  (H, W) = target map
    (default: the coords' own, i.e. the reference shape)."""
    B = coords.shape[0]
    H = coords.shape[2] if H is None else H
    W = coords.shape[3] if W is None else W
    pp, c, o = _ptrs(levels, "pyr"), _dev(coords, "coords"), _dev(out, "out")
    _check_levels(levels, B * _nq(coords), H, W, "pyr")
    K = (2 * radius + 1) ** 2
    if out.numel() != B * len(levels) * K * _nq(coords):
        raise ValueError(f"out has {out.numel()} floats, the lookup writes {B}x{len(levels) * K}x{_nq(coords)}")
    with torch.cuda.device(coords.device):
        _check(load().corr_lookup_rows(pp, c, B, _nq(coords), H, W, len(levels), radius, o,
                                       _stream(coords)))


def lookup_bwd(coords, grad_out, radius, grad_levels, H=None, W=None):
    B = coords.shape[0]
    H = coords.shape[2] if H is None else H
    W = coords.shape[3] if W is None else W
    c, g, gp = _dev(coords, "coords"), _dev(grad_out, "grad_out"), _ptrs(grad_levels, "grad_pyr")
    _check_levels(grad_levels, B * _nq(coords), H, W, "grad_pyr", tiled=False)
    with torch.cuda.device(coords.device):
        _check(load().corr_lookup_bwd_rows(c, g, B, _nq(coords), H, W, len(grad_levels), radius, gp,
                                           _stream(coords)))


def pool_bwd(grad_levels, H, W):
    BN = grad_levels[0].shape[0]
    gp = _ptrs(grad_levels, "grad_pyr")
    _check_levels(grad_levels, BN, H, W, "grad_pyr", tiled=False)
    with torch.cuda.device(grad_levels[0].device):
        _check(load().corr_pool_bwd(gp, BN, H, W, len(grad_levels), _stream(grad_levels[0])))


def build_bwd(grad_c, fmap1, fmap2, algo=None):
    """Returns (dfmap1, dfmap2) for grad_c = dLoss/dcorr ([B*NQ, H*W] or any view of it).
    With a row slab fmap1, dfmap1 is the slab's and dfmap2 is this slab's partial sum.
    algo: BUILD_BF16X6 (default, see backward_algo), BUILD_F16X3 or BUILD_FP32 (corr_build_bwd_ex)."""
    algo = backward_algo() if algo is None else algo
    B, D, H, W = fmap2.shape
    for t, nm in ((grad_c, "grad_c"), (fmap1, "fmap1"), (fmap2, "fmap2")):
        _dev(t, nm)
    lib = load()
    NQ = _nq(fmap1)
    if grad_c.numel() != B * NQ * H * W:
        raise ValueError(f"grad_c has {grad_c.numel()} values, expected {B * NQ}x{H * W}")
    ws_bytes = lib.corr_build_bwd_ex_workspace(algo, B, D, NQ, H, W)
    if ws_bytes == ctypes.c_size_t(-1).value:
        raise CorrError(CORR_EUNSUPPORTED, f"unknown backward algorithm {algo}")
    df1 = torch.empty_like(fmap1)
    df2 = torch.empty_like(fmap2)
    ws = torch.empty(max(1, (ws_bytes + 3) // 4), dtype=torch.float32, device=fmap1.device)
    with torch.cuda.device(fmap1.device):
        _check(lib.corr_build_bwd_ex(algo, grad_c.data_ptr(), fmap1.data_ptr(), NQ, fmap2.data_ptr(), B,
                                     D, H, W, df1.data_ptr(), df2.data_ptr(), ws.data_ptr(),
                                     ws.numel() * 4, _stream(fmap1)))
    return df1, df2


def lookup_bwd_multi(coords_list, grad_list, radius, grad_levels, H=None, W=None):
    """corr_lookup_bwd_multi: the lookups' input-gradients, in order, into grad_levels, which it
    OVERWRITES (no zeroing needed)."""
    c0 = coords_list[0]
    B = c0.shape[0]
    H = c0.shape[2] if H is None else H
    W = c0.shape[3] if W is None else W
    cp, gp = _ptrs(coords_list, "coords"), _ptrs(grad_list, "grad_out")
    _check_levels(grad_levels, B * _nq(c0), H, W, "grad_pyr", tiled=False)
    with torch.cuda.device(c0.device):
        _check(load().corr_lookup_bwd_multi(cp, gp, len(coords_list), B, _nq(c0), H, W, len(grad_levels), radius,
                                            _ptrs(grad_levels, "grad_pyr"), _stream(c0)))


def pool_fold(grad_levels, B, H, W):
    """corr_pool_fold: the pool-backward chain folded into grad_levels[0] in one pass."""
    NQ = grad_levels[0].shape[0] // B
    _check_levels(grad_levels, B * NQ, H, W, "grad_pyr", tiled=False)
    with torch.cuda.device(grad_levels[0].device):
        _check(load().corr_pool_fold(_ptrs(grad_levels, "grad_pyr"), B, NQ, H, W, len(grad_levels),
                                     _stream(grad_levels[0])))


def exact_fold() -> bool:
    """ERAFT_AMD_EXACT_FOLD=1: corr_backward's fused fold replays grid_sampler_2d_backward's
    per-tap products bit for bit (CORR_BACKWARD_EXACT_FOLD) instead of the separable closed form
    (dC within ~1e-7 of the staged path, the default)."""
    return os.environ.get("ERAFT_AMD_EXACT_FOLD", "0") == "1"


def backward(coords_list, grad_list, radius, grad_levels, fmap1, fmap2, algo=None, exact=None):
    """corr_backward: (dfmap1, dfmap2) of one build and its lookups (all at once, in order).
    grad_levels: scratch gradient pyramid (overwritten; level 0 ends as dLoss/dcorr).
    algo: the GEMMs' algorithm (default: backward_algo()); exact: the bit-exact fold (default:
    exact_fold())."""
    algo = backward_algo() if algo is None else algo
    exact = exact_fold() if exact is None else exact
    B, D, H, W = fmap2.shape
    lib = load()
    NQ = _nq(fmap1)
    ws_bytes = lib.corr_backward_workspace(algo, B, D, NQ, H, W, radius)
    if exact:
        algo |= BACKWARD_EXACT_FOLD
    if ws_bytes == ctypes.c_size_t(-1).value:
        raise CorrError(CORR_EUNSUPPORTED, f"unknown backward algorithm {algo}")
    _check_levels(grad_levels, B * NQ, H, W, "grad_pyr", tiled=False)
    df1 = torch.empty_like(fmap1)
    df2 = torch.empty_like(fmap2)
    ws = torch.empty(max(1, (ws_bytes + 3) // 4), dtype=torch.float32, device=fmap1.device)
    cp, gp = _ptrs(coords_list, "coords"), _ptrs(grad_list, "grad_out")
    with torch.cuda.device(fmap1.device):
        _check(lib.corr_backward(algo, cp, gp, len(coords_list), _dev(fmap1, "fmap1"), NQ, _dev(fmap2, "fmap2"), B, D,
                                 H, W, len(grad_levels), radius, _ptrs(grad_levels, "grad_pyr"), df1.data_ptr(),
                                 df2.data_ptr(), ws.data_ptr(), ws.numel() * 4, _stream(fmap1)))
    return df1, df2


def fused_backward() -> bool:
    """ERAFT_AMD_FUSED_BWD=0 selects the per-lookup backward (lookup_bwd per call + pool_bwd +
    build_bwd) instead of corr_backward at the build's backward."""
    return os.environ.get("ERAFT_AMD_FUSED_BWD", "1") != "0"


def forward_splat(flow, out):
    """corr_forward_splat: flow [B, 2, H, W] -> out (same shape), caller-allocated."""
    B, C, H, W = flow.shape
    if C != 2:
        raise ValueError(f"flow must be [B, 2, H, W] (got {tuple(flow.shape)})")
    f, o = _dev(flow, "flow"), _dev(out, "out")
    lib = load()
    n = lib.corr_forward_splat_workspace(B, H, W)
    ws = torch.empty(max(1, (n + 3) // 4), dtype=torch.int32, device=flow.device)
    with torch.cuda.device(flow.device):
        _check(lib.corr_forward_splat(f, B, H, W, o, ws.data_ptr(), ws.numel() * 4, _stream(flow)))


def convex_upsample(flow, mask, out):
    """corr_convex_upsample: flow [N, 2, h, w], mask [N, 576, h, w] -> out [N, 2, 8h, 8w]."""
    N, C, h, w = flow.shape
    if C != 2 or tuple(mask.shape) != (N, 576, h, w) or tuple(out.shape) != (N, 2, 8 * h, 8 * w):
        raise ValueError(f"convex_upsample: flow {tuple(flow.shape)}, mask {tuple(mask.shape)}, "
                         f"out {tuple(out.shape)}")
    f, m, o = _dev(flow, "flow"), _dev(mask, "mask"), _dev(out, "out")
    with torch.cuda.device(flow.device):
        _check(load().corr_convex_upsample(f, m, N, h, w, o, _stream(flow)))


def convex_upsample_bwd(flow, mask, grad_out):
    """corr_convex_upsample_bwd: -> (dflow [N, 2, h, w], dmask [N, 576, h, w])."""
    N, _, h, w = flow.shape
    if tuple(mask.shape) != (N, 576, h, w) or tuple(grad_out.shape) != (N, 2, 8 * h, 8 * w):
        raise ValueError(f"convex_upsample_bwd: flow {tuple(flow.shape)}, mask {tuple(mask.shape)}, "
                         f"grad_out {tuple(grad_out.shape)}")
    lib = load()
    dflow = torch.empty_like(flow)
    dmask = torch.empty_like(mask)
    ws = torch.empty(lib.corr_convex_upsample_bwd_workspace(N, h, w), dtype=torch.uint8, device=flow.device)
    with torch.cuda.device(flow.device):
        _check(lib.corr_convex_upsample_bwd(_dev(flow, "flow"), _dev(mask, "mask"), _dev(grad_out, "grad_out"),
                                            N, h, w, _dev(dflow, "dflow"), _dev(dmask, "dmask"),
                                            ws.data_ptr(), ws.numel(), _stream(flow)))
    return dflow, dmask


def voxel_grid(x, y, t, p, out, normalize):
    """corr_voxel_grid: float32 device event arrays (x, y, t, p) -> out [C, H, W]."""
    C, H, W = out.shape
    M = x.numel()
    for v, nm in ((y, "y"), (t, "t"), (p, "p")):
        if v.numel() != M:
            raise ValueError(f"{nm} has {v.numel()} events, x has {M}")
    ptrs = [_dev(v, nm) if M else 0 for v, nm in ((x, "x"), (y, "y"), (t, "t"), (p, "p"))]
    o = _dev(out, "out")
    lib = load()
    n = lib.corr_voxel_grid_workspace(M, C, H, W)
    ws = torch.empty(max(1, (n + 3) // 4), dtype=torch.int32, device=out.device)
    with torch.cuda.device(out.device):
        _check(lib.corr_voxel_grid(*ptrs, M, C, H, W, int(bool(normalize)), o, ws.data_ptr(), ws.numel() * 4,
                                   _stream(out)))


def voxel_grid_tbilinear(events, out, normalize):
    """corr_voxel_grid_tbilinear: float64 device events [M, 4] (t, x, y, p) -> out [C, H, W]."""
    C, H, W = out.shape
    if events.dim() != 2 or events.shape[1] != 4:
        raise ValueError(f"events must be [M, 4] (t, x, y, p) (got {tuple(events.shape)})")
    if events.device.type != "cuda":
        raise RuntimeError(f"events is on {events.device}: eraft_amd runs only on an MI355X (HIP) device")
    if events.dtype != torch.float64 or not events.is_contiguous():
        raise TypeError("events must be a contiguous float64 tensor")
    M = events.shape[0]
    o = _dev(out, "out")
    lib = load()
    n = lib.corr_voxel_grid_tbilinear_workspace(M, C, H, W)
    ws = torch.empty(max(1, (n + 3) // 4), dtype=torch.int32, device=out.device)
    with torch.cuda.device(out.device):
        _check(lib.corr_voxel_grid_tbilinear(events.data_ptr() if M else 0, M, C, H, W, int(bool(normalize)), o,
                                             ws.data_ptr(), ws.numel() * 4, _stream(out)))


def lookup_conv_weights(weight):
    """corr_lookup_conv_weights: convc1.weight [256, C(, 1, 1)] -> the packed split (an opaque buffer)."""
    w = weight.detach().reshape(weight.shape[0], -1).contiguous().float()
    lib = load()
    packed = torch.empty((lib.corr_lookup_conv_weights_bytes() + 3) // 4, dtype=torch.float32, device=w.device)
    with torch.cuda.device(w.device):
        _check(lib.corr_lookup_conv_weights(_dev(w, "weight"), w.shape[0], w.shape[1], packed.data_ptr(),
                                            _stream(w)))
    return packed


def lookup_conv(levels, coords, radius, packed, bias, out, relu=True):
    """corr_lookup_conv: fused lookup + 1x1 conv (+ReLU) -> out [B, 256, H, W]."""
    B, _, H, W = coords.shape
    pp, c = _ptrs(levels, "pyr"), _dev(coords, "coords")
    _check_levels(levels, B * H * W, H, W, "pyr")
    pw, bs, o = _dev(packed, "packed_weight"), _dev(bias, "bias"), _dev(out, "out")
    with torch.cuda.device(coords.device):
        _check(load().corr_lookup_conv(pp, c, B, H, W, len(levels), radius, pw, bs, int(bool(relu)), o,
                                       _stream(coords)))


def lookup_conv_bwd(levels, coords, radius, packed, out, relu, grad_out, grad_weight=None, grad_bias=None,
                    grad_lookup=None):
    """corr_lookup_conv_bwd: the fused lookup + conv's backward.  grad_weight [256, C] /
    grad_bias [256] / grad_lookup [B, C, H, W] (fp32, contiguous; None = not computed) are
    overwritten."""
    B, _, H, W = coords.shape
    lib = load()
    pp, c = _ptrs(levels, "pyr"), _dev(coords, "coords")
    _check_levels(levels, B * H * W, H, W, "pyr")
    g = _dev(grad_out, "grad_out")
    o = _dev(out, "out") if relu else None
    opt = lambda t, name: None if t is None else _dev(t, name)
    ws, nbytes = None, 0
    if grad_weight is not None or grad_bias is not None:
        nbytes = lib.corr_lookup_conv_bwd_workspace(B, H, W, len(levels))
        ws = torch.empty((nbytes + 3) // 4, dtype=torch.float32, device=coords.device)
    with torch.cuda.device(coords.device):
        _check(lib.corr_lookup_conv_bwd(pp, c, B, H, W, len(levels), radius, _dev(packed, "packed_weight"), o,
                                        int(bool(relu)), g, opt(grad_weight, "grad_weight"),
                                        opt(grad_bias, "grad_bias"), opt(grad_lookup, "grad_lookup"),
                                        None if ws is None else ws.data_ptr(), nbytes, _stream(coords)))
