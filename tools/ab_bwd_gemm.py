"""A/B: corr_build_bwd_ex (F16X3) of the current library vs a previous build of it
(tools/_build/libcorr_prev.so, the packed-convert GEMMs): dfmap1 / dfmap2 must be bit-identical.
Includes rows whose max is inf / tiny and NaN entries (the split's edge cases)."""
import ctypes
import sys

import numpy as np
import torch

sys.path.insert(0, "e-raft_amd")
from eraft_amd import _lib  # noqa: E402

cur = _lib.load()
prev = ctypes.CDLL("tools/_build/libcorr_prev.so", mode=ctypes.RTLD_LOCAL)
vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
for L in (cur, prev):
    L.corr_build_bwd_ex_workspace.argtypes = [i, i, i, i, i, i]
    L.corr_build_bwd_ex_workspace.restype = sz
    L.corr_build_bwd_ex.argtypes = [i, vp, vp, i, vp, i, i, i, i, vp, vp, vp, sz, vp]
dev = "cuda:0"
ok = True
for (B, D, H, W, seed) in [(2, 32, 18, 24, 1), (1, 20, 17, 23, 2), (8, 256, 36, 48, 3), (1, 64, 60, 80, 4)]:
    g = torch.Generator(device=dev).manual_seed(seed)
    N = H * W
    f1 = torch.randn(B, D, H, W, device=dev, generator=g)
    f2 = torch.randn(B, D, H, W, device=dev, generator=g)
    gc = torch.randn(B * N, N, device=dev, generator=g)
    gc[::7] *= 1e-30
    gc[3, 5] = float("inf")
    gc[4, :3] = float("nan")
    f1[0, 1] *= 1e20
    outs = []
    for L in (cur, prev):
        wsb = L.corr_build_bwd_ex_workspace(1, B, D, N, H, W)
        ws = torch.empty((wsb + 3) // 4, device=dev)
        d1, d2 = torch.empty_like(f1), torch.empty_like(f2)
        rc = L.corr_build_bwd_ex(1, gc.data_ptr(), f1.data_ptr(), N, f2.data_ptr(), B, D, H, W, d1.data_ptr(),
                                 d2.data_ptr(), ws.data_ptr(), wsb, torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc
        torch.cuda.synchronize()
        outs.append((d1.cpu().numpy(), d2.cpu().numpy()))
    for a, b in zip(outs[0], outs[1]):
        same = np.array_equal(a.view(np.uint32), b.view(np.uint32))
        ok &= same
        print((B, D, H, W), "bit-identical" if same else f"DIFFER ({(a.view(np.uint32) != b.view(np.uint32)).sum()} words)")
print("ALL BIT-IDENTICAL" if ok else "MISMATCH")
sys.exit(0 if ok else 1)
