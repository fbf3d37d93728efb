"""A/B of corr_build_bwd_ex (BF16X6: dF1 + dF2 GEMMs and their split-K sums) between the current
library and a previous build of it (tools/_build/libcorr_prev.so): bit-identity of dfmap1 /
dfmap2 on shapes with edge cases (inf / NaN / tiny dC entries, huge features), then HIP-event
timing of both, interleaved, at the train shape (config 4: B8 36x48 D256).

    python tools/ab_bwd_bf16.py [rounds]
"""
import ctypes
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "e-raft_amd"))
from eraft_amd import _lib  # noqa: E402

ALGO = 2  # bf16x6
cur = _lib.load()
prev = ctypes.CDLL(os.path.join(ROOT, "tools/_build/libcorr_prev.so"), mode=ctypes.RTLD_LOCAL)
vp, i, sz = ctypes.c_void_p, ctypes.c_int, ctypes.c_size_t
for L in (cur, prev):
    L.corr_build_bwd_ex_workspace.argtypes = [i, i, i, i, i, i]
    L.corr_build_bwd_ex_workspace.restype = sz
    L.corr_build_bwd_ex.argtypes = [i, vp, vp, i, vp, i, i, i, i, vp, vp, vp, sz, vp]
dev = "cuda:0"


def runner(L, gc, f1, f2, B, D, H, W):
    N = H * W
    wsb = L.corr_build_bwd_ex_workspace(ALGO, B, D, N, H, W)
    ws = torch.empty((wsb + 3) // 4, device=dev)
    d1, d2 = torch.empty_like(f1), torch.empty_like(f2)

    def run():
        rc = L.corr_build_bwd_ex(ALGO, gc.data_ptr(), f1.data_ptr(), N, f2.data_ptr(), B, D, H, W, d1.data_ptr(),
                                 d2.data_ptr(), ws.data_ptr(), wsb, torch.cuda.current_stream().cuda_stream)
        assert rc == 0, rc
    return run, d1, d2


ok = True
for (B, D, H, W, seed) in [(2, 32, 18, 24, 1), (1, 20, 17, 23, 2), (8, 256, 36, 48, 3), (1, 256, 60, 80, 4),
                           (3, 64, 20, 36, 5)]:
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
        run, d1, d2 = runner(L, gc, f1, f2, B, D, H, W)
        run()
        torch.cuda.synchronize()
        outs.append((d1.cpu().numpy(), d2.cpu().numpy()))
    for name, a, b in zip(("dF1", "dF2"), outs[0], outs[1]):
        same = np.array_equal(a.view(np.uint32), b.view(np.uint32))
        ok &= same
        print((B, D, H, W), name, "bit-identical" if same else f"DIFFER ({(a.view(np.uint32) != b.view(np.uint32)).sum()} words)",
              flush=True)

rounds = int(sys.argv[1]) if len(sys.argv) > 1 else 20
for (B, D, H, W) in [(8, 256, 36, 48), (1, 256, 60, 80)]:
    g = torch.Generator(device=dev).manual_seed(11)
    N = H * W
    f1 = torch.randn(B, D, H, W, device=dev, generator=g)
    f2 = torch.randn(B, D, H, W, device=dev, generator=g)
    gc = torch.randn(B * N, N, device=dev, generator=g)
    runs = {"cur": runner(cur, gc, f1, f2, B, D, H, W)[0], "prev": runner(prev, gc, f1, f2, B, D, H, W)[0]}
    ts = {k: [] for k in runs}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(rounds):
        for k, run in runs.items():
            run()
            e0.record()
            for _ in range(10):
                run()
            e1.record()
            e1.synchronize()
            ts[k].append(e0.elapsed_time(e1) * 100)  # us per call
    print((B, D, H, W), "  ".join(f"{k}: median {np.median(v):.1f} us min {np.min(v):.1f}" for k, v in ts.items()),
          flush=True)
print("ALL BIT-IDENTICAL" if ok else "MISMATCH")
sys.exit(0 if ok else 1)
