"""A/B of bench.py's step (the build + 12 lookups, one HIP graph per library) between the in-tree
library and tools/_build/libcorr_alt.so, alternated in ONE process on the same inputs and
pyramid memory, so box-to-box spread drops out.  Also checks that both produce the same pyramid
and lookup bits.
    python tools/ab_step.py [workload] [trials]      (workloads as bench.py: dsec, train, ...)
Prints per-library median ms per step and the per-kernel medians of a graph of each kernel."""
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "e-raft_amd"))
sys.path.insert(0, ROOT)
from eraft_amd import _lib  # noqa: E402
from eraft_amd.corr import _alloc_pyramid  # noqa: E402

from bench import WORKLOADS  # noqa: E402


def main():
    wl = sys.argv[1] if len(sys.argv) > 1 else "dsec"
    trials = int(sys.argv[2]) if len(sys.argv) > 2 else 7
    B, D, H, W, L, r, iters = WORKLOADS[wl]
    libs = {"cur": _lib.load(), "alt": _lib.load(os.path.join(ROOT, "tools", "_build", "libcorr_alt.so"))}
    dev = torch.device("cuda", 0)
    g = torch.Generator(device=dev).manual_seed(1234)
    f1 = torch.randn(B, D, H, W, device=dev, generator=g)
    f2 = torch.randn(B, D, H, W, device=dev, generator=g)
    base = torch.stack(torch.meshgrid(torch.arange(H, device=dev), torch.arange(W, device=dev),
                                      indexing="ij")[::-1]).float()[None].repeat(B, 1, 1, 1)
    coords = [(base + 0.5 * t * torch.randn(B, 2, H, W, device=dev, generator=g)).contiguous() for t in range(iters)]
    K = (2 * r + 1) ** 2
    algo = _lib.default_algo()
    pyr = _alloc_pyramid(B, H, W, L, f1)
    ws = _lib.build_workspace(f1, f2, algo)
    out = torch.empty(B, L * K, H, W, device=dev)
    stream = torch.cuda.Stream()

    def step():
        _lib.build(f1, f2, pyr, algo, ws)
        for c in coords:
            _lib.lookup(pyr, c, r, out, H, W)

    bits, graphs = {}, {}
    with torch.cuda.stream(stream):
        for name, lib in libs.items():
            _lib._lib = lib
            step()
            torch.cuda.synchronize()
            bits[name] = ([p.cpu().numpy().copy() for p in pyr], out.cpu().numpy().copy())
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=stream):
                step()
            graphs[name] = gr
    same = all(np.array_equal(a.view(np.uint32), b.view(np.uint32))
               for a, b in zip(bits["cur"][0] + [bits["cur"][1]], bits["alt"][0] + [bits["alt"][1]]))
    print(f"{wl}: pyramid and lookup output bit-identical: {same}")
    steps = 200 if wl in ("dsec", "mvsec_crop") else 50
    res = {n: [] for n in graphs}
    for t in range(trials + 1):
        for n, gr in graphs.items():
            for _ in range(10):
                gr.replay()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(steps):
                gr.replay()
            torch.cuda.synchronize()
            if t:  # trial 0 warms both
                res[n].append((time.perf_counter() - t0) / steps * 1e3)
    for n, v in res.items():
        v = sorted(v)
        print(f"{wl} {n}: step median {v[len(v) // 2]:.4f} ms  min {v[0]:.4f}  ({B / v[len(v) // 2] * 1e3:.0f} pairs/s)")
    _lib._lib = libs["cur"]
    return 0 if same else 1


if __name__ == "__main__":
    sys.exit(main())
