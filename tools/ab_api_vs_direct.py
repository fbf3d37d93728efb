"""A/B the bench step through the library calls (one preallocated pyramid, 12 preallocated
outputs) against the drop-in CorrBlock API (pyramid and each output allocated per call from the
graph pool), alternating, to separate an order / clock effect from a memory-reuse effect.
Also the direct path with ONE reused output buffer.  GPU only; prints JSON lines."""
import json
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "e-raft_amd"))
from eraft_amd import CorrBlock, _lib  # noqa: E402
from eraft_amd.corr import _alloc_pyramid  # noqa: E402

SHAPES = {"dsec": (1, 256, 60, 80), "mvsec": (16, 256, 36, 44)}


def main():
    name = sys.argv[1] if len(sys.argv) > 1 else "dsec"
    B, D, H, W = SHAPES[name]
    L, r, iters, steps = 4, 4, 12, 50
    dev = "cuda"
    g = torch.Generator(device=dev).manual_seed(1234)
    f1 = torch.randn(B, D, H, W, device=dev, generator=g)
    f2 = torch.randn(B, D, H, W, device=dev, generator=g)
    base = torch.stack(torch.meshgrid(torch.arange(H, device=dev), torch.arange(W, device=dev),
                                      indexing="ij")[::-1]).float()[None].repeat(B, 1, 1, 1)
    coords = [(base + 0.5 * t * torch.randn(B, 2, H, W, device=dev, generator=g)).contiguous()
              for t in range(iters)]
    pyr = _alloc_pyramid(B, H, W, L, f1)
    outs = [torch.empty(B, L * 81, H, W, device=dev) for _ in range(iters)]
    one = torch.empty(B, L * 81, H, W, device=dev)
    algo = _lib.default_algo()
    ws = _lib.build_workspace(f1, f2, algo)
    stream = torch.cuda.Stream()

    def direct():
        _lib.build(f1, f2, pyr, algo, ws)
        for c, o in zip(coords, outs):
            _lib.lookup(pyr, c, r, o, H, W)

    def direct_one():
        _lib.build(f1, f2, pyr, algo, ws)
        for c in coords:
            _lib.lookup(pyr, c, r, one, H, W)

    def api():
        cb = CorrBlock(f1, f2, num_levels=L, radius=r)
        for c in coords:
            cb(c)

    graphs = {}
    with torch.cuda.stream(stream):
        for nm, fn in (("direct", direct), ("direct_one_out", direct_one), ("api", api)):
            fn()
            torch.cuda.synchronize()
            gr = torch.cuda.CUDAGraph()
            with torch.cuda.graph(gr, stream=stream):
                fn()
            graphs[nm] = gr
        res = {k: [] for k in graphs}
        for rnd in range(4):
            for nm, gr in graphs.items():
                for _ in range(10):
                    gr.replay()
                torch.cuda.synchronize()
                t0 = time.perf_counter()
                for _ in range(steps):
                    gr.replay()
                torch.cuda.synchronize()
                res[nm].append(round(B * steps / (time.perf_counter() - t0), 1))
    print(json.dumps({"shape": name, "frame_pairs_per_s": res}))


if __name__ == "__main__":
    main()
