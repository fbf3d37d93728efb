"""Time the fused lookup + convc1 forward (corr_lookup_conv) and backward (corr_lookup_conv_bwd)
against the compositions they replace (forward: lookup, MIOpen conv2d, ReLU; backward: the round-3 torch
composition (HIP lookup into a 324-channel tensor, threshold backward, bias sum,
torch.bmm for dW, torch.matmul for W^T g) at config 4's shape (B 8, 36 x 48, 4 levels).
GPU only; prints one JSON line."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "e-raft_amd"))
from eraft_amd import CorrBlock, _lib  # noqa: E402
from eraft_amd.corr import _weight_pack  # noqa: E402


def main():
    args = sys.argv[1:]
    if args and args[0].startswith("--lib="):  # an A/B build of the library
        _lib._lib = _lib.load(args.pop(0)[6:])
    B, D, H, W, L, r = (int(x) for x in (args or [8, 256, 36, 48, 4, 4]))
    C = L * (2 * r + 1) ** 2
    dev = "cuda"
    g0 = torch.Generator(device="cpu").manual_seed(5)
    f1 = torch.randn(B, D, H, W, generator=g0).to(dev)
    f2 = torch.randn(B, D, H, W, generator=g0).to(dev)
    cb = CorrBlock(f1, f2, num_levels=L, radius=r)
    ys, xs = torch.meshgrid(torch.arange(H, dtype=torch.float32), torch.arange(W, dtype=torch.float32), indexing="ij")
    coords = (torch.stack([xs, ys])[None].repeat(B, 1, 1, 1) + 2.0 * torch.randn(B, 2, H, W, generator=g0)).to(dev)
    w = (0.05 * torch.randn(256, C, 1, 1, generator=g0)).to(dev)
    bias = (0.1 * torch.randn(256, generator=g0)).to(dev)
    g = torch.randn(B, 256, H, W, generator=g0).to(dev)
    out = cb.lookup_conv(coords, w, bias)
    packed = _weight_pack(w)
    dW = torch.empty(256, C, device=dev)
    db = torch.empty(256, device=dev)
    dl = torch.empty(B, C, H, W, device=dev)

    def fused():
        _lib.lookup_conv_bwd(cb._state.levels, coords, r, packed, out, True, g, dW, db, dl)

    def composed():
        gm = torch.where(out <= 0, torch.zeros((), device=dev), g)
        gf = gm.view(B, 256, H * W)
        gb = gf.sum(dim=(0, 2))
        lk = torch.empty(B, C, H, W, device=dev)
        _lib.lookup(cb._state.levels, coords, r, lk)
        gw = torch.bmm(gf, lk.view(B, C, H * W).transpose(1, 2)).sum(0)
        gl = torch.matmul(w.view(256, C).t(), gf)
        return gb, gw, gl

    import torch.nn.functional as F
    fout = torch.empty(B, 256, H, W, device=dev)

    def fwd_fused():  # corr_lookup_conv (what CorrBlock.lookup_conv runs at inference)
        _lib.lookup_conv(cb._state.levels, coords, r, packed, bias, fout, True)

    def fwd_composed():  # the reference composition: lookup, then convc1 (MIOpen) and ReLU
        torch.relu(F.conv2d(cb(coords), w, bias))

    res = {"shape": [B, D, H, W, L, r], "lib": os.path.basename(_lib.load()._name)}
    for name, fn in (("fused_us", fused), ("torch_composition_us", composed), ("fwd_fused_us", fwd_fused),
                     ("fwd_lookup_conv2d_relu_us", fwd_composed)):
        for _ in range(5):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        n = 50
        e0.record()
        for _ in range(n):
            fn()
        e1.record()
        torch.cuda.synchronize()
        res[name] = round(e0.elapsed_time(e1) * 1000.0 / n, 2)
    gb, gw, gl = composed()
    fused()
    torch.cuda.synchronize()
    res["max_rel_dW"] = float((dW - gw).abs().max() / gw.abs().max())
    res["max_rel_dlk"] = float((dl.view(B, C, -1) - gl).abs().max() / gl.abs().max())
    res["max_rel_db"] = float((db - gb).abs().max() / gb.abs().max())
    print(json.dumps(res))


if __name__ == "__main__":
    main()
