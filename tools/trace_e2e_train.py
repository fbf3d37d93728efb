"""One E-RAFT training step (config 4's 288x384 crops, B=2, 4 GRU iterations, sequence loss,
backward to every parameter) through the fused lookup + convc1 (CorrBlock.lookup_conv and its
corr_lookup_conv_bwd backward), repeated a few times, for a rocprofv3 kernel trace: the trace
shows which kernels a training step runs (no lookup_kernel: the 324-channel lookup output is
never written, forward or backward).  GPU only.
    rocprofv3 --kernel-trace --stats -d gpurun_out/prof_e2e_train -o run -- python3 tools/trace_e2e_train.py
"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "e-raft_amd"), os.path.join(ROOT, "tests", "golden")]
import prng  # noqa: E402
from eraft_amd.model import ERAFT  # noqa: E402


def main():
    dev = "cuda:0"
    model = ERAFT({"subtype": "warm_start"}, n_first_channels=15)
    sd = model.state_dict()
    with torch.no_grad():
        for name, t in sd.items():
            v = prng.param_init(name, tuple(t.shape))
            if v is not None:
                t.copy_(torch.from_numpy(v))
    model = model.to(dev).train()
    assert model.fuse_lookup_conv
    im1 = torch.from_numpy(prng.voxel_grid(1, (2, 15, 288, 384))).to(dev)
    im2 = torch.from_numpy(prng.voxel_grid(3, (2, 15, 288, 384))).to(dev)
    gt = torch.from_numpy(prng.gauss(5, (2, 2, 288, 384), 2.0)).to(dev)
    for _ in range(3):
        model.zero_grad(set_to_none=True)
        _, preds = model(im1, im2, iters=4)
        loss = sum(0.8 ** (len(preds) - 1 - i) * (p - gt).abs().mean() for i, p in enumerate(preds))
        loss.backward()
    torch.cuda.synchronize()
    g = model.update_block.encoder.convc1.weight.grad
    print("convc1 grad finite:", bool(torch.isfinite(g).all()), "fnet grad sum:",
          float(model.fnet.conv1.weight.grad.abs().sum()))


if __name__ == "__main__":
    main()
