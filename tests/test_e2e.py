"""End-to-end check of the north_star: the full E-RAFT forward at DSEC 480x640 (15-bin
voxels, 12 GRU iterations, random-init weights) with the MI355X CorrBlock must give the same
flow as the reference model — mean EPE difference <= 0.01 px, cold and warm-start.

Golden: tests/golden/g_e2e_dsec.npz, produced by the reference ERAFT
(model/eraft.py:37-146) on CPU with weights from prng.param_init (keyed by parameter name),
see tests/golden/make_golden.py::case_e2e.  The warm-start flow_init is the reference's own
forward splat of the cold result (utils/image_utils.py:52-83), stored in the golden.
"""
import numpy as np
import pytest
import torch

import prng
from _util import load

EPE_TOL = 0.01  # px (north_star)


def _model(bins):
    from eraft_amd.model import ERAFT
    m = ERAFT({"subtype": "warm_start"}, n_first_channels=bins).eval()
    sd = m.state_dict()
    with torch.no_grad():
        for name, t in sd.items():
            v = prng.param_init(name, tuple(t.shape))
            if v is not None:
                t.copy_(torch.from_numpy(v))
    return m


def test_state_dict_matches_reference_checkpoint_format():
    """Every parameter / buffer name and shape of the reference model exists here (so a
    reference checkpoint loads with load_state_dict, main.py:116-117)."""
    g = load("g_e2e_dsec")
    bins = int(g["meta"][3])
    from eraft_amd.model import ERAFT
    m = ERAFT({"subtype": "warm_start"}, n_first_channels=bins)
    mine = [f"{k}:{tuple(v.shape)}" for k, v in m.state_dict().items()]
    assert mine == list(g["state_keys"])


def _epe(a, b):
    return float(np.sqrt(((np.asarray(a, np.float64) - b) ** 2).sum(1)).mean())


@pytest.mark.gpu
def test_e2e_flow_matches_reference(monkeypatch):
    """Cold and warm start with the unfused lookup + MIOpen convc1 (the fused default is the
    next test)."""
    from eraft_amd.model import ERAFT
    monkeypatch.setattr(ERAFT, "fuse_lookup_conv", False)
    g = load("g_e2e_dsec")
    seed, H, W, bins, iters = (int(v) for v in g["meta"])
    dev = "cuda:0"
    im1 = torch.from_numpy(prng.voxel_grid(seed, (1, bins, H, W))).to(dev)
    im2 = torch.from_numpy(prng.voxel_grid(seed + 2, (1, bins, H, W))).to(dev)
    model = _model(bins).to(dev)
    with torch.no_grad():
        low, ups = model(im1, im2, iters=iters)
    e_low = _epe(low.cpu().numpy(), g["low"])
    e_up = _epe(ups[-1][..., ::4, ::4].cpu().numpy(), g["up_sub"])
    print(f"cold: EPE lowres {e_low:.2e} px, full-res {e_up:.2e} px (|flow| ~ {g['up_mean_abs'][0]:.1f})")
    assert e_low <= EPE_TOL and e_up <= EPE_TOL

    model_w = _model(bins).to(dev)
    finit = torch.from_numpy(g["flow_init"]).to(dev)
    with torch.no_grad():
        low_w, ups_w = model_w(im1, im2, iters=iters, flow_init=finit)
    e_low_w = _epe(low_w.cpu().numpy(), g["low_warm"])
    e_up_w = _epe(ups_w[-1][..., ::4, ::4].cpu().numpy(), g["up_warm_sub"])
    print(f"warm: EPE lowres {e_low_w:.2e} px, full-res {e_up_w:.2e} px")
    assert e_low_w <= EPE_TOL and e_up_w <= EPE_TOL


@pytest.mark.gpu
def test_e2e_training_step_runs_through_hip_backward():
    """Config 4 shape (288x384 crops, B=2 here): forward + sequence-loss backward through
    the HIP CorrBlock; gradients reach the feature encoder and are finite."""
    dev = "cuda:0"
    model = _model(15).to(dev).train()
    im1 = torch.from_numpy(prng.voxel_grid(1, (2, 15, 288, 384))).to(dev)
    im2 = torch.from_numpy(prng.voxel_grid(3, (2, 15, 288, 384))).to(dev)
    gt = torch.from_numpy(prng.gauss(5, (2, 2, 288, 384), 2.0)).to(dev)
    _, preds = model(im1, im2, iters=4)
    loss = sum(0.8 ** (len(preds) - 1 - i) * (p - gt).abs().mean() for i, p in enumerate(preds))
    loss.backward()
    g = model.fnet.conv1.weight.grad
    assert g is not None and torch.isfinite(g).all() and g.abs().sum() > 0


@pytest.mark.gpu
def test_e2e_with_fused_lookup_conv_matches_reference(monkeypatch):
    """The same cold-start golden with the lookup fused into convc1 (corr_lookup_conv)."""
    from eraft_amd.model import ERAFT
    monkeypatch.setattr(ERAFT, "fuse_lookup_conv", True)
    g = load("g_e2e_dsec")
    seed, H, W, bins, iters = (int(v) for v in g["meta"])
    dev = "cuda:0"
    im1 = torch.from_numpy(prng.voxel_grid(seed, (1, bins, H, W))).to(dev)
    im2 = torch.from_numpy(prng.voxel_grid(seed + 2, (1, bins, H, W))).to(dev)
    model = _model(bins).to(dev)
    with torch.no_grad():
        low, ups = model(im1, im2, iters=iters)
    assert _epe(low.cpu().numpy(), g["low"]) <= EPE_TOL
    assert _epe(ups[-1][..., ::4, ::4].cpu().numpy(), g["up_sub"]) <= EPE_TOL
