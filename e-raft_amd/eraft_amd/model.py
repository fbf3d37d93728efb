"""Host-side E-RAFT forward around the MI355X CorrBlock (the caller of the hot path).

A restatement, in plain PyTorch, of the reference model that calls CorrBlock
(AhmedHumais/E-RAFT model/eraft.py:37-146, model/extractor.py, model/update.py,
utils/image_utils.py:85-123).  The dense convolutions stay on PyTorch-ROCm/MIOpen (out of
scope); only the correlation build and lookups go through libcorr_mi355x.so.

Module and parameter names follow the reference so that a reference checkpoint's
``state_dict`` loads unchanged (main.py:116-117: ``model.load_state_dict(ckpt['model'])``).
It exists to run the north_star's end-to-end check (flow EPE vs the reference model on
identical random weights, tests/test_e2e.py) and as the integration example.
"""
from __future__ import annotations

import os

import torch
import torch.nn as nn
import torch.nn.functional as F

from .corr import CorrBlock
from .utils import coords_grid


def _norm(kind: str, ch: int, groups: int = 8):
    if kind == "group":
        return nn.GroupNorm(num_groups=groups, num_channels=ch)
    if kind == "batch":
        return nn.BatchNorm2d(ch)
    if kind == "instance":
        return nn.InstanceNorm2d(ch)
    return nn.Sequential()


class ResidualBlock(nn.Module):
    """3x3-3x3 residual unit with an optional strided 1x1 projection (extractor.py:7-52)."""

    def __init__(self, cin, cout, norm_fn="group", stride=1):
        super().__init__()
        self.conv1 = nn.Conv2d(cin, cout, 3, padding=1, stride=stride)
        self.conv2 = nn.Conv2d(cout, cout, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)
        g = cout // 8
        self.norm1 = _norm(norm_fn, cout, g)
        self.norm2 = _norm(norm_fn, cout, g)
        if stride != 1:
            self.norm3 = _norm(norm_fn, cout, g)
            self.downsample = nn.Sequential(nn.Conv2d(cin, cout, 1, stride=stride), self.norm3)
        else:
            self.downsample = None

    def forward(self, x):
        y = self.relu(self.norm1(self.conv1(x)))
        y = self.relu(self.norm2(self.conv2(y)))
        skip = x if self.downsample is None else self.downsample(x)
        return self.relu(skip + y)


class BasicEncoder(nn.Module):
    """7x7/2 stem + three residual stages (64, 96/2, 128/2) + 1x1 head (extractor.py:137-189)."""

    def __init__(self, output_dim=128, norm_fn="batch", dropout=0.0, n_first_channels=1):
        super().__init__()
        self.norm_fn = norm_fn
        self.norm1 = _norm(norm_fn, 64)
        self.conv1 = nn.Conv2d(n_first_channels, 64, 7, stride=2, padding=3)
        self.relu1 = nn.ReLU(inplace=True)
        stages, cin = [], 64
        for cout, stride in ((64, 1), (96, 2), (128, 2)):
            stages.append(nn.Sequential(ResidualBlock(cin, cout, norm_fn, stride),
                                        ResidualBlock(cout, cout, norm_fn, 1)))
            cin = cout
        self.layer1, self.layer2, self.layer3 = stages
        self.conv2 = nn.Conv2d(128, output_dim, 1)
        self.dropout = nn.Dropout2d(p=dropout) if dropout > 0 else None
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, (nn.BatchNorm2d, nn.InstanceNorm2d, nn.GroupNorm)):
                if m.weight is not None:
                    nn.init.constant_(m.weight, 1)
                if m.bias is not None:
                    nn.init.constant_(m.bias, 0)

    def forward(self, x):
        pair = isinstance(x, (list, tuple))
        if pair:
            n = x[0].shape[0]
            x = torch.cat(x, dim=0)
        x = self.relu1(self.norm1(self.conv1(x)))
        x = self.layer3(self.layer2(self.layer1(x)))
        x = self.conv2(x)
        if self.training and self.dropout is not None:
            x = self.dropout(x)
        return torch.split(x, [n, n], dim=0) if pair else x


class BasicMotionEncoder(nn.Module):
    """Consumes the lookup output: convc1 is the 324 -> 256 1x1 (update.py:63-82)."""

    def __init__(self, corr_levels=4, corr_radius=4):
        super().__init__()
        planes = corr_levels * (2 * corr_radius + 1) ** 2
        self.convc1 = nn.Conv2d(planes, 256, 1)
        self.convc2 = nn.Conv2d(256, 192, 3, padding=1)
        self.convf1 = nn.Conv2d(2, 128, 7, padding=3)
        self.convf2 = nn.Conv2d(128, 64, 3, padding=1)
        self.conv = nn.Conv2d(64 + 192, 128 - 2, 3, padding=1)

    def forward(self, flow, corr, fused=False):
        # fused: corr already is relu(convc1(lookup)) (CorrBlock.lookup_conv)
        c = F.relu(self.convc2(corr if fused else F.relu(self.convc1(corr))))
        f = F.relu(self.convf2(F.relu(self.convf1(flow))))
        return torch.cat([F.relu(self.conv(torch.cat([c, f], dim=1))), flow], dim=1)


class SepConvGRU(nn.Module):
    """Horizontal (1x5) then vertical (5x1) convolutional GRU (update.py:34-61)."""

    def __init__(self, hidden_dim=128, input_dim=192 + 128):
        super().__init__()
        c = hidden_dim + input_dim
        for tag, k, p in (("1", (1, 5), (0, 2)), ("2", (5, 1), (2, 0))):
            for gate in "zrq":
                setattr(self, f"conv{gate}{tag}", nn.Conv2d(c, hidden_dim, k, padding=p))

    def _step(self, h, x, tag):
        hx = torch.cat([h, x], dim=1)
        z = torch.sigmoid(getattr(self, f"convz{tag}")(hx))
        r = torch.sigmoid(getattr(self, f"convr{tag}")(hx))
        q = torch.tanh(getattr(self, f"convq{tag}")(torch.cat([r * h, x], dim=1)))
        return (1 - z) * h + z * q

    def forward(self, h, x):
        return self._step(self._step(h, x, "1"), x, "2")


class FlowHead(nn.Module):
    def __init__(self, input_dim=128, hidden_dim=256):
        super().__init__()
        self.conv1 = nn.Conv2d(input_dim, hidden_dim, 3, padding=1)
        self.conv2 = nn.Conv2d(hidden_dim, 2, 3, padding=1)
        self.relu = nn.ReLU(inplace=True)

    def forward(self, x):
        return self.conv2(self.relu(self.conv1(x)))


class BasicUpdateBlock(nn.Module):
    """Motion encoder + SepConvGRU + flow head + convex-upsampling mask (update.py:85-107)."""

    def __init__(self, corr_levels=4, corr_radius=4, hidden_dim=128):
        super().__init__()
        self.encoder = BasicMotionEncoder(corr_levels, corr_radius)
        self.gru = SepConvGRU(hidden_dim=hidden_dim, input_dim=128 + hidden_dim)
        self.flow_head = FlowHead(hidden_dim, hidden_dim=256)
        self.mask = nn.Sequential(nn.Conv2d(128, 256, 3, padding=1), nn.ReLU(inplace=True),
                                  nn.Conv2d(256, 64 * 9, 1))

    def forward(self, net, inp, corr, flow, fused=False):
        motion = self.encoder(flow, corr, fused)
        net = self.gru(net, torch.cat([inp, motion], dim=1))
        return net, 0.25 * self.mask(net), self.flow_head(net)


class ImagePadder:
    """Zero-pads top/left to a multiple of min_size (utils/image_utils.py:85-123)."""

    def __init__(self, min_size=64):
        self.min_size = min_size
        self.pad_height = self.pad_width = None

    def pad(self, image):
        h, w = image.shape[-2:]
        ph = (self.min_size - h % self.min_size) % self.min_size
        pw = (self.min_size - w % self.min_size) % self.min_size
        if self.pad_width is None:
            self.pad_height, self.pad_width = ph, pw
        elif (ph, pw) != (self.pad_height, self.pad_width):
            raise RuntimeError("ImagePadder: image size changed between calls")
        return F.pad(image, (self.pad_width, 0, self.pad_height, 0))

    def unpad(self, image):
        return image[..., self.pad_height:, self.pad_width:]


class _ConvexUpsampleFn(torch.autograd.Function):
    """ERAFT.upsample_flow on the MI355X: forward corr_convex_upsample, backward
    corr_convex_upsample_bwd (softmax and unfold backward fused; the 9x-expanded product of
    the torch composition is never materialised in either direction)."""

    @staticmethod
    def forward(ctx, flow, mask):
        from . import _lib
        n, _, h, w = flow.shape
        out = torch.empty((n, 2, 8 * h, 8 * w), dtype=torch.float32, device=flow.device)
        _lib.convex_upsample(flow, mask, out)
        ctx.save_for_backward(flow, mask)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        from . import _lib
        flow, mask = ctx.saved_tensors
        dflow, dmask = _lib.convex_upsample_bwd(flow, mask, grad_out.contiguous())
        return dflow, dmask


class ERAFT(nn.Module):
    """E-RAFT (model/eraft.py:37-146) with the MI355X CorrBlock on its hot path."""

    hidden_dim = 128
    context_dim = 128
    corr_levels = 4
    corr_radius = 4
    # lookup fused with convc1 (corr_lookup_conv, bf16x6 MFMA; in training its backward is
    # corr_lookup_conv_bwd); ERAFT_AMD_FUSE_CONV=0 keeps lookup + MIOpen convc1.  DSEC: 20.1 vs
    # 38.9 us per GRU iteration (profiles/r04k_conv_fwd_bwd_timing.jsonl)
    fuse_lookup_conv = os.environ.get("ERAFT_AMD_FUSE_CONV", "1") == "1"

    def __init__(self, config, n_first_channels):
        super().__init__()
        self.subtype = config["subtype"].lower()
        if self.subtype not in ("standard", "warm_start"):
            raise ValueError(f"unknown subtype {self.subtype}")
        self.image_padder = ImagePadder(min_size=32)
        hdim, cdim = self.hidden_dim, self.context_dim
        self.fnet = BasicEncoder(output_dim=256, norm_fn="instance", dropout=0,
                                 n_first_channels=n_first_channels)
        self.cnet = BasicEncoder(output_dim=hdim + cdim, norm_fn="batch", dropout=0,
                                 n_first_channels=n_first_channels)
        self.update_block = BasicUpdateBlock(self.corr_levels, self.corr_radius, hidden_dim=hdim)

    def freeze_bn(self):
        for m in self.modules():
            if isinstance(m, nn.BatchNorm2d):
                m.eval()

    @staticmethod
    def upsample_flow(flow, mask):
        """Convex combination of 3x3 neighbours, x8 (eraft.py:75-86).  On the MI355X: the
        one-pass HIP kernel (corr_convex_upsample), with its HIP backward under autograd
        (_ConvexUpsampleFn); on the CPU the torch composition below (what bench.py's CPU
        baseline runs)."""
        if flow.is_cuda:
            return _ConvexUpsampleFn.apply(flow.float().contiguous(), mask.float().contiguous())
        n, _, h, w = flow.shape
        mask = torch.softmax(mask.view(n, 1, 9, 8, 8, h, w), dim=2)
        up = F.unfold(8 * flow, [3, 3], padding=1).view(n, 2, 9, 1, 1, h, w)
        up = torch.sum(mask * up, dim=2).permute(0, 1, 4, 2, 5, 3)
        return up.reshape(n, 2, 8 * h, 8 * w)

    def forward(self, image1, image2, iters=12, flow_init=None, upsample=True):
        image1 = self.image_padder.pad(image1).contiguous()
        image2 = self.image_padder.pad(image2).contiguous()
        fmap1, fmap2 = self.fnet([image1, image2])
        corr_fn = CorrBlock(fmap1.float(), fmap2.float(), num_levels=self.corr_levels,
                            radius=self.corr_radius)
        net, inp = torch.split(self.cnet(image2), [self.hidden_dim, self.context_dim], dim=1)
        net, inp = torch.tanh(net), torch.relu(inp)
        n, _, h, w = image1.shape
        coords0 = coords_grid(n, h // 8, w // 8, device=image1.device)
        coords1 = coords0.clone()
        if flow_init is not None:
            coords1 = coords1 + flow_init
        predictions = []
        # on the MI355X the lookup feeds convc1 on-chip (corr_lookup_conv), at inference and, with
        # its autograd backward (corr._LookupConvFn), in training
        fuse = (self.fuse_lookup_conv and image1.is_cuda and self.corr_radius == 4
                and hasattr(corr_fn, "lookup_conv"))
        for _ in range(iters):
            coords1 = coords1.detach()
            if fuse:
                enc = self.update_block.encoder
                corr = corr_fn.lookup_conv(coords1, enc.convc1.weight, enc.convc1.bias)
            else:
                corr = corr_fn(coords1)
            net, up_mask, delta = self.update_block(net, inp, corr, coords1 - coords0, fuse)
            coords1 = coords1 + delta
            predictions.append(self.image_padder.unpad(self.upsample_flow(coords1 - coords0, up_mask)))
        return coords1 - coords0, predictions
