"""Drop-in CorrBlock for E-RAFT on MI355X.

Same constructor, call signature, attributes and output as the reference class
(AhmedHumais/E-RAFT model/corr.py:12-60):

    corr_fn = CorrBlock(fmap1, fmap2, num_levels=4, radius=4)   # eraft.py:108
    corr    = corr_fn(coords1)                                  # eraft.py:129
    vol     = CorrBlock.corr(fmap1, fmap2)                      # [B, H, W, 1, H, W]

Swapping it into the reference model is a one-line import change.
Every computation goes through libcorr_mi355x.so (gfx950 HIP kernels, C-ABI); there is no
CPU or eager fallback — CPU tensors raise.

Autograd (training, BASELINE config 4): gradients flow to fmap1 / fmap2 only (coords are
detached by the caller, eraft.py:128, and the reference never needs d/dcoords).  Instead of
materialising a dense pyramid gradient per lookup as torch autograd does, every lookup's
backward only STASHES its (coords, upstream gradient); the build's backward then runs
corr_backward once: all lookups' input-gradients into one gradient pyramid in one launch, the
avg-pool backward folded into level 0 in one pass, and the two MFMA GEMMs.
(ERAFT_AMD_FUSED_BWD=0: the per-lookup path — a kernel per lookup backward, then the fold.)
"""
from __future__ import annotations

import weakref

import torch

from . import _lib


def level_shapes(H: int, W: int, num_levels: int):
    """avg_pool2d(2, stride 2) floor halving (corr.py:25-27)."""
    return [(H >> l, W >> l) for l in range(num_levels)]


def _alloc_pyramid(B: int, H: int, W: int, num_levels: int, like: torch.Tensor, zero=False):
    """One allocation holding every level, viewed as the reference's [B*H*W, 1, H_l, W_l]."""
    BN = B * H * W
    shapes = level_shapes(H, W, num_levels)
    sizes = [BN * h * w for h, w in shapes]
    # keep every level 16-byte aligned (float4 paths)
    offs, tot = [], 0
    for s in sizes:
        offs.append(tot)
        tot += (s + 3) // 4 * 4
    fn = torch.zeros if zero else torch.empty
    buf = fn(tot, dtype=torch.float32, device=like.device)
    return [buf[o:o + s].view(BN, 1, h, w) for o, s, (h, w) in zip(offs, sizes, shapes)]


def _validate_fmaps(fmap1, fmap2, num_levels):
    for t, nm in ((fmap1, "fmap1"), (fmap2, "fmap2")):
        if not isinstance(t, torch.Tensor) or t.device.type != "cuda":
            raise RuntimeError(f"{nm} must be a tensor on an MI355X (HIP) device: eraft_amd has no "
                               "CPU fallback")
    if fmap1.dim() != 4 or fmap1.shape != fmap2.shape:
        raise ValueError(f"fmap1 / fmap2 must both be [B, D, H, W] (got {tuple(fmap1.shape)}, "
                         f"{tuple(fmap2.shape)})")
    if not (1 <= num_levels <= _lib.MAX_LEVELS):
        raise ValueError(f"num_levels must be in [1, {_lib.MAX_LEVELS}]")
    _, _, H, W = fmap1.shape
    if (H >> (num_levels - 1)) < 1 or (W >> (num_levels - 1)) < 1:
        # the reference raises inside avg_pool2d (corr.py:26)
        raise RuntimeError(f"{H}x{W} feature maps are too small for {num_levels} pyramid levels")


_WEIGHT_PACKS = {}  # id(weight) -> (weakref to the weight, (data_ptr, _version), pack)


def _weight_pack(weight):
    """convc1.weight's packed split for lookup_conv, cached per weight tensor in a module-level
    map keyed by the tensor's id and held by a weak reference (nothing is attached to the
    Parameter, so pickling or torch.save of the model is unaffected, and the entry goes when the
    tensor does), together with the (data_ptr, _version) it was made from: a new tensor
    (another model, a reloaded checkpoint) never sees another tensor's pack, and an in-place
    update (optimizer step, load_state_dict's copy_) bumps _version and re-packs.  (A
    WeakKeyDictionary cannot hold tensors: its key comparison calls Tensor.__eq__.)"""
    key = (weight.data_ptr(), weight._version)
    wid = id(weight)
    ent = _WEIGHT_PACKS.get(wid)
    if ent is None or ent[0]() is not weight or ent[1] != key:
        ref = weakref.ref(weight, lambda _r, wid=wid: _WEIGHT_PACKS.pop(wid, None))
        ent = (ref, key, _lib.lookup_conv_weights(weight))
        _WEIGHT_PACKS[wid] = ent
    return ent[2]


class _State:
    """Per-block state shared by the build and lookup autograd nodes."""

    __slots__ = ("levels", "grad_levels", "H", "W", "radius", "stash", "trains")

    def __init__(self, H, W, radius):
        self.trains = False      # the build is in the autograd graph (gradients reach the fmaps)
        self.levels = None
        self.grad_levels = None  # per-lookup path: the accumulated gradient pyramid
        self.stash = []          # fused path: (coords, grad_out) of every lookup backward
        self.H, self.W, self.radius = H, W, radius


class _BuildFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fmap1, fmap2, num_levels, state):
        B, _, H, W = fmap1.shape
        levels = _alloc_pyramid(B, H, W, num_levels, fmap1)
        _lib.build(fmap1, fmap2, levels)
        # the lookups read state.levels, not these outputs: no zero-filled level gradients
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(fmap1, fmap2)
        ctx.state = state
        # autograd anchor: every lookup depends on it; its value is never read (no fill kernel)
        token = fmap1.new_empty(())
        return (*levels, token)

    @staticmethod
    def backward(ctx, *grads):
        fmap1, fmap2 = ctx.saved_tensors
        st = ctx.state
        direct = grads[:-1]  # grads[-1] (the token's) carries no value
        stash, st.stash = st.stash, []
        if st.grad_levels is None and not any(g is not None for g in direct):
            if not stash:
                return None, None, None, None
            # fused: every lookup's backward + the fold + the GEMMs in corr_backward
            B, _, H, W = fmap1.shape
            gl = _alloc_pyramid(B, H, W, len(direct), fmap1)  # scratch, overwritten
            df1, df2 = _lib.backward([c for c, _ in stash], [g for _, g in stash], st.radius, gl, fmap1, fmap2)
            return df1, df2, None, None
        gl = st.grad_levels
        if stash:  # direct gradients reached corr_pyramid: run the stashed lookups' backward too
            if gl is None:
                B, _, H, W = fmap1.shape
                gl = _alloc_pyramid(B, H, W, len(direct), fmap1, zero=True)
            for c, g in stash:
                _lib.lookup_bwd(c, g, st.radius, gl)
        if any(g is not None for g in direct):
            # gradients that reached corr_pyramid outside the lookups
            if gl is None:
                B, _, H, W = fmap1.shape
                gl = _alloc_pyramid(B, H, W, len(direct), fmap1, zero=True)
            for acc, g in zip(gl, direct):
                if g is not None:
                    acc.add_(g)
        st.grad_levels = None
        if gl is None:
            return None, None, None, None
        _lib.pool_bwd(gl, st.H, st.W)
        df1, df2 = _lib.build_bwd(gl[0], fmap1, fmap2)
        return df1, df2, None, None


class _LookupFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, coords, token, radius, state):
        levels = state.levels
        B, _, H, W = coords.shape
        K = (2 * radius + 1) ** 2
        out = torch.empty((B, len(levels) * K, H, W), dtype=torch.float32, device=coords.device)
        _lib.lookup(levels, coords, radius, out)
        ctx.save_for_backward(coords)
        ctx.radius = radius
        ctx.state = state
        return out

    @staticmethod
    def stash_backward(st, coords, grad_out, radius):
        if _lib.fused_backward():
            st.stash.append((coords, grad_out.contiguous()))  # run by the build's backward
        else:
            if st.grad_levels is None:
                B, _, H, W = coords.shape
                st.grad_levels = _alloc_pyramid(B, H, W, len(st.levels), coords, zero=True)
            _lib.lookup_bwd(coords, grad_out.contiguous(), radius, st.grad_levels)

    @staticmethod
    def backward(ctx, grad_out):
        (coords,) = ctx.saved_tensors
        _LookupFn.stash_backward(ctx.state, coords, grad_out, ctx.radius)
        # No gradient for the token: the engine still runs the build's backward, after every
        # lookup backward (it depends on all of them), and nothing is filled or summed for it.
        return None, None, None, None


class _LookupConvFn(torch.autograd.Function):
    """relu(convc1(lookup(coords))) (update.py:68,75) as one fused kernel in the forward; the
    324-channel lookup output is never written.  Backward (training, config 4): one
    corr_lookup_conv_bwd call — ReLU's threshold backward, d bias, dW = g' lk^T with the lookup
    recomputed on chip (never stored), and the lookup's own gradient W^T g', which goes into the
    build's stash exactly as a plain lookup's backward does, so corr_backward folds it with every
    other lookup."""

    @staticmethod
    def forward(ctx, coords, token, weight, bias, relu, radius, state):
        levels = state.levels
        B, _, H, W = coords.shape
        out = torch.empty((B, weight.shape[0], H, W), dtype=torch.float32, device=coords.device)
        _lib.lookup_conv(levels, coords, radius, _weight_pack(weight), bias.detach().contiguous().float(), out, relu)
        ctx.save_for_backward(coords, weight, out)
        ctx.relu, ctx.radius, ctx.state = relu, radius, state
        return out

    @staticmethod
    def backward(ctx, grad_out):
        coords, weight, out = ctx.saved_tensors
        st = ctx.state
        g = grad_out.contiguous().float()
        B, O, H, W = g.shape
        C = len(st.levels) * (2 * ctx.radius + 1) ** 2
        dev = coords.device
        dW = torch.empty((O, C), dtype=torch.float32, device=dev) if ctx.needs_input_grad[2] else None
        dbias = torch.empty((O,), dtype=torch.float32, device=dev) if ctx.needs_input_grad[3] else None
        dlk = torch.empty((B, C, H, W), dtype=torch.float32, device=dev) if st.trains else None
        _lib.lookup_conv_bwd(st.levels, coords, ctx.radius, _weight_pack(weight), out, ctx.relu, g, dW, dbias, dlk)
        if dlk is not None:  # the lookup's upstream gradient, for the build's backward
            _LookupFn.stash_backward(st, coords, dlk, ctx.radius)
        if dW is not None:
            dW = dW.view_as(weight).to(weight.dtype)
        return None, None, dW, dbias, None, None, None


class CorrBlock:
    """MI355X-native replacement for model/corr.py:12 ``CorrBlock``."""

    def __init__(self, fmap1, fmap2, num_levels=4, radius=4):
        self.num_levels = num_levels
        self.radius = radius
        if not (0 <= radius <= _lib.MAX_RADIUS):
            raise ValueError(f"radius must be in [0, {_lib.MAX_RADIUS}]")
        _validate_fmaps(fmap1, fmap2, num_levels)
        fmap1 = fmap1.contiguous()
        fmap2 = fmap2.contiguous()
        _, _, H, W = fmap1.shape
        self._state = _State(H, W, radius)
        self._token = None
        if torch.is_grad_enabled() and (fmap1.requires_grad or fmap2.requires_grad):
            outs = _BuildFn.apply(fmap1, fmap2, num_levels, self._state)
            self.corr_pyramid = list(outs[:-1])
            self._token = outs[-1]
            self._state.trains = True
        else:
            B = fmap1.shape[0]
            self.corr_pyramid = _alloc_pyramid(B, H, W, num_levels, fmap1)
            _lib.build(fmap1.detach(), fmap2.detach(), self.corr_pyramid)
        self._state.levels = [p.detach() for p in self.corr_pyramid]

    def _check_coords(self, coords):
        if coords.dim() != 4 or coords.shape[1] != 2:
            raise ValueError(f"coords must be [B, 2, H, W] (got {tuple(coords.shape)})")
        B, _, H, W = coords.shape
        if B * H * W != self.corr_pyramid[0].shape[0] or (H, W) != (self._state.H, self._state.W):
            raise ValueError("coords do not match the feature maps this block was built from")

    def __call__(self, coords):
        self._check_coords(coords)
        B, _, H, W = coords.shape
        # the reference accepts any strides (permute at corr.py:31); fp32 as in eraft.py:128
        coords = coords.detach().contiguous()
        if self._token is not None and torch.is_grad_enabled():
            return _LookupFn.apply(coords, self._token, self.radius, self._state)
        K = (2 * self.radius + 1) ** 2
        out = torch.empty((B, self.num_levels * K, H, W), dtype=torch.float32, device=coords.device)
        _lib.lookup(self._state.levels, coords, self.radius, out)
        return out

    def lookup_conv(self, coords, weight, bias, relu=True):
        """Lookup fused with the motion encoder's first layer, relu(convc1(self(coords)))
        (update.py:68,75), without materialising the lookup output.  weight: convc1.weight
        [256, L*K, 1, 1]; bias [256].  Under autograd (training) gradients reach the weight,
        the bias and, through the build's backward, both feature maps (_LookupConvFn)."""
        self._check_coords(coords)
        B, _, H, W = coords.shape
        K = (2 * self.radius + 1) ** 2
        C = self.num_levels * K
        if tuple(weight.shape) not in ((256, C, 1, 1), (256, C)) or tuple(bias.shape) != (256,):
            raise ValueError(f"lookup_conv needs weight [256, {C}, 1, 1] and bias [256] "
                             f"(got {tuple(weight.shape)}, {tuple(bias.shape)})")
        coords = coords.detach().contiguous()
        if torch.is_grad_enabled() and (self._token is not None or weight.requires_grad or bias.requires_grad):
            token = self._token
            if token is None:  # the pyramid is constant; gradients reach only the weight and bias
                token = coords.new_empty(())
            return _LookupConvFn.apply(coords, token, weight, bias, relu, self.radius, self._state)
        cached = _weight_pack(weight)  # split once per weight version (every GRU iteration reuses it)
        out = torch.empty((B, weight.shape[0], H, W), dtype=torch.float32, device=coords.device)
        _lib.lookup_conv(self._state.levels, coords, self.radius, cached,
                         bias.detach().contiguous().float(), out, relu)
        return out

    @staticmethod
    def corr(fmap1, fmap2):
        """model/corr.py:52-60: all-pairs volume [B, H, W, 1, H, W] scaled by 1/sqrt(D)."""
        _validate_fmaps(fmap1, fmap2, 1)
        B, _, H, W = fmap1.shape
        (lvl,) = _alloc_pyramid(B, H, W, 1, fmap1)
        _lib.build(fmap1.detach().contiguous(), fmap2.detach().contiguous(), [lvl])
        return lvl.view(B, H, W, 1, H, W)
