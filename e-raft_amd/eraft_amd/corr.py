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


TILE_W = _lib.TILE_W  # cells per tile row (include/corr_mi355x.h): tiles of 4 rows x TILE_W cells
map_floats = _lib.map_floats  # floats of one query's tiled level map


def _alloc_pyramid(B: int, H: int, W: int, num_levels: int, like: torch.Tensor, zero=False, NQ=None):
    """The build's output / the lookups' input: one allocation holding every level in the
    library's tiled layout, level l viewed [B*NQ, map_floats(H_l, W_l)] (NQ = H*W queries per
    batch item by default; a row slab's otherwise).  Materialise the reference's
    [B*N, 1, H_l, W_l] view with _lib.pyramid_export (CorrBlock.corr_pyramid does)."""
    BN = B * (H * W if NQ is None else NQ)
    sizes = [BN * map_floats(h, w) for h, w in level_shapes(H, W, num_levels)]
    offs, tot = [], 0
    for s in sizes:  # multiples of 16 floats: every level 64-B aligned
        offs.append(tot)
        tot += s
    fn = torch.zeros if zero else torch.empty
    buf = fn(tot, dtype=torch.float32, device=like.device)
    return [buf[o:o + s].view(BN, s // BN) for o, s in zip(offs, sizes)]


def _alloc_grad_pyramid(B: int, H: int, W: int, num_levels: int, like: torch.Tensor, zero=False, NQ=None):
    """A gradient pyramid: the reference's row-major layout, level l [B*NQ, 1, H_l, W_l] in one
    allocation (corr_lookup_bwd / corr_pool_bwd / corr_backward's scratch; level 0 ends as dC)."""
    BN = B * (H * W if NQ is None else NQ)
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

    __slots__ = ("levels", "grad_levels", "H", "W", "radius", "stash", "trains", "direct")

    def __init__(self, H, W, radius):
        self.trains = False      # the build is in the autograd graph (gradients reach the fmaps)
        self.levels = None       # the tiled pyramid (_alloc_pyramid)
        self.grad_levels = None  # per-lookup path: the accumulated gradient pyramid
        self.stash = []          # fused path: (coords, grad_out) of every lookup backward
        self.direct = None       # gradients that reached corr_pyramid's exported view, per level
        self.H, self.W, self.radius = H, W, radius


class _BuildFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fmap1, fmap2, num_levels, state):
        B, _, H, W = fmap1.shape
        state.levels = _alloc_pyramid(B, H, W, num_levels, fmap1)
        _lib.build(fmap1, fmap2, state.levels)
        ctx.set_materialize_grads(False)
        ctx.save_for_backward(fmap1, fmap2)
        ctx.state = state
        ctx.num_levels = num_levels
        # autograd anchor: every lookup (and corr_pyramid's exported view) depends on it; its value
        # is never read (no fill kernel)
        return fmap1.new_empty(())

    @staticmethod
    def backward(ctx, _token_grad):
        fmap1, fmap2 = ctx.saved_tensors
        st = ctx.state
        L = ctx.num_levels
        direct = st.direct if st.direct is not None else [None] * L
        st.direct = None
        stash, st.stash = st.stash, []
        if st.grad_levels is None and not any(g is not None for g in direct):
            if not stash:
                return None, None, None, None
            # fused: every lookup's backward + the fold + the GEMMs in corr_backward
            B, _, H, W = fmap1.shape
            gl = _alloc_grad_pyramid(B, H, W, L, fmap1)  # scratch, overwritten
            df1, df2 = _lib.backward([c for c, _ in stash], [g for _, g in stash], st.radius, gl, fmap1, fmap2)
            return df1, df2, None, None
        gl = st.grad_levels
        if stash:  # direct gradients reached corr_pyramid: run the stashed lookups' backward too
            if gl is None:
                B, _, H, W = fmap1.shape
                gl = _alloc_grad_pyramid(B, H, W, L, fmap1, zero=True)
            for c, g in stash:
                _lib.lookup_bwd(c, g, st.radius, gl)
        if any(g is not None for g in direct):
            # gradients that reached corr_pyramid outside the lookups
            if gl is None:
                B, _, H, W = fmap1.shape
                gl = _alloc_grad_pyramid(B, H, W, L, fmap1, zero=True)
            for acc, g in zip(gl, direct):
                if g is not None:
                    acc.add_(g)
        st.grad_levels = None
        if gl is None:
            return None, None, None, None
        _lib.pool_bwd(gl, st.H, st.W)
        df1, df2 = _lib.build_bwd(gl[0], fmap1, fmap2)
        return df1, df2, None, None


class _PyramidViewFn(torch.autograd.Function):
    """corr_pyramid under autograd: the tiled pyramid exported to the reference's
    [B*N, 1, H_l, W_l] levels (corr.py:16,24,27,36); gradients that reach them are kept for the
    build's backward, which adds them to the lookups' gradient pyramid (as autograd sums a
    level's gradients in the reference)."""

    @staticmethod
    def forward(ctx, token, state):
        ctx.state = state
        ctx.set_materialize_grads(False)
        return tuple(_lib.pyramid_export(state.levels, state.H, state.W))

    @staticmethod
    def backward(ctx, *grads):
        st = ctx.state
        if st.direct is None:
            st.direct = [None] * len(grads)
        for l, g in enumerate(grads):
            if g is not None:
                st.direct[l] = g.contiguous() if st.direct[l] is None else st.direct[l] + g
        # no gradient for the token: the engine still runs the build's backward after this one
        return None, None


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
                st.grad_levels = _alloc_grad_pyramid(B, H, W, len(st.levels), coords, zero=True)
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
        # the levels this output was made from (an assignment to corr_pyramid installs new ones),
        # and whether the build is upstream (a constant pyramid's token carries no gradient)
        ctx.levels, ctx.trains = levels, ctx.needs_input_grad[1]
        return out

    @staticmethod
    def backward(ctx, grad_out):
        coords, weight, out = ctx.saved_tensors
        st = ctx.state
        g = grad_out.contiguous().float()
        if g.data_ptr() % 16:  # the kernel's 16-B loads need an aligned base (a view with an odd offset)
            g = g.clone()
        B, O, H, W = g.shape
        C = len(ctx.levels) * (2 * ctx.radius + 1) ** 2
        dev = coords.device
        dW = torch.empty((O, C), dtype=torch.float32, device=dev) if ctx.needs_input_grad[2] else None
        dbias = torch.empty((O,), dtype=torch.float32, device=dev) if ctx.needs_input_grad[3] else None
        dlk = torch.empty((B, C, H, W), dtype=torch.float32, device=dev) if ctx.trains else None
        _lib.lookup_conv_bwd(ctx.levels, coords, ctx.radius, _weight_pack(weight), out, ctx.relu, g, dW, dbias, dlk)
        if dlk is not None:  # the lookup's upstream gradient, for the build's backward
            _LookupFn.stash_backward(st, coords, dlk, ctx.radius)
        if dW is not None:
            dW = dW.view_as(weight).to(weight.dtype)
        return None, None, dW, dbias, None, None, None


class _CorrFn(torch.autograd.Function):
    """CorrBlock.corr under autograd.  The reference's static corr (corr.py:52-60) is a torch
    matmul scaled by 1/sqrt(D), so gradients reach both feature maps; here the forward is the
    one-level build exported to [B, H, W, 1, H, W] and the backward the library's GEMMs on dC
    (corr_build_bwd_ex: dF1 = F2 dC^T / sqrt(D), dF2 = F1 dC / sqrt(D))."""

    @staticmethod
    def forward(ctx, fmap1, fmap2):
        B, _, H, W = fmap1.shape
        lvl = _alloc_pyramid(B, H, W, 1, fmap1)
        _lib.build(fmap1, fmap2, lvl)
        ctx.save_for_backward(fmap1, fmap2)
        ctx.set_materialize_grads(False)
        return _lib.pyramid_export(lvl, H, W)[0].view(B, H, W, 1, H, W)

    @staticmethod
    def backward(ctx, grad):
        if grad is None:
            return None, None
        fmap1, fmap2 = ctx.saved_tensors
        B, _, H, W = fmap1.shape
        df1, df2 = _lib.build_bwd(grad.contiguous().view(B * H * W, H * W), fmap1, fmap2)
        return (df1 if ctx.needs_input_grad[0] else None, df2 if ctx.needs_input_grad[1] else None)


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
        self._view = None  # corr_pyramid's exported levels, made on first access ...
        self._view_grad = False  # ... with (True) or without autograd
        self._assigned = False  # corr_pyramid was assigned: later lookups carry no gradient
        if torch.is_grad_enabled() and (fmap1.requires_grad or fmap2.requires_grad):
            self._token = _BuildFn.apply(fmap1, fmap2, num_levels, self._state)
            self._state.trains = True
        else:
            B = fmap1.shape[0]
            self._state.levels = _alloc_pyramid(B, H, W, num_levels, fmap1)
            _lib.build(fmap1.detach(), fmap2.detach(), self._state.levels)

    @property
    def corr_pyramid(self):
        """The pyramid as the reference holds it (corr.py:16,24,27,36): a list of num_levels
        tensors [B*H*W, 1, H_l, W_l].  The library keeps it tiled (include/corr_mi355x.h), so the
        view is materialised (corr_pyramid_export) on first access; with the build in the autograd
        graph, gradients that reach it flow to both fmaps as in the reference.  Assigning a list
        of such tensors installs them (corr_pyramid_import) for the following lookups."""
        st = self._state
        grad = self._token is not None and not self._assigned and torch.is_grad_enabled()
        if self._view is None or (grad and not self._view_grad):
            # (re-)export: a view first made under no_grad (or by inspection only) must not stand
            # in for the differentiable one a later grad-enabled read needs
            if grad:
                self._view = list(_PyramidViewFn.apply(self._token, st))
            else:
                self._view = _lib.pyramid_export(st.levels, st.H, st.W)
            self._view_grad = grad
        return self._view

    @corr_pyramid.setter
    def corr_pyramid(self, levels):
        """Install a pyramid for the following lookups (corr_pyramid_import).  As in the
        reference, those lookups then read the assigned tensors, not the build: they send no
        gradient to fmap1 / fmap2.  Gradients INTO assigned tensors that require grad are not
        supported (the tiled copy is not in their graph): that raises instead of losing them."""
        st = self._state
        if len(levels) != len(st.levels):
            raise ValueError(f"corr_pyramid needs {len(st.levels)} levels (got {len(levels)})")
        if torch.is_grad_enabled() and any(getattr(l, "requires_grad", False) for l in levels):
            raise NotImplementedError("assigning corr_pyramid levels that require grad: gradients cannot "
                                      "reach them through the tiled copy; assign detached levels")
        B = st.levels[0].shape[0] // (st.H * st.W)
        # a fresh buffer: a lookup_conv backward still pending reads the levels it was made from
        fresh = _alloc_pyramid(B, st.H, st.W, len(st.levels), st.levels[0])
        _lib.pyramid_import([l.detach() for l in levels], fresh, st.H, st.W)
        st.levels = fresh
        self._assigned = True
        self._view = None
        self._view_grad = False

    def _check_coords(self, coords):
        if coords.dim() != 4 or coords.shape[1] != 2:
            raise ValueError(f"coords must be [B, 2, H, W] (got {tuple(coords.shape)})")
        B, _, H, W = coords.shape
        if B * H * W != self._state.levels[0].shape[0] or (H, W) != (self._state.H, self._state.W):
            raise ValueError("coords do not match the feature maps this block was built from")

    def __call__(self, coords):
        self._check_coords(coords)
        B, _, H, W = coords.shape
        # the reference accepts any strides (permute at corr.py:31); fp32 as in eraft.py:128
        coords = coords.detach().contiguous()
        if self._token is not None and not self._assigned and torch.is_grad_enabled():
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
        live = self._token is not None and not self._assigned
        if torch.is_grad_enabled() and (live or weight.requires_grad or bias.requires_grad):
            token = self._token if live else None
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
        """model/corr.py:52-60: all-pairs volume [B, H, W, 1, H, W] scaled by 1/sqrt(D);
        differentiable w.r.t. both feature maps as the reference's matmul is (_CorrFn)."""
        _validate_fmaps(fmap1, fmap2, 1)
        f1, f2 = fmap1.contiguous(), fmap2.contiguous()
        if torch.is_grad_enabled() and (f1.requires_grad or f2.requires_grad):
            return _CorrFn.apply(f1, f2)
        B, _, H, W = fmap1.shape
        lvl = _alloc_pyramid(B, H, W, 1, fmap1)
        _lib.build(f1.detach(), f2.detach(), lvl)
        return _lib.pyramid_export(lvl, H, W)[0].view(B, H, W, 1, H, W)
