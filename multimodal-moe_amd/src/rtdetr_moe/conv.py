"""Convolutions of the RT-DETR body on libmoe_hip's implicit-GEMM kernels
(csrc/conv.hip: rtdetr_conv_fwd / rtdetr_conv_dgrad / rtdetr_conv_wgrad).

``conv2d(x, weight, stride, padding)`` takes the HIP kernels for the
convolutions they cover -- padding (k - 1) / 2, 1x1 or 3x3, stride 1 (or 2
for 3x3: the ResNet-D stage-entry and HybridEncoder downsampling layers, whose
MIOpen weight-gradient solvers are not graph-replay safe: DESIGN.md 5), no groups,
channel counts that are multiples of 64, bf16 channels_last activations and
weights on the GPU (the HybridEncoder's RepVGG / CSP layers and the ResNet
bottleneck convolutions of 64 .. 2048 channels) -- and
F.conv2d (MIOpen) for the rest.  Forward: one implicit-GEMM launch (no im2col
buffer).  Backward: the data gradient is the same kernel over dY with the
weight flipped and transposed (written to a workspace for large problems,
read in place for small ones); the weight gradient is split over pixel slices
with fp32 partials summed in a fixed order (deterministic).
MOE_HIP_CONV=0 keeps every convolution on MIOpen (A/B switch).
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F

_ENABLED = [os.environ.get("MOE_HIP_CONV", "1") != "0"]
_ZERO = {}


def _zero(dev):
    z = _ZERO.get(dev)
    if z is None:
        z = _ZERO[dev] = torch.zeros(256, dtype=torch.bfloat16, device=dev)
    return z


def _nhwc(t):
    return t if t.is_contiguous(memory_format=torch.channels_last) else t.contiguous(memory_format=torch.channels_last)


def hip_conv_ok(x, w, stride=1, padding=None, dilation=1, groups=1) -> bool:
    """Whether conv2d(x, w) runs on the HIP implicit-GEMM kernels."""
    if not (x.dim() == 4 and x.shape[0] > 0):
        return False
    return hip_conv_ok_for(x.is_cuda, x.dtype, x.shape[1], w, stride, padding, dilation, groups)


def hip_conv_ok_for(is_cuda, dtype, cin, w, stride=1, padding=None, dilation=1, groups=1, w_dtype=None) -> bool:
    """hip_conv_ok for an input of that device kind, dtype and channel count
    (a consumer's check before its input exists); w_dtype overrides w.dtype."""
    if not (_ENABLED[0] and is_cuda and w.dim() == 4):
        return False
    N, C, kh, kw = w.shape
    ks = kh
    st = stride if isinstance(stride, int) else (stride[0] if stride[0] == stride[1] else -1)
    pd = padding if isinstance(padding, int) else (padding[0] if padding[0] == padding[1] else -1)
    dl = dilation if isinstance(dilation, int) else (dilation[0] if dilation[0] == dilation[1] else -1)
    return (dtype == torch.bfloat16 and (w_dtype or w.dtype) == torch.bfloat16 and kh == kw and ks in (1, 3)
            and (st == 1 or (st == 2 and ks == 3)) and pd == (ks - 1) // 2 and dl == 1 and groups == 1
            and cin == C and C % 64 == 0 and N % 64 == 0)


def _stride(stride) -> int:
    return stride if isinstance(stride, int) else stride[0]


def _out(n, ks, st):
    return (n + 2 * ((ks - 1) // 2) - ks) // st + 1


def _fwd(x, w, bias=None, resid=None, relu=False, st=1):
    from ..moe import _lib as L

    B, C, H, W = x.shape
    N, _, ks, _ = w.shape
    y = torch.empty((B, N, _out(H, ks, st), _out(W, ks, st)), dtype=torch.bfloat16, device=x.device,
                    memory_format=torch.channels_last)
    L._check(L.lib().rtdetr_conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), _zero(x.device).data_ptr(),
                                     B, H, W, C, N, ks, st, None if bias is None else bias.data_ptr(),
                                     None if resid is None else resid.data_ptr(), int(relu), L._stream()),
             "rtdetr_conv_fwd")
    return y


def conv_act_eval(x, w, bias, act, resid=None, st=1, out=None, out_row=0):
    """Inference only (no autograd): act(conv(x, w) + bias) [+ resid after the
    activation, bf16 SiLU-then-add] in one rtdetr_conv_fwd_act launch
    (act 0 none, 1 ReLU, 2 SiLU): the folded BatchNorm / RepVgg layers of
    evalfold.py.  out ([B, S, N] bf16, contiguous): write image b's Ho Wo
    output rows at out[b, out_row:out_row + Ho Wo] instead (returns out)."""
    from ..moe import _lib as L

    x = _nhwc(x)
    if x.data_ptr() % 16:
        x = x.clone(memory_format=torch.channels_last)
    if resid is not None:
        resid = _nhwc(resid)
        if resid.data_ptr() % 16:
            resid = resid.clone(memory_format=torch.channels_last)
    B, C, H, W = x.shape
    N, _, ks, _ = w.shape
    Ho, Wo = _out(H, ks, st), _out(W, ks, st)
    if out is not None:
        if resid is not None or not (out.dim() == 3 and out.shape[0] == B and out.shape[2] == N
                                     and out.dtype == torch.bfloat16 and out.is_contiguous()
                                     and 0 <= out_row and out_row + Ho * Wo <= out.shape[1]):
            raise ValueError("conv_act_eval: out must be a contiguous bf16 [B, S, N] holding the rows")
        y, rows = out, out.shape[1]
    else:
        y = torch.empty((B, N, Ho, Wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        rows = 0
    if resid is not None and resid.shape != y.shape:
        raise ValueError(f"conv_act_eval: resid {tuple(resid.shape)} vs output {tuple(y.shape)}")
    L._check(L.lib().rtdetr_conv_fwd_act(x.data_ptr(), w.data_ptr(), y.data_ptr(), _zero(x.device).data_ptr(),
                                         B, H, W, C, N, ks, st, bias.data_ptr(),
                                         None if resid is None else resid.data_ptr(), int(act),
                                         1 if resid is not None else 0, rows, int(out_row) if rows else 0,
                                         L._stream()),
             "rtdetr_conv_fwd_act")
    return y


def _stats_blocks(x, w, st=1):
    """Row blocks of rtdetr_conv_fwd_stats' BatchNorm partials for y =
    conv(x, w) (0: too many for the BatchNorm finalize -- take bn_stats)."""
    from ..moe import _lib as L

    B, C, H, W = x.shape
    N, _, ks, _ = w.shape
    rows = L.lib().rtdetr_conv_fwd_stats_rows(B, H, W, C, N, ks, st)
    if rows <= 0:
        return 0
    nblk = -(-(B * _out(H, ks, st) * _out(W, ks, st)) // rows)
    return nblk if nblk <= 2048 else 0


def _fwd_stats(x, w, part, st=1):
    """conv(x, w) that also writes its output's BatchNorm partials into part
    (fp32 [nblk, 2, N], rtdetr_conv_fwd_stats)."""
    from ..moe import _lib as L

    B, C, H, W = x.shape
    N, _, ks, _ = w.shape
    y = torch.empty((B, N, _out(H, ks, st), _out(W, ks, st)), dtype=torch.bfloat16, device=x.device,
                    memory_format=torch.channels_last)
    L._check(L.lib().rtdetr_conv_fwd_stats(x.data_ptr(), w.data_ptr(), y.data_ptr(), _zero(x.device).data_ptr(),
                                           B, H, W, C, N, ks, st, part.data_ptr(), L._stream()),
             "rtdetr_conv_fwd_stats")
    return y


# Batched weight flips (GraphedStep): the data gradients of the flipping
# shapes read W' from persistent per-weight buffers, all written by ONE
# rtdetr_conv_weight_flip_multi launch right before the backward (49 flip
# launches per C2 step before).  Entries are keyed by (weight address, shape):
# the flip runs after the forward, so whatever bf16 weight lives at a key's
# address then is the one its data gradient reads (captured graphs keep every
# address); an unregistered weight takes the per-call flip and registers.
_FLIP_ON = [False]     # inside batched_flips(): register, and use W' buffers flipped at entry
_FLIP_VALID = [False]  # the W' buffers hold this backward's weights
_FLIP_REG: dict = {}
_FLIP_TABLE = [None, 0, 0, 0]  # (device table, n, total blocks, registry size it was built for)


def _flip_entry(w, nb):
    key = (w.data_ptr(), tuple(w.shape))
    e = _FLIP_REG.get(key)
    if e is None and _FLIP_ON[0]:
        e = _FLIP_REG[key] = torch.empty(nb // 2, dtype=torch.bfloat16, device=w.device)
    return e


def _flip_all(dev):
    import numpy as np

    from ..moe import _lib as L

    if not _FLIP_REG:
        return
    if _FLIP_TABLE[3] != len(_FLIP_REG):
        dt = np.dtype([("w", np.uint64), ("wt", np.uint64), ("N", np.int32), ("C", np.int32), ("KS", np.int32),
                       ("block0", np.int32)])
        rec = np.zeros(len(_FLIP_REG), dtype=dt)
        b0 = 0
        for i, ((ptr, shape), buf) in enumerate(_FLIP_REG.items()):
            N, C, ks = shape[0], shape[1], shape[2]
            rec[i] = (ptr, buf.data_ptr(), N, C, ks, b0)
            b0 += (C // 64) * (N // 64) * ks * ks
        _FLIP_TABLE[:] = [torch.from_numpy(rec.view(np.uint8).copy()).to(dev), len(_FLIP_REG), b0, len(_FLIP_REG)]
    t, n, blocks, _ = _FLIP_TABLE
    L._check(L.lib().rtdetr_conv_weight_flip_multi(t.data_ptr(), n, blocks, L._stream()),
             "rtdetr_conv_weight_flip_multi")


class batched_flips:
    """Context for a backward (GraphedStep): every registered weight flipped in
    one launch at entry, the data gradients then read the flipped buffers."""

    def __init__(self, device):
        self.device = device

    def __enter__(self):
        if _BATCHED_FLIPS:
            _FLIP_ON[0] = True
            if _FLIP_TABLE[3] != len(_FLIP_REG) and torch.cuda.is_current_stream_capturing():
                return self  # (a table rebuild copies from the host: not inside a capture) register only
            _flip_all(self.device)
            _FLIP_VALID[0] = True
        return self

    def __exit__(self, *exc):
        _FLIP_ON[0] = False
        _FLIP_VALID[0] = False
        return False


# MOE_BATCHED_FLIPS=0: every flipping data gradient writes its own W' (A/B switch)
_BATCHED_FLIPS = os.environ.get("MOE_BATCHED_FLIPS", "1") != "0"


def _bwd(x, w, g, need_x, need_w, mask_input, add=None, st=1):
    """(dx, dw) of y = conv(x, w) for the output gradient g; dx += add (x's
    other consumer's gradient, when given), then dx is zeroed where x <= 0 when
    mask_input (the ReLU backward of the activation x, fused)."""
    from ..moe import _lib as L

    B, C, H, W = x.shape
    N, _, ks, _ = w.shape
    g = _nhwc(g.to(torch.bfloat16))
    z = _zero(x.device).data_ptr()
    s = L._stream()
    gx = gw = None
    if need_x:
        gx = torch.empty((B, C, H, W), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        nb = L.lib().rtdetr_conv_dgrad_workspace(B, H, W, C, N, ks)
        pre = None
        if nb > 0 and _FLIP_ON[0] and w.dtype == torch.bfloat16:
            key = (w.data_ptr(), tuple(w.shape))
            if _FLIP_VALID[0] and key in _FLIP_REG:
                pre = _FLIP_REG[key]  # flipped at the backward's entry
            work = _flip_entry(w, nb)  # (registers it: flipped in place by this call, batched from then on)
        else:
            work = torch.empty(nb // 2, dtype=torch.bfloat16, device=x.device) if nb > 0 else None
        addp = None if add is None else _nhwc(add).data_ptr()
        maskp = x.data_ptr() if mask_input else None
        if pre is not None:
            L._check(L.lib().rtdetr_conv_dgrad_preflipped(g.data_ptr(), w.data_ptr(), pre.data_ptr(), gx.data_ptr(), z,
                                                          B, H, W, C, N, ks, st, addp, maskp, s),
                     "rtdetr_conv_dgrad_preflipped")
        else:
            L._check(L.lib().rtdetr_conv_dgrad(g.data_ptr(), w.data_ptr(), None if work is None else work.data_ptr(),
                                               gx.data_ptr(), z, B, H, W, C, N, ks, st, addp, maskp, s),
                     "rtdetr_conv_dgrad")
    if need_w:
        ns = L.lib().rtdetr_conv_wgrad_splits(B, _out(H, ks, st), _out(W, ks, st), C, N, ks)
        part = torch.empty(ns * N * C * ks * ks, dtype=torch.float32, device=x.device)
        gw = torch.empty_like(w, memory_format=torch.channels_last)
        pend = _WG_PENDING[0]
        if pend is not None:  # the slice sum runs in the scope's batched reduction (deferred_wgrads)
            L._check(L.lib().rtdetr_conv_wgrad_part(g.data_ptr(), x.data_ptr(), part.data_ptr(), ns, z, B, H, W,
                                                    C, N, ks, st, s), "rtdetr_conv_wgrad_part")
            pend.append((part, ns, N * C * ks * ks, gw))
        else:
            L._check(L.lib().rtdetr_conv_wgrad(g.data_ptr(), x.data_ptr(), part.data_ptr(), ns, gw.data_ptr(), 1,
                                               z, B, H, W, C, N, ks, st, s), "rtdetr_conv_wgrad")
    return gx, gw


# MOE_CONV_WG_DEFER=0: one slice-sum launch per convolution weight gradient
# instead of the batched reduction at the end of the backward (A/B switch)
_WG_DEFER_ON = os.environ.get("MOE_CONV_WG_DEFER", "1") != "0"
# (part, nsplit, numel, gw) of the weight gradients whose slice sums are
# pending, while a deferred_wgrads scope is open; None otherwise
_WG_PENDING: list = [None]
_WG_BATCH = 48  # descriptors per rtdetr_conv_wgrad_reduce_batch launch


class deferred_wgrads:
    """Scope of one backward pass (GraphedStep._grads): every HIP convolution's
    weight gradient writes only its fp32 pixel slices (rtdetr_conv_wgrad_part)
    and the slice sums of all of them run as one or two
    rtdetr_conv_wgrad_reduce_batch launches -- bitwise the per-convolution
    reductions -- when the scope closes, or earlier at flush_wgrads() (a
    consumer of the gradients inside the backward: backbone._FoldAll).  Until
    then the returned gradient tensors hold no values, so the scope is only
    opened where nothing else reads them first: bf16 weights (no autocast
    cast node between the parameter and the convolution), torch.autograd.grad
    (no AccumulateGrad).  The ~94 small reduction launches of a C2 step were
    0.62 ms of it (profiles/r05/c2/step_breakdown.txt)."""

    def __init__(self, enabled=True):
        self.on = bool(enabled) and _WG_DEFER_ON

    def __enter__(self):
        if self.on:
            if _WG_PENDING[0] is not None:
                raise RuntimeError("deferred_wgrads: scopes do not nest")
            _WG_PENDING[0] = []
        return self

    def __exit__(self, exc_type, *exc):
        if self.on:
            try:
                if exc_type is None:
                    flush_wgrads()
            finally:
                _WG_PENDING[0] = None
        return False


def flush_wgrads():
    """Run the pending slice sums now (no-op outside a deferred_wgrads scope)."""
    pend = _WG_PENDING[0]
    if not pend:
        return
    import ctypes

    from ..moe import _lib as L

    s = L._stream()
    for i in range(0, len(pend), _WG_BATCH):
        chunk = pend[i:i + _WG_BATCH]
        n = len(chunk)
        parts = (ctypes.c_void_p * n)(*[c[0].data_ptr() for c in chunk])
        nsplit = (ctypes.c_int * n)(*[c[1] for c in chunk])
        numel = (ctypes.c_longlong * n)(*[c[2] for c in chunk])
        dws = (ctypes.c_void_p * n)(*[c[3].data_ptr() for c in chunk])
        cv = lambda a: ctypes.cast(a, ctypes.c_void_p)  # noqa: E731
        L._check(L.lib().rtdetr_conv_wgrad_reduce_batch(n, cv(parts), cv(nsplit), cv(numel), cv(dws), 1, s),
                 "rtdetr_conv_wgrad_reduce_batch")
    pend.clear()


class GradLink:
    """Hand-off between a residual block's output y = relu(s) (made by
    _ConvHIPFork) and the next block when its shortcut is the identity: y's
    gradient is mask(y) * (g_a + g_s) with g_a from the next block's branch2a
    data gradient and g_s the next block's own output gradient (its fork's
    g, which reaches y through the identity shortcut).  The next fork's
    backward stores g_s here; branch2a's backward, which autograd runs after
    it, adds g_s and applies the mask in its dgrad epilogue and marks the
    result final; y's fork then takes it as is (no rtdetr_relu_grad2 pass)."""

    __slots__ = ("g_short", "final", "g_ext", "ext_used")

    def __init__(self):
        self.g_short = None
        self.final = False
        # a returned stage output's gradient from its external consumer (the
        # encoder), handed over by backbone.stage_taps instead of autograd's
        # accumulation; ext_used: the average-pool backward folded it into the
        # shortcut gradient (so branch2a's dgrad epilogue adds and masks it)
        self.g_ext = None
        self.ext_used = False


class _ConvHIP(torch.autograd.Function):
    """y = relu?(conv(x, w) + bias) on the HIP kernels (bias: frozen fp32
    [N] or None, no gradient).

    mask_input: x is a ReLU output whose ONLY consumer is this convolution;
    the data gradient is then masked by (x > 0) in the dgrad epilogue, so the
    producer may skip its own ReLU backward.  grad_premasked: this layer's
    ReLU output feeds only a convolution that does that, so the incoming
    gradient is already masked (no threshold pass here)."""

    @staticmethod
    def forward(ctx, x, w, bias=None, relu=False, mask_input=False, grad_premasked=False, link=None, st=1):
        x = _nhwc(x)
        w = _nhwc(w)
        y = _fwd(x, w, bias, None, relu, st)
        ctx.st = st
        ctx.flags = (bool(relu) and not grad_premasked, bool(mask_input))
        ctx.link = link  # x is a block output (GradLink): finish its gradient here when the hand-off is there
        ctx.save_for_backward(x, w, y if ctx.flags[0] else None)
        return y

    @staticmethod
    def backward(ctx, gy):
        x, w, y = ctx.saved_tensors
        relu_here, mask_input = ctx.flags
        g = torch.ops.aten.threshold_backward(gy, y, 0) if relu_here else gy
        link, add = ctx.link, None
        if link is not None and link.g_short is not None and ctx.needs_input_grad[0]:
            add, mask_input = link.g_short, True
            link.g_short, link.final = None, True
        gx, gw = _bwd(x, w, g, ctx.needs_input_grad[0], ctx.needs_input_grad[1], mask_input, add, ctx.st)
        return gx, gw, None, None, None, None, None, None


class _ConvHIPFork(torch.autograd.Function):
    """(y, y') with y = relu((conv(x, w) + resid) + bias) and y' aliasing y: a
    residual block's output for its two consumers (the next block's branch2a
    and shortcut), the add and ReLU fused into the convolution's epilogue.
    Backward: g = (dy + dy') * (y > 0) in one pass (rtdetr_relu_grad2_nhwc),
    the gradient of both the convolution output and resid."""

    @staticmethod
    def forward(ctx, x, w, resid, bias, mask_input=False, link_in=None, link_out=None):
        x = _nhwc(x)
        w = _nhwc(w)
        y = _fwd(x, w, bias, _nhwc(resid), True)
        ctx.set_materialize_grads(False)  # an unused handle: no zero-filled gradient
        ctx.mask_input = bool(mask_input)
        ctx.links = (link_in, link_out)  # link_in: resid is the previous block's output (identity shortcut)
        ctx.save_for_backward(x, w, y)
        return y, y.view_as(y)

    @staticmethod
    def backward(ctx, dy1, dy2):
        from ..moe import _lib as L

        x, w, y = ctx.saved_tensors
        link_in, link_out = ctx.links
        ext = None  # the encoder's gradient of this output (stage_taps), unless already folded in
        if link_out is not None:
            if link_out.g_ext is not None and not link_out.ext_used:
                ext = link_out.g_ext
            link_out.g_ext, link_out.ext_used = None, False
        if link_out is not None and link_out.final:
            g = dy1  # the next block's branch2a dgrad already added dy2 and masked (GradLink)
            link_out.final = False
            if ext is not None:  # (not folded in by the shortcut's pool backward: masked here)
                g = g + torch.where(y > 0, ext, torch.zeros_like(ext))
        else:
            if link_out is not None:
                link_out.g_short = None
            if ext is not None:
                dy1 = ext if dy1 is None else dy1 + ext
            if dy1 is None and dy2 is None:
                return None, None, None, None, None, None, None
            if dy1 is None:
                dy1, dy2 = dy2, None
            g = L.relu_grad2_nhwc(_nhwc(dy1), None if dy2 is None else _nhwc(dy2), y)
        if link_in is not None:
            link_in.g_short = g
        gx, gw = _bwd(x, w, g, ctx.needs_input_grad[0], ctx.needs_input_grad[1], ctx.mask_input)
        return gx, gw, g if ctx.needs_input_grad[2] else None, None, None, None, None


class GradSlot:
    """Hand-off of an activation's gradient between its two convolution
    consumers (the encoder's PAN inputs P3 / P4: the encoder's downsampling
    convolution and the decoder's input projection).  The first consumer
    created (collector) runs its backward LAST (autograd runs later-created
    nodes first); the later one (depositor) parks its data gradient here and
    returns none, and the collector's dgrad epilogue adds it (the `add`
    operand) -- no autograd accumulation launch.  A depositor that runs after
    the collector (closed slot) returns its gradient to autograd as usual."""

    __slots__ = ("g", "closed", "has_collector", "__weakref__")

    def __init__(self):
        self.g = None
        self.closed = False
        self.has_collector = False
        _OPEN_SLOTS.append(self)
        if len(_OPEN_SLOTS) > 256:  # forwards whose backward never ran (no check after them)
            del _OPEN_SLOTS[:128]


_OPEN_SLOTS: list = []


def check_grad_slots():
    """After a backward: every GradSlot created since the last check must have
    handed its parked gradient to the collector.  A gradient still parked means
    the collector's backward never ran (its output did not reach the loss) and
    the depositor's data gradient would be lost silently -- raise instead."""
    pending = [s for s in _OPEN_SLOTS if s.g is not None]
    _OPEN_SLOTS.clear()
    if pending:
        for s in pending:
            s.g = None
        raise RuntimeError(f"{len(pending)} GradSlot gradient(s) were parked but never collected: the collecting "
                           "convolution's output did not reach the loss")


class _ConvHIPStats(torch.autograd.Function):
    """(conv(x, w), BatchNorm partials fp32 [1, nblk, 2, N] of its output) for
    a training BatchNorm that follows (fused.bn_act(parts=...)): the
    statistics pass over y is folded into the convolution's epilogue.
    slot / collect: see GradSlot (collect True: this is the collector)."""

    @staticmethod
    def forward(ctx, x, w, nblk, st, slot=None, collect=False):
        x = _nhwc(x)
        w = _nhwc(w)
        part = torch.empty((1, nblk, 2, w.shape[0]), dtype=torch.float32, device=x.device)
        y = _fwd_stats(x, w, part[0], st)
        ctx.st = st
        ctx.slot, ctx.collect = slot, collect
        ctx.save_for_backward(x, w)
        ctx.mark_non_differentiable(part)
        ctx.set_materialize_grads(False)
        return y, part

    @staticmethod
    def backward(ctx, gy, _gpart):
        x, w = ctx.saved_tensors
        slot = ctx.slot
        add = None
        if slot is not None and ctx.collect:
            add, slot.g, slot.closed = slot.g, None, True
        if gy is None:
            if add is not None:
                return add, None, None, None, None, None
            return None, None, None, None, None, None
        gx, gw = _bwd(x, w, gy, ctx.needs_input_grad[0], ctx.needs_input_grad[1], False, add, ctx.st)
        if slot is not None and not ctx.collect and not slot.closed and gx is not None and slot.g is None:
            slot.g, gx = gx, None  # parked for the collector's dgrad epilogue
        return gx, gw, None, None, None, None


def conv_module_stats(conv: torch.nn.Conv2d, x):
    """(conv(x), BatchNorm partials or None): `conv_module` whose HIP forward
    also sums its output's BatchNorm statistics (_ConvHIPStats) when that
    applies (MOE_CONV_BN_STATS=0: never)."""
    if _STATS_ON and conv.bias is None:
        xc, wc = _autocast_operands(x, conv.weight, conv.stride, conv.padding, conv.dilation, conv.groups)
        if hip_conv_ok(xc, wc, conv.stride, conv.padding, conv.dilation, conv.groups):
            st = _stride(conv.stride)
            nblk = _stats_blocks(xc, wc, st)
            if nblk > 0:
                slot = getattr(x, "grad_slot", None) if xc is x and torch.is_grad_enabled() else None
                collect = False
                if slot is not None and not slot.has_collector:
                    slot.has_collector = collect = True
                return _ConvHIPStats.apply(xc, wc, nblk, st, slot, collect)
            return _ConvHIP.apply(xc, wc, None, False, False, False, None, st), None
    return conv_module(conv, x), None


class _ConvHIPPair(torch.autograd.Function):
    """(conv(x, w1), conv(x, w2)): two stride-1 convolutions of the same input
    (RT-DETR's RepVgg 3x3 + 1x1 branches, CSPRep's two 1x1 entry layers).
    Backward: the second data gradient adds the first in its epilogue (the
    `add` operand of rtdetr_conv_dgrad), so x's gradient needs no separate
    accumulation launch by autograd.  nblk > 0: the forwards also write their
    outputs' BatchNorm partials, returned as a third output [2, nblk, 2, N]."""

    @staticmethod
    def forward(ctx, x, w1, w2, nblk=0):
        x = _nhwc(x)
        w1, w2 = _nhwc(w1), _nhwc(w2)
        ctx.save_for_backward(x, w1, w2)
        ctx.set_materialize_grads(False)
        if nblk > 0:
            part = torch.empty((2, nblk, 2, w1.shape[0]), dtype=torch.float32, device=x.device)
            ctx.mark_non_differentiable(part)
            return _fwd_stats(x, w1, part[0]), _fwd_stats(x, w2, part[1]), part
        return _fwd(x, w1), _fwd(x, w2)

    @staticmethod
    def backward(ctx, g1, g2, _gpart=None):
        x, w1, w2 = ctx.saved_tensors
        nx, nw1, nw2 = ctx.needs_input_grad[:3]
        gx = gw1 = gw2 = None
        if g1 is not None:
            gx, gw1 = _bwd(x, w1, g1, nx, nw1, False)
        if g2 is not None:
            gx, gw2 = _bwd(x, w2, g2, nx, nw2, False, add=gx)
        return gx, gw1, gw2, None


def conv_pair(conv1: torch.nn.Conv2d, conv2: torch.nn.Conv2d, x, stats=False):
    """(conv1(x), conv2(x)[, parts]) for two bias-free stride-1 nn.Conv2d on
    the same input: one autograd node on the HIP kernels (_ConvHIPPair) when
    both take them (after autocast's casts), else conv_module twice.
    stats=True: a third element, the outputs' BatchNorm partials
    [2, nblk, 2, N] for fused.bn_act(parts=...), or None."""
    if (_PAIR_ON and conv1.bias is None and conv2.bias is None and _stride(conv1.stride) == 1
            and _stride(conv2.stride) == 1 and conv1.out_channels == conv2.out_channels):
        xc, w1 = _autocast_operands(x, conv1.weight, conv1.stride, conv1.padding, conv1.dilation, conv1.groups)
        _, w2 = _autocast_operands(x, conv2.weight, conv2.stride, conv2.padding, conv2.dilation, conv2.groups)
        if (hip_conv_ok(xc, w1, conv1.stride, conv1.padding, conv1.dilation, conv1.groups)
                and hip_conv_ok(xc, w2, conv2.stride, conv2.padding, conv2.dilation, conv2.groups)):
            if not stats:
                return _ConvHIPPair.apply(xc, w1, w2)
            nblk = _stats_blocks(xc, w1) if _STATS_ON else 0
            if nblk > 0 and nblk == _stats_blocks(xc, w2):
                return _ConvHIPPair.apply(xc, w1, w2, nblk)
            return _ConvHIPPair.apply(xc, w1, w2) + (None,)
    if stats:
        return conv_module(conv1, x), conv_module(conv2, x), None
    return conv_module(conv1, x), conv_module(conv2, x)


_PAIR_ON = os.environ.get("MOE_CONV_PAIR", "1") != "0"
_STATS_ON = os.environ.get("MOE_CONV_BN_STATS", "1") != "0"


def _autocast_operands(x, w, stride, padding, dilation=1, groups=1):
    """Under bf16 autocast (TrainStep precision "amp": fp32 weights) a
    convolution computes on bf16 casts of its input and weight -- autocast's
    own rule for F.conv2d -- so the cast operands go to the HIP kernels too
    (MIOpen's atomic weight-gradient solvers are not graph-replay safe:
    DESIGN.md 5)."""
    if (x.is_cuda and x.dim() == 4 and x.shape[0] > 0 and torch.is_autocast_enabled("cuda")
            and torch.get_autocast_dtype("cuda") == torch.bfloat16
            and x.dtype in (torch.float32, torch.bfloat16) and w.dtype in (torch.float32, torch.bfloat16)
            and hip_conv_ok_for(True, torch.bfloat16, x.shape[1], w, stride, padding, dilation, groups,
                                w_dtype=torch.bfloat16)):
        return x.to(torch.bfloat16), w.to(torch.bfloat16)
    return x, w


def conv2d(x, weight, stride=1, padding=0):
    """F.conv2d(x, weight, None, stride, padding) -- on the HIP kernels when
    hip_conv_ok (after autocast's bf16 casts), else MIOpen."""
    xc, wc = _autocast_operands(x, weight, stride, padding)
    if hip_conv_ok(xc, wc, stride, padding):
        return _ConvHIP.apply(xc, wc, None, False, False, False, None, _stride(stride))
    return F.conv2d(x, weight, None, stride, padding)


def conv2d_bias_relu(x, weight, bias, mask_input=False, grad_premasked=False, link=None, stride=1):
    """relu(conv2d(x, weight) + bias[c]) in one HIP launch (padding (k-1)/2;
    the caller checked hip_conv_ok).  bias: fp32 [Cout], no gradient.
    See _ConvHIP for mask_input / grad_premasked, GradLink for link (x a
    block output whose other consumer is the identity shortcut)."""
    return _ConvHIP.apply(x, weight, bias.float().contiguous(), True, mask_input, grad_premasked, link,
                          _stride(stride))


def conv2d_add_bias_relu_fork(x, weight, resid, bias, mask_input=False, link_in=None):
    """(y, y) with y = relu((conv2d(x, weight) + resid) + bias[c]) in one HIP
    launch -- see _ConvHIPFork.  link_in: resid is the previous block's output
    through an identity shortcut (GradLink).  y carries the GradLink for the
    next block as y.grad_link."""
    link_out = GradLink()
    y, y2 = _ConvHIPFork.apply(x, weight, resid, None if bias is None else bias.float().contiguous(), mask_input,
                               link_in, link_out)
    y.grad_link = link_out
    return y, y2


def conv_module(conv: torch.nn.Conv2d, x):
    """A bias-free nn.Conv2d applied through conv2d (falls back to the module)."""
    if conv.bias is None:
        xc, wc = _autocast_operands(x, conv.weight, conv.stride, conv.padding, conv.dilation, conv.groups)
        if hip_conv_ok(xc, wc, conv.stride, conv.padding, conv.dilation, conv.groups):
            return _ConvHIP.apply(xc, wc, None, False, False, False, None, _stride(conv.stride))
    return conv(x)
