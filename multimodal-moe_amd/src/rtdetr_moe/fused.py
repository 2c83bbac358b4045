"""Frozen-BatchNorm convolution epilogues of the backbone.

rtdetrv2_r50vd freezes the backbone's BatchNorm statistics (``freeze_norm``),
so conv + BN is a convolution with per-output-channel scaled weights plus a
channel bias.  The scale is folded into the (tiny) weight tensor; the bias is
applied together with what follows it in one pass over the NHWC activation by
the HIP kernels of libmoe_hip (include/moe_hip.h, rtdetr_*_nhwc):

  BiasReLU      y = relu(conv + bias)             branch2a / branch2b / stem
  AddBiasReLU   y = relu(conv_c + short + bias)   block output (bias = both BNs' shifts)

Backward is one mask of the incoming gradient (threshold_backward on y),
shared by both inputs of AddBiasReLU; the bias carries no gradient (frozen).
AddBiasReLUFork returns the block output twice -- one handle for the next
block's branch2a, one for its shortcut -- so that its backward receives the
two gradients separately and sums + masks them in one pass
(rtdetr_relu_grad2_nhwc) instead of autograd's accumulate + threshold.
CPU tensors (config C1 plumbing) take the same math in torch ops.
"""
from __future__ import annotations

import os

import torch

from ..moe import _lib as L


def _gpu_ok(t: torch.Tensor) -> bool:
    return t.is_cuda and t.dtype == torch.bfloat16 and t.is_contiguous(memory_format=torch.channels_last)


class BiasReLU(torch.autograd.Function):
    """y = relu(x + bias[c]), in place on x (a fresh convolution output)."""

    @staticmethod
    def forward(ctx, x, bias):
        if x.is_cuda:
            if not _gpu_ok(x):
                raise L.MoEKernelError("BiasReLU needs a channels_last bf16 activation on the GPU")
            L.bias_act_nhwc(x, bias.float().contiguous(), True, out=x)
        else:
            x.add_(bias.to(x.dtype).view(1, -1, 1, 1)).relu_()
        ctx.mark_dirty(x)
        ctx.save_for_backward(x)
        return x

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        return torch.ops.aten.threshold_backward(dy, y, 0), None


class AddBiasReLU(torch.autograd.Function):
    """y = relu(a + b + bias[c]) (bias may be None)."""

    @staticmethod
    def forward(ctx, a, b, bias):
        if a.is_cuda:
            if not (_gpu_ok(a) and _gpu_ok(b)):
                raise L.MoEKernelError("AddBiasReLU needs channels_last bf16 activations on the GPU")
            y = L.add_bias_relu_nhwc(a, b, None if bias is None else bias.float().contiguous())
        else:
            y = a + b
            if bias is not None:
                y = y + bias.to(y.dtype).view(1, -1, 1, 1)
            y = y.relu_()
        ctx.save_for_backward(y)
        return y

    @staticmethod
    def backward(ctx, dy):
        (y,) = ctx.saved_tensors
        g = torch.ops.aten.threshold_backward(dy, y, 0)
        return g, g, None


def _nhwc_ok(*ts) -> bool:
    return all(t is None or _gpu_ok(t) for t in ts)


class AddBiasReLUFork(torch.autograd.Function):
    """(y, y') with y = relu(a + b + bias[c]); y' aliases y.  Backward:
    g = (dy + dy') * (y > 0) for both a and b, one pass."""

    @staticmethod
    def forward(ctx, a, b, bias):
        y = AddBiasReLU.forward(ctx, a, b, bias)
        ctx.set_materialize_grads(False)  # an unused handle: no zero-filled gradient
        return y, y.view_as(y)

    @staticmethod
    def backward(ctx, dy1, dy2):
        (y,) = ctx.saved_tensors
        if dy1 is None and dy2 is None:
            return None, None, None
        if dy1 is None:
            dy1, dy2 = dy2, None
        if y.is_cuda and _nhwc_ok(dy1, dy2):
            g = L.relu_grad2_nhwc(dy1, dy2, y)
        else:
            g = torch.ops.aten.threshold_backward(dy1 if dy2 is None else dy1 + dy2, y, 0)
        return g, g, None


# ---------------------------------------------------------------------------
# Training-mode BatchNorm + activation of the HybridEncoder (not frozen):
# ConvNormLayer(act="silu") is silu(BN(conv)), RepVggBlock is
# silu(BN1(conv3x3) + BN2(conv1x1)).  libmoe_hip's rtdetr_bn_act_fwd/_bwd do
# the batch statistics, the normalisation of both branches, their sum and the
# SiLU in three launches each way (torch: three MIOpen kernels per BN each way
# plus add / silu / silu_backward passes).
# ---------------------------------------------------------------------------
class _BatchNormAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, act, eps, momentum, bns, parts, resid, *args):
        nb = len(bns)
        xs, gammas, betas = args[:nb], args[nb:2 * nb], args[2 * nb:3 * nb]
        rms = [bn.running_mean for bn in bns]
        rvs = [bn.running_var for bn in bns]
        if parts is not None:  # statistics summed by the producing convolution (conv.conv_module_stats)
            y, saved = L.bn_act_fwd_part(list(xs), list(gammas), list(betas), rms, rvs, act, eps, momentum, parts,
                                         resid=resid)
        else:
            y, saved = L.bn_act_fwd(list(xs), list(gammas), list(betas), rms, rvs, act, eps, momentum, resid=resid)
        ctx.act, ctx.nb = act, nb
        ctx.save_for_backward(*xs, *gammas, saved)
        return y

    @staticmethod
    def backward(ctx, dy):
        nb = ctx.nb
        t = ctx.saved_tensors
        xs, gammas, saved = list(t[:nb]), list(t[nb:2 * nb]), t[2 * nb]
        dy = dy.contiguous(memory_format=torch.channels_last)
        dxs, dgb = L.bn_act_bwd(dy, xs, gammas, saved, ctx.act)
        dres = dy if ctx.needs_input_grad[5] else None  # y = act(z) + resid: resid's gradient is dy itself
        return (None, None, None, None, None, dres, *dxs, *[dgb[i, 0] for i in range(nb)],
                *[dgb[i, 1] for i in range(nb)])


def bn_act_ok(xs, bns) -> bool:
    """The fused kernels apply: GPU channels_last bf16 branches of one shape,
    training-mode affine BatchNorm2d with running statistics and a momentum,
    C a power of two in [8, 2048]."""
    x = xs[0]
    if not (x.is_cuda and x.dim() == 4 and all(_gpu_ok(t) and t.shape == x.shape for t in xs)):
        return False
    C = x.shape[1]
    if C < 8 or C > 2048 or C & (C - 1) or x.numel() // C < 2:
        return False
    for bn in bns:
        if not (isinstance(bn, torch.nn.BatchNorm2d) and bn.training and bn.affine and bn.track_running_stats
                and bn.momentum is not None and bn.running_mean is not None
                and bn.weight.dtype == torch.float32 and bn.eps == bns[0].eps and bn.momentum == bns[0].momentum):
            return False
    return True


# MOE_BN_EVAL=0: inference-mode BatchNorms through torch (A/B switch)
_BN_EVAL = os.environ.get("MOE_BN_EVAL", "1") != "0"


def bn_eval_ok(xs, bns) -> bool:
    """Inference-mode BatchNorms (running statistics, no gradient wanted) that
    rtdetr_bn_act_eval takes: GPU channels_last bf16 branches of one shape, C
    a power of two in [8, 2048], fp32 affine and statistics."""
    if not _BN_EVAL or torch.is_grad_enabled():
        return False
    x = xs[0]
    if not (x.is_cuda and x.dim() == 4 and all(_gpu_ok(t) and t.shape == x.shape for t in xs)):
        return False
    C = x.shape[1]
    if C < 8 or C > 2048 or C & (C - 1):
        return False
    return all(isinstance(bn, torch.nn.BatchNorm2d) and not bn.training and bn.affine and bn.track_running_stats
               and bn.running_mean is not None and bn.running_var is not None
               and all(t.dtype == torch.float32 for t in (bn.weight, bn.bias, bn.running_mean, bn.running_var))
               and bn.eps == bns[0].eps for bn in bns)


def bn_act_eval(xs, bns, act: str | None, resid=None):
    """act(sum_i BN_i(x_i)) [+ resid] with running statistics in one HIP pass
    (callers check bn_eval_ok)."""
    bns = list(bns)
    if resid is not None and not (_gpu_ok(resid) and resid.shape == xs[0].shape and resid.data_ptr() % 16 == 0):
        return bn_act_eval(xs, bns, act) + resid
    return L.bn_act_eval(list(xs), [bn.weight for bn in bns], [bn.bias for bn in bns],
                         [bn.running_mean for bn in bns], [bn.running_var for bn in bns],
                         1 if act == "silu" else 0, float(bns[0].eps), resid)


def bn_act(xs, bns, act: str | None, parts=None, resid=None):
    """act(sum_i BN_i(x_i)) [+ resid] through libmoe_hip (callers check
    bn_act_ok).  parts: the branches' batch-statistics partials fp32
    [nb, nblk, 2, C] from their convolutions' epilogues
    (conv.conv_module_stats / conv_pair), or None (a statistics pass over x).
    resid: a tensor like x added after the activation in the same pass (the
    CSPRep layer's shortcut branch; bits of the bf16 activation then a bf16
    add).  num_batches_tracked is not advanced (it only matters with
    momentum=None)."""
    bns = list(bns)
    a = 1 if act == "silu" else 0
    if resid is not None and not (_gpu_ok(resid) and resid.shape == xs[0].shape and resid.data_ptr() % 16 == 0):
        return _BatchNormAct.apply(a, float(bns[0].eps), float(bns[0].momentum), bns, parts, None, *xs,
                                   *[bn.weight for bn in bns], *[bn.bias for bn in bns]) + resid
    return _BatchNormAct.apply(a, float(bns[0].eps), float(bns[0].momentum), bns, parts, resid, *xs,
                               *[bn.weight for bn in bns], *[bn.bias for bn in bns])
