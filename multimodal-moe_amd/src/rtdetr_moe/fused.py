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
