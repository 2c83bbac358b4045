"""Convolutions of the RT-DETR body on libmoe_hip's implicit-GEMM kernels
(csrc/conv.hip: rtdetr_conv_fwd / rtdetr_conv_dgrad / rtdetr_conv_wgrad).

``conv2d(x, weight, stride, padding)`` takes the HIP kernels for the
convolutions they cover -- stride 1, "same" padding, 1x1 or 3x3, no groups,
channel counts that are multiples of 128, bf16 channels_last activations and
weights on the GPU (the HybridEncoder's RepVGG / CSP layers and the ResNet
bottleneck convolutions of 128 / 256 / 512 / 1024 / 2048 channels) -- and
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
    if not (_ENABLED[0] and x.is_cuda and x.dim() == 4 and w.dim() == 4):
        return False
    N, C, kh, kw = w.shape
    ks = kh
    st = stride if isinstance(stride, int) else (stride[0] if stride[0] == stride[1] else -1)
    pd = padding if isinstance(padding, int) else (padding[0] if padding[0] == padding[1] else -1)
    dl = dilation if isinstance(dilation, int) else (dilation[0] if dilation[0] == dilation[1] else -1)
    return (x.dtype == torch.bfloat16 and w.dtype == torch.bfloat16 and kh == kw and ks in (1, 3) and st == 1
            and pd == (ks - 1) // 2 and dl == 1 and groups == 1 and x.shape[1] == C and C % 128 == 0
            and N % 128 == 0 and x.shape[0] > 0)


class _ConvHIP(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, w):
        from ..moe import _lib as L

        B, C, H, W = x.shape
        N, _, ks, _ = w.shape
        x = _nhwc(x)
        w = _nhwc(w)
        y = torch.empty((B, N, H, W), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        L._check(L.lib().rtdetr_conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), _zero(x.device).data_ptr(),
                                         B, H, W, C, N, ks, L._stream()), "rtdetr_conv_fwd")
        ctx.save_for_backward(x, w)
        return y

    @staticmethod
    def backward(ctx, gy):
        from ..moe import _lib as L

        x, w = ctx.saved_tensors
        B, C, H, W = x.shape
        N, _, ks, _ = w.shape
        gy = _nhwc(gy.to(torch.bfloat16))
        z = _zero(x.device).data_ptr()
        s = L._stream()
        gx = gw = None
        if ctx.needs_input_grad[0]:
            gx = torch.empty((B, C, H, W), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
            nb = L.lib().rtdetr_conv_dgrad_workspace(B, H, W, C, N, ks)
            work = torch.empty(nb // 2, dtype=torch.bfloat16, device=x.device) if nb > 0 else None
            L._check(L.lib().rtdetr_conv_dgrad(gy.data_ptr(), w.data_ptr(), None if work is None else work.data_ptr(),
                                               gx.data_ptr(), z, B, H, W, C, N, ks, s), "rtdetr_conv_dgrad")
        if ctx.needs_input_grad[1]:
            ns = L.lib().rtdetr_conv_wgrad_splits(B, H, W, C, N, ks)
            part = torch.empty(ns * N * C * ks * ks, dtype=torch.float32, device=x.device)
            gw = torch.empty_like(w, memory_format=torch.channels_last)
            L._check(L.lib().rtdetr_conv_wgrad(gy.data_ptr(), x.data_ptr(), part.data_ptr(), ns, gw.data_ptr(), 1,
                                               z, B, H, W, C, N, ks, s), "rtdetr_conv_wgrad")
        return gx, gw


def conv2d(x, weight, stride=1, padding=0):
    """F.conv2d(x, weight, None, stride, padding) -- on the HIP kernels when
    hip_conv_ok, else MIOpen."""
    if hip_conv_ok(x, weight, stride, padding):
        return _ConvHIP.apply(x, weight)
    return F.conv2d(x, weight, None, stride, padding)


def conv_module(conv: torch.nn.Conv2d, x):
    """A bias-free nn.Conv2d applied through conv2d (falls back to the module)."""
    if conv.bias is None and hip_conv_ok(x, conv.weight, conv.stride, conv.padding, conv.dilation, conv.groups):
        return _ConvHIP.apply(x, conv.weight)
    return conv(x)
