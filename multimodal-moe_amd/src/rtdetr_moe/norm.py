"""Residual add + LayerNorm of the post-norm transformer layers.

Every AIFI encoder layer and decoder layer of RT-DETR computes
``norm(x + sublayer(x))`` (reference engine: the
Ultralytics RT-DETR transformer layers behind ``rtdetr.py:82-94``).
``AddLayerNorm`` is an ``nn.LayerNorm`` (same parameters and state-dict keys)
whose ``forward(a, b=None)`` returns ``LayerNorm(a + b)``: on the GPU one HIP
launch forward and two backward (libmoe_hip ``rtdetr_add_layer_norm_*``,
fp32 statistics, deterministic parameter gradients), in place of the residual
add and torch's layer-norm kernels; on the CPU (config C1) the same math in
torch ops.
"""
from __future__ import annotations

import os

import torch
import torch.nn.functional as F
from torch import nn

from ..moe import _lib as L

# MOE_FUSED_LN=0: torch's add + layer_norm instead (A/B switch)
_FUSED_LN = os.environ.get("MOE_FUSED_LN", "1") != "0"


def _fused_ok(a: torch.Tensor, b: torch.Tensor | None, w: torch.Tensor, bias: torch.Tensor | None) -> bool:
    d = a.shape[-1]
    if not (_FUSED_LN and a.is_cuda and a.dtype == torch.bfloat16 and a.is_contiguous() and d in (128, 256, 512)):
        return False
    if b is not None and not (b.dtype == torch.bfloat16 and b.shape == a.shape and b.is_contiguous()):
        return False
    return bias is not None and w.dtype in (torch.bfloat16, torch.float32) and bias.dtype == w.dtype


class _AddLayerNorm(torch.autograd.Function):
    @staticmethod
    def forward(ctx, a, b, weight, bias, eps):
        d = a.shape[-1]
        T = a.numel() // d
        w = weight.contiguous()
        bb = bias.contiguous()
        out = torch.empty_like(a)
        mean = torch.empty(T, dtype=torch.float32, device=a.device)
        rstd = torch.empty(T, dtype=torch.float32, device=a.device)
        wb = int(w.dtype == torch.bfloat16)
        L._check(L.lib().rtdetr_add_layer_norm_fwd(a.data_ptr(), b.data_ptr() if b is not None else None,
                                                   w.data_ptr(), bb.data_ptr(), wb, T, d, float(eps),
                                                   out.data_ptr(), mean.data_ptr(), rstd.data_ptr(), L._stream()),
                 "rtdetr_add_layer_norm_fwd")
        ctx.save_for_backward(a, b if b is not None else torch.empty(0, device=a.device), w, mean, rstd)
        ctx.has_b = b is not None
        return out

    @staticmethod
    def backward(ctx, dout):
        a, b, w, mean, rstd = ctx.saved_tensors
        b = b if ctx.has_b else None
        d = a.shape[-1]
        T = a.numel() // d
        dout = dout.to(torch.bfloat16).contiguous()
        ds = torch.empty_like(a)
        lib = L.lib()
        P = int(lib.rtdetr_add_layer_norm_parts(T))
        parts = torch.empty((P, 2 * d), dtype=torch.float32, device=a.device)
        dwb = torch.empty((2, d), dtype=w.dtype, device=a.device)
        L._check(lib.rtdetr_add_layer_norm_bwd(dout.data_ptr(), a.data_ptr(), b.data_ptr() if b is not None else None,
                                               w.data_ptr(), int(w.dtype == torch.bfloat16), mean.data_ptr(),
                                               rstd.data_ptr(), T, d, ds.data_ptr(), parts.data_ptr(), P,
                                               dwb.data_ptr(), L._stream()),
                 "rtdetr_add_layer_norm_bwd")
        return ds, (ds if ctx.has_b else None), dwb[0], dwb[1], None


def add_layer_norm(a: torch.Tensor, b: torch.Tensor | None, weight: torch.Tensor, bias: torch.Tensor,
                   eps: float = 1e-5) -> torch.Tensor:
    """LayerNorm(a + b) over the last dimension (b may be None)."""
    if _fused_ok(a, b, weight, bias):
        return _AddLayerNorm.apply(a, b, weight, bias, eps)
    s = a if b is None else a + b
    return F.layer_norm(s, (a.shape[-1],), weight, bias, eps)


class AddLayerNorm(nn.LayerNorm):
    """nn.LayerNorm whose forward(a, b=None) is LayerNorm(a + b) (fused on the GPU)."""

    def forward(self, a: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:  # type: ignore[override]
        if len(self.normalized_shape) != 1 or self.weight is None:
            s = a if b is None else a + b
            return super().forward(s)
        return add_layer_norm(a, b, self.weight, self.bias, self.eps)
