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
from . import linear as _LIN

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
        ctx.leaves = (weight, bias)
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
        defer = _defer_ln(ctx.leaves, w)
        dwb = None if defer else torch.empty((2, d), dtype=w.dtype, device=a.device)
        L._check(lib.rtdetr_add_layer_norm_bwd(dout.data_ptr(), a.data_ptr(), b.data_ptr() if b is not None else None,
                                               w.data_ptr(), int(w.dtype == torch.bfloat16), mean.data_ptr(),
                                               rstd.data_ptr(), T, d, ds.data_ptr(), parts.data_ptr(), P,
                                               None if defer else dwb.data_ptr(), L._stream()),
                 "rtdetr_add_layer_norm_bwd")
        if defer:  # [dgamma; dbeta] from the partials after the backward, batched
            _LIN._ACTIVE[0].add_ln(parts, *ctx.leaves)
            return ds, (ds if ctx.has_b else None), None, None, None
        return ds, (ds if ctx.has_b else None), dwb[0], dwb[1], None


class _AddLayerNormPos(torch.autograd.Function):
    """(t, t + pos) with t = LayerNorm(a + b) in one launch (the decoder's
    cross-attention query); backward: t's two gradients summed inside the
    LayerNorm backward (no autograd accumulation launch), pos's gradient is
    the second one itself."""

    @staticmethod
    def forward(ctx, a, b, weight, bias, pos, eps):
        d = a.shape[-1]
        T = a.numel() // d
        w = weight.contiguous()
        bb = bias.contiguous()
        out = torch.empty_like(a)
        out2 = torch.empty_like(a)
        mean = torch.empty(T, dtype=torch.float32, device=a.device)
        rstd = torch.empty(T, dtype=torch.float32, device=a.device)
        L._check(L.lib().rtdetr_add_layer_norm_pos_fwd(a.data_ptr(), b.data_ptr(), w.data_ptr(), bb.data_ptr(),
                                                       int(w.dtype == torch.bfloat16), T, d, float(eps),
                                                       pos.data_ptr(), out.data_ptr(), out2.data_ptr(),
                                                       mean.data_ptr(), rstd.data_ptr(), L._stream()),
                 "rtdetr_add_layer_norm_pos_fwd")
        ctx.save_for_backward(a, b, w, mean, rstd)
        ctx.set_materialize_grads(False)
        ctx.leaves = (weight, bias)
        return out, out2

    @staticmethod
    def backward(ctx, dout, dout2):
        a, b, w, mean, rstd = ctx.saved_tensors
        if dout is None and dout2 is None:
            return None, None, None, None, None, None
        d = a.shape[-1]
        T = a.numel() // d
        g1 = (dout if dout is not None else dout2).to(torch.bfloat16).contiguous()
        g2 = dout2.to(torch.bfloat16).contiguous() if (dout is not None and dout2 is not None) else None
        ds = torch.empty_like(a)
        lib = L.lib()
        P = int(lib.rtdetr_add_layer_norm_parts(T))
        parts = torch.empty((P, 2 * d), dtype=torch.float32, device=a.device)
        defer = _defer_ln(ctx.leaves, w)
        dwb = None if defer else torch.empty((2, d), dtype=w.dtype, device=a.device)
        L._check(lib.rtdetr_add_layer_norm_bwd2(g1.data_ptr(), g2.data_ptr() if g2 is not None else None,
                                                a.data_ptr(), b.data_ptr(), w.data_ptr(),
                                                int(w.dtype == torch.bfloat16), mean.data_ptr(), rstd.data_ptr(),
                                                T, d, ds.data_ptr(), parts.data_ptr(), P,
                                                None if defer else dwb.data_ptr(), L._stream()),
                 "rtdetr_add_layer_norm_bwd2")
        if defer:
            _LIN._ACTIVE[0].add_ln(parts, *ctx.leaves)
            return ds, ds, None, None, dout2, None
        return ds, ds, dwb[0], dwb[1], dout2, None


# MOE_DEFER_LN=0: each LayerNorm's [dgamma; dbeta] final right after its row
# pass (A/B switch; default: deferred into linear.DeferredWgrad's batched flush)
_DEFER_LN = os.environ.get("MOE_DEFER_LN", "1") != "0"


def _defer_ln(leaves, w) -> bool:
    """Whether this backward parks its LayerNorm partials for the batched
    final: inside a collecting backward (linear.deferred_weight_grads), leaf
    gamma / beta of one dtype."""
    wl, bl = leaves
    return (_DEFER_LN and _LIN._ACTIVE[0] is not None and wl is not None and bl is not None and wl.is_leaf
            and bl.is_leaf and wl.dtype == bl.dtype == w.dtype and wl.requires_grad and bl.requires_grad)


# MOE_LN_POS=0: the decoder's t + pos as a separate add (A/B switch)
_LN_POS = os.environ.get("MOE_LN_POS", "1") != "0"


def add_layer_norm(a: torch.Tensor, b: torch.Tensor | None, weight: torch.Tensor, bias: torch.Tensor,
                   eps: float = 1e-5) -> torch.Tensor:
    """LayerNorm(a + b) over the last dimension (b may be None)."""
    if _fused_ok(a, b, weight, bias):
        return _AddLayerNorm.apply(a, b, weight, bias, eps)
    s = a if b is None else a + b
    return F.layer_norm(s, (a.shape[-1],), weight, bias, eps)


class AddLayerNorm(nn.LayerNorm):
    """nn.LayerNorm whose forward(a, b=None) is LayerNorm(a + b) (fused on the GPU)."""

    def with_pos(self, a: torch.Tensor, b: torch.Tensor, pos: torch.Tensor):
        """(t, t + pos) with t = LayerNorm(a + b): one launch each way on the
        GPU (_AddLayerNormPos) when the fused path applies."""
        if (_LN_POS and len(self.normalized_shape) == 1 and self.weight is not None
                and _fused_ok(a, b, self.weight, self.bias) and pos.dtype == torch.bfloat16
                and pos.shape == a.shape and pos.is_contiguous()):
            return _AddLayerNormPos.apply(a, b, self.weight, self.bias, pos, self.eps)
        t = self(a, b)
        return t, t + pos

    def forward(self, a: torch.Tensor, b: torch.Tensor | None = None) -> torch.Tensor:  # type: ignore[override]
        if len(self.normalized_shape) != 1 or self.weight is None:
            s = a if b is None else a + b
            return super().forward(s)
        return add_layer_norm(a, b, self.weight, self.bias, self.eps)
