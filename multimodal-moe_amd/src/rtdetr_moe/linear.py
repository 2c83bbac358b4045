"""Linear layer for inputs with a very large row count (the decoder's value
projection over all B*S encoder-memory tokens: 154,560 rows at 1280x736,
batch 8).

The weight gradient dW = dY^T X reduces over all rows.  As one GEMM with a
256x256 output, hipBLASLt picks a tiling that puts only 16 workgroups on the
chip (~380 us on MI355X); split into S row chunks as a batched GEMM
(S independent [256, K/S] x [K/S, 256] products, then a fp32 sum over S) it
fills the chip (~50 us, tools/mm_probe.py).  Forward and input gradient are
the usual GEMMs.  Every linear layer of the RT-DETR body is a TokenLinear on
the GPU: its bias gradient comes from rtdetr_bias_grad (deterministic
two-launch column sum) instead of torch's reduce kernel.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F
from torch import nn

BIG_ROWS = 65536  # below this, the plain GEMM is already well shaped
DENSE_WGRAD_ROWS = [512]  # from this many rows, conforming shapes use libmoe_hip's wgrad (list: A/B switch)


def chunked_wgrad(gy: torch.Tensor, x: torch.Tensor, target_chunk: int = 2560) -> torch.Tensor:
    """sum_r gy[r, :]^T x[r, :] -> fp32 [m, n] as a batched GEMM over row chunks."""
    K, m = gy.shape
    n = x.shape[1]
    S = max(1, min(256, K // target_chunk))
    kc = K // S
    head = S * kc
    out = torch.bmm(gy[:head].view(S, kc, m).transpose(1, 2), x[:head].view(S, kc, n)).sum(0, dtype=torch.float32)
    if head < K:
        out += gy[head:].t().float().mm(x[head:].float())
    return out


def bias_grad(g2: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Column sum of the bf16 output gradient [M, N] in the bias dtype: the HIP
    kernel pair rtdetr_bias_grad (fixed-order fp32 accumulation, two launches)
    on bf16 CUDA gradients; torch's sum elsewhere (fp32 layers)."""
    M, N = g2.shape
    if not (g2.is_cuda and g2.dtype == torch.bfloat16 and dtype in (torch.bfloat16, torch.float32)
            and M > 0 and (N % 8 == 0 and N <= 2048 or N <= 256)):
        return g2.sum(0, dtype=torch.float32).to(dtype)
    from ..moe import _lib as L

    if N % 8 == 0 and g2.data_ptr() % 16 != 0:
        g2 = g2.clone()  # 16-B row vectors
    lib = L.lib()
    P = int(lib.rtdetr_bias_grad_parts(M, N))
    parts = torch.empty((P, N), dtype=torch.float32, device=g2.device)
    out = torch.empty((N,), dtype=dtype, device=g2.device)
    L._check(lib.rtdetr_bias_grad(g2.data_ptr(), M, N, parts.data_ptr(), P, out.data_ptr(),
                                  int(dtype == torch.bfloat16), L._stream()), "rtdetr_bias_grad")
    return out


class _TokenLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, dtype):
        xc, wc = x.to(dtype), weight.to(dtype)
        bc = bias.to(dtype) if bias is not None else None
        ctx.save_for_backward(xc, wc)
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.weight_dtype = weight.dtype
        return F.linear(xc, wc, bc)

    @staticmethod
    def backward(ctx, gy):
        xc, wc = ctx.saved_tensors
        g2 = gy.reshape(-1, gy.shape[-1]).to(wc.dtype).contiguous()
        x2 = xc.reshape(-1, xc.shape[-1])
        gx = g2.mm(wc).view(xc.shape) if ctx.needs_input_grad[0] else None
        gw = gb = None
        K, M = g2.shape
        N = x2.shape[1]
        if (ctx.needs_input_grad[1] and ctx.has_bias and ctx.needs_input_grad[2] and g2.is_cuda
                and g2.dtype == x2.dtype == torch.bfloat16 and M % 64 == 0 and N % 128 == 0
                and DENSE_WGRAD_ROWS[0] <= K < BIG_ROWS and x2.is_contiguous()):
            # weight + bias gradient in one libmoe_hip launch (split over rows):
            # hipBLASLt's dY^T X on these few-tile outputs plus the bias column
            # sum took ~31 us at 2,400 rows, this ~14 us (tools/mm_probe_small.py)
            from ..moe import _lib as L

            odt = torch.bfloat16 if ctx.weight_dtype == torch.bfloat16 else torch.float32
            gw, gb = L.linear_wgrad(g2, x2, odt)
            return gx, gw, gb.to(ctx.bias_dtype), None
        if ctx.needs_input_grad[1]:
            gw = chunked_wgrad(g2, x2) if x2.shape[0] >= BIG_ROWS else g2.t().mm(x2)
        gb = bias_grad(g2, ctx.bias_dtype) if ctx.has_bias and ctx.needs_input_grad[2] else None
        return gx, gw, gb, None


class TokenLinear(nn.Linear):
    """nn.Linear (same parameters and state dict) whose backward splits the
    weight-gradient reduction over row chunks when the input has many rows and
    takes the bias gradient from the HIP column-sum kernels (bias_grad)."""

    def forward(self, x):
        if x.is_cuda and x.numel() > 0:
            dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
            with torch.autocast("cuda", enabled=False):
                return _TokenLinear.apply(x, self.weight, self.bias, dtype)
        return super().forward(x)


class TokenSelfAttention(nn.Module):
    """Self-attention with nn.MultiheadAttention(batch_first=True)'s parameters
    and state-dict keys (in_proj_weight [3d, d], in_proj_bias, out_proj), for
    the RT-DETR layers' q = k = x + pos, v = x pattern: q and k come from ONE
    [d -> 2d] GEMM on x + pos and v from one [d -> d] GEMM on x (MHA's packed
    path needs q, k and v from one tensor and otherwise issues three), every
    projection through TokenLinear's backward (fused weight + bias gradient),
    then scaled-dot-product attention and the output projection.  Same math as
    nn.MultiheadAttention (dropout 0)."""

    def __init__(self, d: int, nhead: int):
        super().__init__()
        self.embed_dim, self.num_heads = d, nhead
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * d))
        self.out_proj = TokenLinear(d, d)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.in_proj_bias)
        nn.init.zeros_(self.out_proj.bias)

    def _proj(self, x, lo, hi):
        w, b = self.in_proj_weight[lo:hi], self.in_proj_bias[lo:hi]
        if x.is_cuda and x.numel() > 0:
            dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
            with torch.autocast("cuda", enabled=False):
                return _TokenLinear.apply(x, w, b, dtype)
        return F.linear(x, w, b)

    def forward(self, qk_in: torch.Tensor, v_in: torch.Tensor) -> torch.Tensor:
        """qk_in = x + pos, v_in = x, both [B, L, d] -> [B, L, d]."""
        B, L, d = qk_in.shape
        H = self.num_heads
        qk = self._proj(qk_in, 0, 2 * d)
        v = self._proj(v_in, 2 * d, 3 * d)
        q, k = qk.split(d, -1)
        heads = lambda t: t.reshape(B, L, H, d // H).transpose(1, 2)  # noqa: E731
        o = F.scaled_dot_product_attention(heads(q), heads(k), heads(v))
        return self.out_proj(o.transpose(1, 2).reshape(B, L, d))
