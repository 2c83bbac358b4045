"""CPU (device='cpu') execution of the routed FFN for the C1 plumbing config.

BASELINE.json configs[0] is "CPU-only PyTorch (plumbing, no GPU)": the model
must train on CPU tensors.  This module is that device path, in plain torch
ops with autograd, split like ops.py (route+dispatch / expert FFN / combine)
so the expert-parallel composition in ep.py runs on either device.  It
implements the same semantics as the HIP kernels (include/moe_hip.h) but is
NEVER used for GPU tensors -- MoEFFN sends CUDA tensors to the HIP path, which
raises if libmoe_hip.so is missing.
"""
from __future__ import annotations

import torch
import torch.nn.functional as F


def route(x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize):
    logits = x.float() @ wg.float().t()
    if ctx_bias is not None:
        logits = logits + ctx_bias.float()[ctx_img.long()].repeat_interleave(tokens_per_image, 0)
    probs = torch.softmax(logits, dim=-1)
    lse = torch.logsumexp(logits, dim=-1)
    # stable descending sort keeps the lower expert id first on ties
    order = torch.sort(logits.detach(), dim=-1, descending=True, stable=True).indices
    idx = order[:, :k]
    psel = probs.gather(1, idx)
    w = psel / psel.sum(-1, keepdim=True) if (normalize and k > 1) else psel
    return probs, lse, idx, w


def dispatch_positions(idx, E, cap):
    """Slot-major, token-ordered rank of each assignment inside its expert."""
    T, k = idx.shape
    flat = idx.t().reshape(-1)                       # slot-major order (j, t)
    order = torch.sort(flat, stable=True).indices    # grouped by expert, stable
    hist = torch.bincount(flat, minlength=E)
    starts = torch.cumsum(hist, 0) - hist
    rank_sorted = torch.arange(flat.numel(), device=idx.device) - starts[flat[order]]
    rank = torch.empty_like(flat)
    rank[order] = rank_sorted
    rank = rank.view(k, T).t()
    kept = torch.clamp(hist, max=cap) if cap > 0 else hist
    offsets = torch.cat([kept.new_zeros(1), torch.cumsum(kept, 0)])
    pos = offsets[idx] + rank
    if cap > 0:
        pos = torch.where(rank < cap, pos, torch.full_like(pos, -1))
    return pos, hist, offsets


def route_dispatch_eager(x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize, cap):
    """-> (xp [rows, d], w [T, k], lb, z, pos [T, k], hist [E], offsets [E+1], rows)."""
    T, d = x.shape
    E = wg.shape[0]
    probs, lse, idx, w = route(x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize)
    pos, hist, offsets = dispatch_positions(idx, E, cap)
    rows = int(offsets[-1])
    keep = pos >= 0
    t_idx = torch.arange(T, device=x.device).unsqueeze(1).expand(T, k)[keep]
    xp = torch.zeros((rows, d), dtype=x.dtype, device=x.device)
    xp = xp.index_copy(0, pos[keep], x[t_idx]) if rows else xp
    f = hist.float() / float(max(T * k, 1))
    lb = E * (f * probs.mean(0)).sum()
    z = (lse ** 2).mean()
    return xp, w, lb, z, pos, hist.to(torch.int32), offsets, rows


def expert_ffn_eager(xp, w1, b1, w2, b2, offsets, grad_scale=1.0):
    if grad_scale != 1.0:  # scale the expert-weight gradients only (EP: sum over ranks -> mean)
        w1, b1, w2, b2 = (_ScaleGrad.apply(t, grad_scale) for t in (w1, b1, w2, b2))
    out = torch.zeros((xp.shape[0], w2.shape[1]), dtype=torch.float32, device=xp.device)
    G = w1.shape[0]
    off = [int(v) for v in offsets.tolist()]
    for g in range(G):
        a, b = off[g], off[g + 1]
        if b <= a:
            continue
        h = F.relu(F.linear(xp[a:b].float(), w1[g].float(), b1[g].float()))
        out = out.index_copy(0, torch.arange(a, b, device=xp.device), F.linear(h, w2[g].float(), b2[g].float()))
    return out.to(xp.dtype)


def mx_round(x: torch.Tensor) -> torch.Tensor:
    """Quantize-dequantize through MXFP8 along the last dim (OCP e4m3, one E8M0
    exponent per 32 elements; exponent rule of include/moe_hip.h), in fp32."""
    K = x.shape[-1]
    xb = x.float().reshape(*x.shape[:-1], K // 32, 32)
    amax = xb.abs().amax(-1)
    u = amax.view(torch.int32).long()
    e = ((u >> 23) & 0xFF) - 127 - 8 + ((u & 0x7FFFFF) > 0x600000).long()
    e = torch.where(amax == 0, torch.full_like(e, -127), e).clamp(-127, 127)
    sc = torch.exp2(e.float()).unsqueeze(-1)
    return ((xb / sc).to(torch.float8_e4m3fn).float() * sc).reshape(x.shape)


class _ExpertMX(torch.autograd.Function):
    """One expert's MXFP8 FFN on CPU tensors, with the HIP path's semantics
    (ops._ExpertFFNMX): e4m3 operands forward, ReLU mask from the e4m3 H,
    dgrad through the unquantized weights, weight grads on the e4m3 operands."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2):
        xq = mx_round(x)
        h = torch.relu(xq @ mx_round(w1).t() + b1.float()).to(torch.bfloat16).float()
        hq = mx_round(h)
        y = hq @ mx_round(w2).t() + b2.float()
        ctx.save_for_backward(xq, hq, w1, w2)
        return y

    @staticmethod
    def backward(ctx, dy):
        xq, hq, w1, w2 = ctx.saved_tensors
        dy = dy.float()
        dh = (dy @ w2.float()) * (hq > 0)
        return dh @ w1.float(), dh.t() @ xq, dh.sum(0), dy.t() @ hq, dy.sum(0)


def expert_ffn_mx_eager(xp, w1, b1, w2, b2, offsets, grad_scale=1.0):
    if grad_scale != 1.0:
        w1, b1, w2, b2 = (_ScaleGrad.apply(t, grad_scale) for t in (w1, b1, w2, b2))
    out = torch.zeros((xp.shape[0], w2.shape[1]), dtype=torch.float32, device=xp.device)
    off = [int(v) for v in offsets.tolist()]
    for g in range(w1.shape[0]):
        a, b = off[g], off[g + 1]
        if b > a:
            out = out.index_copy(0, torch.arange(a, b, device=xp.device),
                                 _ExpertMX.apply(xp[a:b].float(), w1[g], b1[g], w2[g], b2[g]))
    return out.to(xp.dtype)


class _ScaleGrad(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, s):
        ctx.s = s
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        return g * ctx.s, None


def combine_eager(yp, w, pos, T):
    y = torch.zeros((T, yp.shape[1]), dtype=torch.float32, device=yp.device)
    for j in range(pos.shape[1]):
        keep = pos[:, j] >= 0
        t = torch.nonzero(keep, as_tuple=True)[0]
        if t.numel():
            y = y.index_add(0, t, yp[pos[t, j]].float() * w[t, j:j + 1])
    return y


def moe_ffn_eager(x, wg, ctx_bias, w1, b1, w2, b2, ctx_img, tokens_per_image, k, normalize, cap,
                  expert_dtype="bf16"):
    T = x.shape[0]
    xp, w, lb, z, pos, hist, offsets, rows = route_dispatch_eager(x, wg, ctx_bias, ctx_img, tokens_per_image, k,
                                                                  normalize, cap)
    if expert_dtype == "fp8":
        yp = expert_ffn_mx_eager(xp, w1, b1, w2, b2, offsets)
    else:
        yp = expert_ffn_eager(xp, w1, b1, w2, b2, offsets)
    y = combine_eager(yp, w, pos, T)
    return y.to(x.dtype), lb, z, hist
