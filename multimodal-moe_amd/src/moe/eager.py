"""CPU (device='cpu') execution of the routed FFN for the C1 plumbing config.

BASELINE.json configs[0] is "CPU-only PyTorch (plumbing, no GPU)": the model
must train on CPU tensors.  This module is that device path, in plain torch
ops with autograd; it implements the same semantics as the HIP kernels
(include/moe_hip.h) but is NEVER used for GPU tensors -- MoEFFN sends CUDA
tensors to ops.moe_ffn_hip, which raises if libmoe_hip.so is missing.
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


def moe_ffn_eager(x, wg, ctx_bias, w1, b1, w2, b2, ctx_img, tokens_per_image, k, normalize, cap):
    T, d = x.shape
    E = w1.shape[0]
    probs, lse, idx, w = route(x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize)
    pos, hist, offsets = dispatch_positions(idx, E, cap)
    y = torch.zeros((T, d), dtype=torch.float32, device=x.device)
    xf = x.float()
    for e in range(E):
        sel = (idx == e) & (pos >= 0)
        t_idx, j_idx = torch.nonzero(sel, as_tuple=True)
        if t_idx.numel() == 0:
            continue
        h = F.relu(F.linear(xf[t_idx], w1[e].float(), b1[e].float()))
        ye = F.linear(h, w2[e].float(), b2[e].float())
        y = y.index_add(0, t_idx, ye * w[t_idx, j_idx].unsqueeze(1))
    f = hist.float() / float(max(T * k, 1))
    lb = E * (f * probs.mean(0)).sum()
    z = (lse ** 2).mean()
    return y.to(x.dtype), lb, z, hist.to(torch.int32)
