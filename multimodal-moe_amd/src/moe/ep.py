"""Expert parallelism (BASELINE config C4).

E experts are sharded over the W ranks of the expert-parallel group (rank r
owns experts [r*E/W, (r+1)*E/W)), every rank keeps its own tokens and
replicated router / non-expert weights (data-parallel, all-reduced by DDP or
the flat all-reduce of TrainStep).  Per MoE layer:

  route + dispatch (all E experts, local tokens)   HIP kernels / eager on CPU
  counts exchange    all_to_all of the per-expert kept counts (W x E/W ints),
                     then ONE device->host copy of the split sizes
  dispatch a2a       all_to_all_single(Xp rows, variable splits) over RCCL/xGMI
  reorder            src-major -> expert-major rows (one gather)
  expert FFN         grouped GEMMs on the E/W local experts
  reorder back, combine a2a (reverse splits), gate-weighted combine
Backward mirrors it (the a2a Function's backward is the reverse a2a); the
split sizes of the forward are reused, so the backward never syncs.
Expert-weight gradients arrive summed over all ranks' tokens; they are scaled
by 1/W to match the data-parallel mean of the replicated weights.
"""
from __future__ import annotations

import torch
import torch.distributed as dist


class _AllToAll(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, send, recv, group):
        out = x.new_empty((sum(recv),) + tuple(x.shape[1:]))
        dist.all_to_all_single(out, x.contiguous(), output_split_sizes=recv, input_split_sizes=send, group=group)
        ctx.send, ctx.recv, ctx.group = send, recv, group
        return out

    @staticmethod
    def backward(ctx, g):
        gi = g.new_empty((sum(ctx.send),) + tuple(g.shape[1:]))
        dist.all_to_all_single(gi, g.contiguous(), output_split_sizes=ctx.send, input_split_sizes=ctx.recv,
                               group=ctx.group)
        return gi, None, None, None


class _DispatchMX(torch.autograd.Function):
    """MXFP8 dispatch exchange (config C5): the e4m3 rows and their exponents
    cross the all-to-all (d + d/32 bytes per row instead of 2d) and are
    reordered expert-major; the bf16 gradient of the rows (dXp) takes the
    reverse path in backward.  ``carrier`` is the zero-stride autograd stand-in
    of the rows (ops._RouteDispatchMX)."""

    @staticmethod
    def forward(ctx, carrier, xq, xs, send, recv, perm, inv, group):
        n_send, R = sum(send), sum(recv)
        qr = xq.new_empty((R, xq.shape[1]))
        sr = xs.new_empty((R, xs.shape[1]))
        dist.all_to_all_single(qr, xq[:n_send].contiguous(), output_split_sizes=recv, input_split_sizes=send,
                               group=group)
        dist.all_to_all_single(sr, xs[:n_send].contiguous(), output_split_sizes=recv, input_split_sizes=send,
                               group=group)
        ctx.send, ctx.recv, ctx.group, ctx.rows = send, recv, group, carrier.shape[0]
        ctx.save_for_backward(inv)
        ce = torch.zeros((1, 1), dtype=carrier.dtype, device=carrier.device).expand(R, carrier.shape[1])
        ctx.mark_non_differentiable(qr, sr)
        return ce, qr.index_select(0, perm), sr.index_select(0, perm)

    @staticmethod
    def backward(ctx, g, _q, _s):
        (inv,) = ctx.saved_tensors
        gr = g.index_select(0, inv).contiguous()
        gi = g.new_zeros((ctx.rows, g.shape[1]))
        dist.all_to_all_single(gi[:sum(ctx.send)], gr, output_split_sizes=ctx.send, input_split_sizes=ctx.recv,
                               group=ctx.group)
        return gi, None, None, None, None, None, None, None


def expert_major_order(recv_mat: torch.Tensor):
    """recv_mat [W, El] (host) rows received from each source for each local
    expert, laid out source-major.  Returns (perm, offsets) with
    rows_expert_major = rows_src_major[perm] and offsets [El+1]."""
    W, El = recv_mat.shape
    cnt = recv_mat.tolist()
    start = [[0] * El for _ in range(W)]
    s = 0
    for src in range(W):
        for e in range(El):
            start[src][e] = s
            s += cnt[src][e]
    segs, offs = [], [0]
    for e in range(El):
        for src in range(W):
            if cnt[src][e]:
                segs.append(torch.arange(start[src][e], start[src][e] + cnt[src][e]))
        offs.append(offs[-1] + sum(cnt[src][e] for src in range(W)))
    perm = torch.cat(segs) if segs else torch.zeros(0, dtype=torch.int64)
    return perm, torch.tensor(offs, dtype=torch.int32)


def moe_ffn_ep(layer, x, ctx_bias, ctx_img, tokens_per_image, cap):
    cfg = layer.cfg
    E, W, k = cfg.num_experts, layer.ep_size, cfg.top_k
    El = E // W
    group = layer.ep_group
    T = x.shape[0]
    dev = x.device
    mx = x.is_cuda and cfg.expert_dtype == "fp8"
    gs = getattr(layer, "ep_grad_scale", 1.0 / W)  # 1.0 when the optimizer applies 1/W (graph-mode TrainStep)
    if mx:
        from .ops import aux_losses, combine_hip as combine, expert_ffn_mx_hip, route_dispatch_mx_hip

        xp, w, auxp, pos, hist, offsets, xq, xs, rows = route_dispatch_mx_hip(
            x, layer.wg, ctx_bias, ctx_img, tokens_per_image, k, cfg.normalize, cap)
        lb, z = aux_losses(auxp, hist, T, k)
    elif x.is_cuda:
        from .ops import aux_losses, combine_hip as combine, expert_ffn_hip as expert_ffn, route_dispatch_hip

        xp, w, auxp, pos, hist, offsets, rows = route_dispatch_hip(x, layer.wg, ctx_bias, ctx_img, tokens_per_image,
                                                                   k, cfg.normalize, cap)
        lb, z = aux_losses(auxp, hist, T, k)
    else:
        from .eager import combine_eager as combine, expert_ffn_eager, expert_ffn_mx_eager, route_dispatch_eager

        expert_ffn = expert_ffn_mx_eager if cfg.expert_dtype == "fp8" else expert_ffn_eager

        xp, w, lb, z, pos, hist, offsets, rows = route_dispatch_eager(x, layer.wg, ctx_bias, ctx_img,
                                                                      tokens_per_image, k, cfg.normalize, cap)
    kept = (offsets[1:] - offsets[:-1]).to(torch.int64).view(W, El).contiguous()
    recv_mat = torch.empty_like(kept)
    dist.all_to_all_single(recv_mat, kept, group=group)
    host = torch.cat([kept.sum(1), recv_mat.reshape(-1)]).cpu()  # the one host sync of the layer
    send = [int(v) for v in host[:W].tolist()]
    recv_h = host[W:].view(W, El)
    recv = [int(v) for v in recv_h.sum(1).tolist()]
    n_send, R = sum(send), sum(recv)

    perm, offs_l = expert_major_order(recv_h)
    perm = perm.to(dev, non_blocking=True)
    inv = torch.empty_like(perm)
    inv[perm] = torch.arange(perm.numel(), device=dev)
    offs_l = offs_l.to(dev, non_blocking=True)
    if mx:
        ce, qe, se = _DispatchMX.apply(xp, xq, xs, send, recv, perm, inv, group)
        ye = expert_ffn_mx_hip(ce, qe, se, layer.w1, layer.b1, layer.w2, layer.b2, offs_l, R, gs) if R else \
            x.new_zeros((0, x.shape[1]), dtype=torch.bfloat16)
        yr = ye.index_select(0, inv)
        yp = _AllToAll.apply(yr, recv, send, group)
        return combine(yp, w, pos, T), lb, z, hist
    xr = _AllToAll.apply(xp[:n_send], send, recv, group)
    xe = xr.index_select(0, perm)
    if x.is_cuda:
        ye = expert_ffn(xe, layer.w1, layer.b1, layer.w2, layer.b2, offs_l, R, gs) if R else \
            xe.new_zeros((0, x.shape[1]))
    else:
        ye = expert_ffn(xe, layer.w1, layer.b1, layer.w2, layer.b2, offs_l, gs)
    yr = ye.index_select(0, inv)
    yp = _AllToAll.apply(yr, recv, send, group)
    y = combine(yp, w, pos, T)
    return y, lb, z, hist
