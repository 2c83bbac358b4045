"""Expert parallelism (BASELINE config C4; SURVEY.md 8(e), 2.2 M9, 7 "EP needs
per-step variable splits").

E experts are sharded over the W ranks of the expert-parallel group (rank r
owns experts [r*E/W, (r+1)*E/W)), every rank keeps its own tokens and
replicated router / non-expert weights (data-parallel, all-reduced by DDP or
the flat all-reduce of TrainStep).

The exchange is FIXED-CAPACITY: every (source rank, expert) pair owns S rows
of the all-to-all buffers (S = ``MoEConfig.ep_slot_rows(T)``: the layer's
capacity when it has one, else ceil(f T k / E) with f = ep_capacity_factor,
2.0 by default (every all-to-all then carries 2x the mean rows), or T --
lossless, the worst case -- with ``-epcf0``), so every split size is
static and nothing about the routing is read on the host.  Per MoE layer:

  route + dispatch      router + scan + permute into the padded send layout:
                        expert e's kept rows at [e S, e S + min(hist_e, S));
                        assignments ranked >= S are dropped exactly like
                        capacity drops (for capacity layers S IS the capacity,
                        so nothing changes)
  counts exchange       all_to_all of the kept counts [W, E/W] (device ints)
  dispatch a2a          all_to_all_single of the [E S, d] rows, equal splits
  compaction map        on the device from the received counts, ONE HIP
                        launch (moe_ep_compaction): compact expert-major row
                        -> received row (``gather``), the local expert offsets
                        and this rank's overflow count
  expert FFN            the fused expert FFN reads the received rows through
                        ``gather`` (no compaction copy) and writes each output
                        row straight back to its received row (no row-gather
                        pass); the backward's dXp lands the same way
                        (torch index maps + two-launch GEMMs remain for the
                        MXFP8 experts and the CPU path)
  combine a2a           the reverse all_to_all_single, then the gate-weighted
                        combine at the padded positions
Backward mirrors it; the transposes of the two row maps are the maps
themselves (bijections on the valid rows; padding rows are never read).
With no host sync and static shapes the layer captures into a hipGraph.
W = 1 (``-ep1``) runs the same code with identity exchanges.
Expert-weight gradients arrive summed over all ranks' tokens; they are scaled
by 1/W (``ep_grad_scale``) to match the data-parallel mean of the replicated
weights.  Assignments beyond S when the layer has no capacity are counted in
``layer.last_ep_overflow`` (device scalar; 0 means the result equals the
single-process layer).
"""
from __future__ import annotations

import torch
import torch.distributed as dist

from .ops import _bias


def _a2a(out, x, group, W):
    if W == 1 and group is None:  # -ep1 without a process group: identity exchange
        out.copy_(x)
    elif x.is_cuda and dist.get_backend(group) == "gloo":
        # gloo moves host memory only (several ranks sharing one GPU in the
        # multi-rank tests): stage through the host; not graph-capturable
        xs = x.detach().contiguous().cpu()
        if xs.dtype in (torch.bfloat16, torch.float16):  # gloo has no 16-bit a2a: widen (exact) and narrow back
            xs = xs.float()
        o = torch.empty(xs.shape, dtype=xs.dtype)
        dist.all_to_all_single(o, xs, group=group)
        out.copy_(o.to(out.device))
    else:
        dist.all_to_all_single(out, x.contiguous(), group=group)
    return out


class _Exchange(torch.autograd.Function):
    """Equal-split all_to_all_single of [W * n, ...] rows; its transpose is
    itself."""

    @staticmethod
    def forward(ctx, x, group, W):
        ctx.group, ctx.W = group, W
        return _a2a(torch.empty_like(x), x, group, W)

    @staticmethod
    def backward(ctx, g):
        return _a2a(torch.empty_like(g), g, ctx.group, ctx.W), None, None


class _RowMap(torch.autograd.Function):
    """out = x[fwd]; backward dx = dout[bwd].  fwd and bwd are mutually inverse
    on the valid rows; padding rows carry don't-care values both ways (a
    scatter-add transpose would fold them into row 0)."""

    @staticmethod
    def forward(ctx, x, fwd, bwd):
        ctx.save_for_backward(bwd)
        return x.index_select(0, fwd)

    @staticmethod
    def backward(ctx, g):
        (bwd,) = ctx.saved_tensors
        return g.index_select(0, bwd), None, None


def compaction_map(recv_cnt: torch.Tensor, S: int):
    """recv_cnt [W, El] rows received from each source for each local expert,
    held at received row (src El + e) S + j, j < recv_cnt[src, e].
    Returns (gather int32 [W El S]: compact expert-major row -> received row,
    inv int64 [W El S]: received row -> compact row (0 for padding),
    offsets int32 [El + 1]); static shapes, device ops only."""
    W, El = recv_cnt.shape
    dev = recv_cnt.device
    cnt = recv_cnt.to(torch.int64)
    per_e = cnt.sum(0)
    offs = torch.zeros(El + 1, dtype=torch.int64, device=dev)
    offs[1:] = torch.cumsum(per_e, 0)
    start = offs[:-1].unsqueeze(0) + torch.cumsum(cnt, 0) - cnt          # [W, El]
    j = torch.arange(S, device=dev)
    valid = j.view(1, 1, S) < cnt.unsqueeze(-1)                          # [W, El, S]
    comp = start.unsqueeze(-1) + j.view(1, 1, S)
    R = W * El * S
    dst = torch.where(valid, comp, torch.full_like(comp, R)).reshape(-1)
    gather = torch.zeros(R + 1, dtype=torch.int64, device=dev)
    gather.scatter_(0, dst, torch.arange(R, device=dev))
    inv = torch.where(valid, comp, torch.zeros_like(comp)).reshape(-1)
    return gather[:R].to(torch.int32).contiguous(), inv.contiguous(), offs.to(torch.int32).contiguous()


def _exchange_counts(kept, group, W):
    """kept [W, El] rows this rank sends to each (peer, expert) -> what it
    receives, device-resident."""
    kept = kept.to(torch.int64).contiguous()
    return _a2a(torch.empty_like(kept), kept, group, W)


class _EPExpertFFN(torch.autograd.Function):
    """The local experts over the received rows, in the received layout.
    Forward: GEMM1 gathers xr[gather] (+b1, ReLU), GEMM2 (+b2), then the
    output rows are put back at their received positions (row gather by inv).
    Backward: the first paired launch reads dYp = dyr[gather] inside the
    GEMMs, the second gathers xr[gather] for dW1; dxr = dXp[inv]."""

    @staticmethod
    def forward(ctx, xr, gather, inv, w1, b1, w2, b2, offsets, grad_scale):
        from . import _lib as L

        G, F, d = w1.shape
        R = xr.shape[0]
        xb = xr.to(torch.bfloat16).contiguous()
        w1b = w1.to(torch.bfloat16).contiguous()
        w2b = w2.to(torch.bfloat16).contiguous()
        h = L.grouped_gemm_gather(xb, gather, w1b, offsets, G, R, F, d, 1, L.EPI_BIAS_RELU, bias=_bias(b1))
        ye = L.grouped_gemm(h, w2b, offsets, G, R, d, F, 1, L.EPI_BIAS, bias=_bias(b2))
        ctx.save_for_backward(xb, gather, inv, h, w1b, w2b, offsets)
        ctx.meta = (G, R, float(grad_scale), xr.dtype)
        ctx.wdtype = w1.dtype if (w1.dtype == b1.dtype == w2.dtype == b2.dtype) else torch.float32
        return ye.index_select(0, inv)

    @staticmethod
    def backward(ctx, dyr):
        from . import _lib as L

        xb, gather, inv, h, w1b, w2b, offsets = ctx.saved_tensors
        G, R, s, xdtype = ctx.meta
        F, d = w1b.shape[1], w1b.shape[2]
        odt = torch.bfloat16 if ctx.wdtype == torch.bfloat16 else torch.float32
        dyb = dyr.to(torch.bfloat16).contiguous()
        dh, dW2, db2 = L.grouped_gemm_bwd_pair(dyb, w2b, offsets, G, R, F, d, L.EPI_RELU_MASK, h, dyb, h,
                                               out_dtype=odt, a_gather=gather, wx_gather=gather)
        dxe, dW1, db1 = L.grouped_gemm_bwd_pair(dh, w1b, offsets, G, R, d, F, L.EPI_NONE, None, dh, xb, gather,
                                                out_dtype=odt)
        if s != 1.0:
            for t in (dW1, db1, dW2, db2):
                t.mul_(s)
        return dxe.index_select(0, inv).to(xdtype), None, None, dW1, db1, dW2, db2, None, None


class _EPExpertFFNScatter(torch.autograd.Function):
    """The local experts over the received rows, in the received layout, with
    no row-gather passes: the fused expert FFN (moe_expert_ffn_fwd) -- or, at
    few rows per expert, GEMM1 gathering + GEMM2 scattering
    (moe_grouped_gemm_scatter) -- reads received row gather[r] for compact
    row r and writes its output row back to received row gather[r]; the backward's first paired launch reads dYp =
    dyr[gather] inside the GEMMs, the second gathers xr[gather] for dW1 and
    stores dXp row r at received row gather[r] (moe_grouped_gemm_bwd_pair_
    scatter).  Received rows no expert row maps to (the slots' padding) are
    left uninitialised both ways: no one reads them (the sender's combine and
    token backward read kept positions only)."""

    @staticmethod
    def forward(ctx, xr, gather, w1, b1, w2, b2, offsets, grad_scale, fused=True, rows=None):
        from . import _lib as L
        from .ops import _bias

        G, F, d = w1.shape
        Rn = xr.shape[0]  # received layout rows (W El S)
        R = Rn if rows is None else min(int(rows), Rn)  # compact row bound
        xb = xr.to(torch.bfloat16).contiguous()
        w1b = w1.to(torch.bfloat16).contiguous()
        w2b = w2.to(torch.bfloat16).contiguous()
        if fused:
            h, yr = L.expert_ffn_fwd(xb, gather, w1b, _bias(b1), w2b, _bias(b2), offsets, G, R, yp_rows=gather,
                                     yp_n=Rn)
        else:  # few rows per expert: two launches (the fused FFN streams every expert's weights per row tile)
            h = L.grouped_gemm_gather(xb, gather, w1b, offsets, G, R, F, d, 1, L.EPI_BIAS_RELU, bias=_bias(b1))
            yr = L.grouped_gemm_scatter(h, w2b, offsets, G, R, d, F, 1, L.EPI_BIAS, gather,
                                        torch.empty((Rn, d), dtype=torch.bfloat16, device=xb.device), bias=_bias(b2))
        ctx.save_for_backward(xb, gather, h, w1b, w2b, offsets)
        ctx.meta = (G, R, Rn, float(grad_scale), xr.dtype)
        ctx.wdtype = w1.dtype if (w1.dtype == b1.dtype == w2.dtype == b2.dtype) else torch.float32
        return yr

    @staticmethod
    def backward(ctx, dyr):
        from . import _lib as L

        xb, gather, h, w1b, w2b, offsets = ctx.saved_tensors
        G, R, Rn, s, xdtype = ctx.meta
        F, d = w1b.shape[1], w1b.shape[2]
        odt = torch.bfloat16 if ctx.wdtype == torch.bfloat16 else torch.float32
        dyb = dyr.to(torch.bfloat16).contiguous()
        dh, dW2, db2 = L.grouped_gemm_bwd_pair(dyb, w2b, offsets, G, R, F, d, L.EPI_RELU_MASK, h, dyb, h,
                                               out_dtype=odt, a_gather=gather, wx_gather=gather)
        dxr, dW1, db1 = L.grouped_gemm_bwd_pair(dh, w1b, offsets, G, R, d, F, L.EPI_NONE, None, dh, xb, gather,
                                                out_dtype=odt, c_rows=gather, c_n=Rn)
        if s != 1.0:
            for t in (dW1, db1, dW2, db2):
                t.mul_(s)
        return dxr.to(xdtype), None, dW1, db1, dW2, db2, None, None, None, None


def _fused_ep_ok(layer, x, fp8):
    """The HIP receive path (moe_ep_compaction + the scattering fused FFN):
    bf16 experts of a shape the fused FFN takes (ops.MOE_FUSED_FFN on)."""
    if not x.is_cuda or fp8:
        return False
    from . import _lib as L
    from .ops import _FUSED_FFN, _bias

    G, F, d = layer.w1.shape
    # the fused FFN reads both biases in one dtype (ops._ffn_forward's rule);
    # mixed fp32 / bf16 biases take the grouped-GEMM gather / scatter branch
    same = _bias(layer.b1).dtype == _bias(layer.b2).dtype
    return _FUSED_FFN and same and L.expert_ffn_supported(G, F, d)


class _CarrierExchange(torch.autograd.Function):
    """MXFP8 path: the routed rows cross as e4m3 + exponents (non-differentiable
    uint8); this node stands for them in the autograd graph.  Forward: a
    zero-stride bf16 carrier of the compact rows; backward: the compact dXp is
    put back in the received layout (inv), then sent home by the reverse
    exchange as the gradient of the sender's padded carrier."""

    @staticmethod
    def forward(ctx, carrier, inv, group, W):
        ctx.save_for_backward(inv)
        ctx.group, ctx.W = group, W
        return torch.zeros((1, 1), dtype=carrier.dtype, device=carrier.device).expand(inv.shape[0],
                                                                                      carrier.shape[1])

    @staticmethod
    def backward(ctx, g):
        (inv,) = ctx.saved_tensors
        gr = g.index_select(0, inv).contiguous()
        return _a2a(torch.empty_like(gr), gr, ctx.group, ctx.W), None, None, None


def _padded_positions(idx, E, S):
    """CPU dispatch into the fixed-capacity layout: pos = e S + rank (slot-major,
    token-ordered rank inside expert e, as eager.dispatch_positions), -1 when
    rank >= S; and the full histogram."""
    T, k = idx.shape
    flat = idx.t().reshape(-1)
    order = torch.sort(flat, stable=True).indices
    hist = torch.bincount(flat, minlength=E)
    starts = torch.cumsum(hist, 0) - hist
    rank_sorted = torch.arange(flat.numel(), device=idx.device) - starts[flat[order]]
    rank = torch.empty_like(flat)
    rank[order] = rank_sorted
    rank = rank.view(k, T).t()
    pos = torch.where(rank < S, idx * S + rank, torch.full_like(rank, -1))
    return pos, hist


def _route_padded_eager(x, wg, ctx_bias, ctx_img, tpi, k, normalize, S):
    from .eager import route

    T, d = x.shape
    E = wg.shape[0]
    probs, lse, idx, w = route(x, wg, ctx_bias, ctx_img, tpi, k, normalize)
    pos, hist = _padded_positions(idx, E, S)
    keep = pos >= 0
    t_idx = torch.arange(T, device=x.device).unsqueeze(1).expand(T, k)[keep]
    xp = torch.zeros((E * S, d), dtype=x.dtype, device=x.device).index_copy(0, pos[keep], x[t_idx])
    f = hist.float() / float(max(T * k, 1))
    lb = E * (f * probs.mean(0)).sum()
    z = (lse ** 2).mean()
    return xp, w, lb, z, pos, hist.to(torch.int32)


def moe_ffn_ep(layer, x, ctx_bias, ctx_img, tokens_per_image, cap, residual=False, aux_coefs=None):
    """-> (y [T, d], lb, z, hist [E]) of one expert-parallel MoE layer;
    residual=True: y = x + FFN(x), on the HIP bf16 path folded into the
    combine (returned with ``y_has_residual`` set on the layer).
    aux_coefs=(lb_coef, z_coef) on the GPU: lb and z come back detached and
    ``layer.ep_aux_weighted`` holds the differentiable lb_coef lb + z_coef z
    from the fused aux-loss kernel (MoEFFN; one launch each way)."""
    layer.ep_aux_weighted = None
    layer.y_has_residual = False
    cfg = layer.cfg
    E, W, k = cfg.num_experts, layer.ep_size, cfg.top_k
    El = E // W
    group = layer.ep_group
    T, d = x.shape
    S = cfg.ep_slot_rows(T, d)
    if cap > 0 and S != cap:
        raise ValueError(f"EP slot rows {S} must equal the layer capacity {cap}")
    fp8 = cfg.expert_dtype == "fp8"
    gs = getattr(layer, "ep_grad_scale", 1.0 / W)  # 1.0 when the optimizer applies 1/W (graph-mode TrainStep)
    if x.is_cuda:
        from . import _lib as L
        from .ops import aux_loss_weighted, aux_losses_hip, combine_hip as combine
        from .ops import expert_ffn_mx_hip, route_dispatch_hip, route_dispatch_mx_hip

        if fp8:
            carrier, w, auxp, pos, hist, _, xq, xs, _ = route_dispatch_mx_hip(
                x, layer.wg, ctx_bias, ctx_img, tokens_per_image, k, cfg.normalize, cap, pad=S)
        else:
            xp, w, auxp, pos, hist, _, _ = route_dispatch_hip(x, layer.wg, ctx_bias, ctx_img, tokens_per_image, k,
                                                              cfg.normalize, cap, pad=S)
        # lb and z from the single-GPU path's aux-loss kernel: one HIP launch each
        # way instead of ~20 torch ops (differentiable, or the weighted sum when
        # the caller passes its coefficients)
        if aux_coefs is not None:
            layer.ep_aux_weighted, raw = aux_loss_weighted(auxp, hist, T, k, *aux_coefs)
            lb, z = raw[0], raw[1]
        else:
            lb, z = aux_losses_hip(auxp, hist, T, k)
    else:
        from .eager import combine_eager as combine, expert_ffn_eager, expert_ffn_mx_eager

        xp, w, lb, z, pos, hist = _route_padded_eager(x, layer.wg, ctx_bias, ctx_img, tokens_per_image, k,
                                                      cfg.normalize, S)
    if _fused_ep_ok(layer, x, fp8):
        # counts exchange (int32; the compaction caps them at S), then the
        # receive map, the local expert offsets and this rank's overflow in ONE
        # launch (moe_ep_compaction).  -ep1 without a process group: the
        # exchanges are identities and are skipped (no copies)
        ident = W == 1 and group is None
        sent = hist.view(W, El)
        recv_cnt = sent if ident else _a2a(torch.empty_like(sent), sent.contiguous(), group, W)
        gather, offs, overflow = L.ep_compaction(recv_cnt, hist, S)
        layer.last_ep_overflow = overflow[0] if cap <= 0 else None
        xr = xp if ident else _Exchange.apply(xp, group, W)
        # the one-launch FFN where each local expert receives enough rows (the
        # single-GPU path's threshold, ops._FUSED_MIN_ROWS), else two launches
        from .ops import _FUSED_MIN_ROWS
        fused = T * k * W >= _FUSED_MIN_ROWS * E
        # compact rows: every source sends at most T k rows (equal T on every
        # rank: static shapes), so the GEMM grids and H need min(W El S, W T k)
        rows = min(W * El * S, W * T * k)
        yr = _EPExpertFFNScatter.apply(xr, gather, layer.w1, layer.b1, layer.w2, layer.b2, offs, gs, fused, rows)
        yp = yr if ident else _Exchange.apply(yr, group, W)
        if residual and x.dtype == torch.bfloat16:
            layer.y_has_residual = True
            return combine(yp, w, pos, T, resid=x), lb, z, hist
        return combine(yp, w, pos, T), lb, z, hist
    recv_cnt = _exchange_counts(hist.clamp(max=S).view(W, El), group, W)
    gather, inv, offs = compaction_map(recv_cnt, S)
    layer.last_ep_overflow = (hist.to(torch.int64) - S).clamp(min=0).sum() if cap <= 0 else None
    if x.is_cuda and fp8:
        qr = _a2a(torch.empty_like(xq), xq, group, W)
        sr = _a2a(torch.empty_like(xs), xs, group, W)
        ce = _CarrierExchange.apply(carrier, inv, group, W)
        ye = expert_ffn_mx_hip(ce, qr.index_select(0, gather), sr.index_select(0, gather), layer.w1, layer.b1,
                               layer.w2, layer.b2, offs, W * El * S, gs)
        yr = _RowMap.apply(ye, inv, gather)
    elif x.is_cuda:
        xr = _Exchange.apply(xp, group, W)
        yr = _EPExpertFFN.apply(xr, gather, inv, layer.w1, layer.b1, layer.w2, layer.b2, offs, gs)
    else:
        xr = _Exchange.apply(xp, group, W)
        xe = _RowMap.apply(xr, gather, inv)
        ffn = expert_ffn_mx_eager if fp8 else expert_ffn_eager
        ye = ffn(xe, layer.w1, layer.b1, layer.w2, layer.b2, offs, gs)
        yr = _RowMap.apply(ye, inv, gather)
    yp = _Exchange.apply(yr, group, W)
    return combine(yp, w, pos, T), lb, z, hist
