"""autograd wrappers of the HIP MoE FFN.

Single-GPU bf16 layers run as ONE autograd node, _MoELayer (8 HIP launches
forward + backward, see its docstring).  The building blocks below remain
for the MXFP8 (C5) and expert-parallel (C4) compositions:
  _RouteIndex     router + top-k + aux partials (K1), then route_dispatch: the
                  scan, K2's index half (pos and the row -> token map; the
                  routed rows are never copied) and the aux losses, one launch
                  backward: token_bwd (dispatch transpose + router backward)
  _ExpertFFNGather the expert FFN forward reading the token rows through the
                  row map: ONE moe_expert_ffn_fwd launch (GEMM1 +b1, ReLU,
                  H written once, GEMM2 +b2 on H still in registers), or
                  GEMM1 and GEMM2 as two grouped GEMMs (MOE_FUSED_FFN=0)
                  backward: up to 1,024 rows per expert (the decoder)
                  moe_expert_ffn_bwd -- dH = dgrad (ReLU mask), then {dW2 +
                  db2, dW1 + db1, dXp} in ONE grid --; above (the encoder)
                  two paired launches (moe_grouped_gemm_bwd_pair): {dH, dW2 +
                  db2} and {dXp = dgrad, dW1 + db1 with the token rows gathered}
  _Combine        gate-weighted combine (K3); backward: combine_bwd
Single GPU (_MoELayer): 4 launches forward (router, route_dispatch, the fused
expert FFN -- or GEMM1 + GEMM2 below 1,536 rows per expert --, combine with
the residual), 4 backward (the expert FFN backward in two launches with the
combine transpose folded in, token_bwd, router_wgrad: dWg and the
context-bias gradient in one launch).  The
expert-parallel path (ep.py) moves real rows through its all-to-alls and runs
_RouteDispatch (permute) + _ExpertFFN (rows in, same paired backward).  Nothing is synchronised with the host: expert
offsets stay on the device, grids are sized from host upper bounds, and the
aux-loss gradients reach the router kernel as device tensors.

Aux losses (row a3), from the router's per-block partials ``auxp``
[nblk, E+1] (column sums of probs, and of lse^2):
  lb = E * sum_e f_e * P_e,  f = hist / (T k),  P = colsum(auxp[:, :E]) / T
  z  = colsum(auxp[:, E]) / T
Their gradient w.r.t. ``auxp`` is uniform over blocks, so _RouteDispatch's
backward reads row 0: dprob_bias = d_auxp[0, :E], z-loss scale = 2 d_auxp[0, E].
"""
from __future__ import annotations

import os

import torch

from . import _lib as L


def _bias(b):
    """A grouped-GEMM bias operand: bf16 parameters as they are (MOE_BIAS_BF16:
    the kernel widens them), anything else as fp32."""
    return b.contiguous() if b.dtype == torch.bfloat16 else b.float().contiguous()


# MOE_FUSED_FFN=0: the expert FFN forward as two grouped GEMMs (A/B switch)
_FUSED_FFN = os.environ.get("MOE_FUSED_FFN", "1") != "0"
# MOE_FFN_BWD2=0: the single-GPU expert FFN backward as the two paired launches
# {dH, dW2}, {dXp, dW1} instead of moe_expert_ffn_bwd's dH, {dXp, dW2, dW1} (A/B)
_FFN_BWD2 = os.environ.get("MOE_FFN_BWD2", "1") != "0"
_FUSED_MIN_ROWS = int(os.environ.get("MOE_FUSED_FFN_MIN_ROWS", "1536"))


def _ffn_forward(xb, tok, w1b, b1, w2b, b2, offsets, G, rows):
    """(h, yp) of the expert FFN forward: ONE moe_expert_ffn_fwd launch (H
    written once, never read back) when the shape allows it, else GEMM1
    (gathering token rows when ``tok`` is given) and GEMM2 as two launches."""
    F, d = w1b.shape[1], w1b.shape[2]
    bb1, bb2 = _bias(b1), _bias(b2)
    # fused only for >= 1,536 rows per expert on average: every workgroup streams its expert's whole
    # W1 and W2, so at the C2 decoder's 600 rows / expert the one-round grid is latency-bound (kbench
    # cold, profiles/r04/kbench: decoder 41.0 us fused vs 11.8 + 14.1 us; encoder 45.6 vs 25.9 + 21.5)
    if (_FUSED_FFN and bb1.dtype == bb2.dtype and L.expert_ffn_supported(G, F, d)
            and rows >= _FUSED_MIN_ROWS * G):
        return L.expert_ffn_fwd(xb, tok, w1b, bb1, w2b, bb2, offsets, G, rows)
    if tok is not None:
        h = L.grouped_gemm_gather(xb, tok, w1b, offsets, G, rows, F, d, 1, L.EPI_BIAS_RELU, bias=bb1)
    else:
        h = L.grouped_gemm(xb, w1b, offsets, G, rows, F, d, 1, L.EPI_BIAS_RELU, bias=bb1)
    yp = L.grouped_gemm(h, w2b, offsets, G, rows, d, F, 1, L.EPI_BIAS, bias=bb2)
    return h, yp


_PADDED_OFFSETS: dict = {}


def _padded_offsets(E, pad, device):
    """Expert e's rows start at e * pad (the fixed-capacity layout of ep.py);
    cached per (E, pad, device): read-only, so no launches per layer call."""
    key = (int(E), int(pad), str(device))
    t = _PADDED_OFFSETS.get(key)
    if t is None:
        t = _PADDED_OFFSETS[key] = (torch.arange(E + 1, dtype=torch.int32, device=device) * int(pad)).contiguous()
    return t


class _RouteDispatch(torch.autograd.Function):
    """Router + scan + permute (rows copied).  ``pad`` > 0: the fixed-capacity
    layout of the expert-parallel send buffer -- expert e's kept rows at
    [e pad, e pad + min(hist_e, pad)), assignments ranked >= pad dropped."""

    @staticmethod
    def forward(ctx, x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize, cap, rows, pad=0):
        T, d = x.shape
        E = wg.shape[0]
        xb = x.to(torch.bfloat16).contiguous()
        wg32 = wg.float().contiguous()
        cb = ctx_bias.float().contiguous() if ctx_bias is not None else None
        idx, w, probs, lse, lrank, bcnt, auxp = L.router_topk_fwd(xb, wg32, cb, ctx_img, tokens_per_image, k,
                                                                   normalize)
        rank_base, hist, offsets = L.route_scan(bcnt, cap)
        if pad:
            offsets, cap = _padded_offsets(E, pad, x.device), pad
        xp, pos = L.permute_fwd(xb, idx, lrank, rank_base, offsets, E, cap, rows)
        ctx.save_for_backward(xb, wg32, idx, w, probs, lse, pos,
                              ctx_img if ctx_img is not None else torch.empty(0))
        ctx.meta = (T, d, E, int(normalize), tokens_per_image, cb is not None, x.dtype,
                    ctx_bias.shape[0] if ctx_bias is not None else 0)
        ctx.mark_non_differentiable(pos, hist, offsets)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the index outputs
        return xp, w, auxp, pos, hist, offsets

    @staticmethod
    def backward(ctx, d_xp, d_w, d_auxp, _p, _h, _o):
        xb, wg32, idx, w, probs, lse, pos, ctx_img = ctx.saved_tensors
        T, d, E, normalize, tpi, has_ctx, xdtype, C = ctx.meta
        dev = xb.device
        if d_xp is None:
            d_xp = torch.zeros((1, d), dtype=torch.bfloat16, device=dev)
            pos_use = torch.full_like(pos, -1)
        else:
            d_xp = d_xp.to(torch.bfloat16).contiguous()
            pos_use = pos
        d_w = torch.zeros_like(w) if d_w is None else d_w.float().contiguous()
        if d_auxp is not None:
            dprob_bias = d_auxp[0, :E].float().contiguous()
            zc = (2.0 * d_auxp[0, E:E + 1]).float().contiguous()
        else:
            dprob_bias, zc = None, None
        dx, dlogits = L.token_bwd(d_xp, pos_use, probs, idx, w, d_w, lse, dprob_bias, zc, wg32, normalize)
        # router weight + context-bias gradients: one HIP launch, fixed-order sums
        dwg, dcb = L.router_wgrad(dlogits, xb, ctx_img if has_ctx else None, tpi, C if has_ctx else 0)
        return dx.to(xdtype), dwg, dcb, None, None, None, None, None, None, None


class _RouteDispatchMX(torch.autograd.Function):
    """_RouteDispatch with the MXFP8 permute (config C5): the routed rows leave
    as e4m3 ``xq`` + E8M0 ``xs`` (non-differentiable), and a zero-stride bf16
    ``carrier`` [rows, d] stands for the permuted rows in the autograd graph so
    that dXp (from _ExpertFFNMX.backward) reaches the dispatch transpose."""

    @staticmethod
    def forward(ctx, x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize, cap, rows, pad=0):
        T, d = x.shape
        E = wg.shape[0]
        xb = x.to(torch.bfloat16).contiguous()
        wg32 = wg.float().contiguous()
        cb = ctx_bias.float().contiguous() if ctx_bias is not None else None
        idx, w, probs, lse, lrank, bcnt, auxp = L.router_topk_fwd(xb, wg32, cb, ctx_img, tokens_per_image, k,
                                                                   normalize)
        rank_base, hist, offsets = L.route_scan(bcnt, cap)
        if pad:
            offsets, cap = _padded_offsets(E, pad, x.device), pad
        xq, xs, pos = L.permute_fwd_mx(xb, idx, lrank, rank_base, offsets, E, cap, rows)
        carrier = torch.zeros((1, 1), dtype=torch.bfloat16, device=x.device).expand(xq.shape[0], d)
        ctx.save_for_backward(xb, wg32, idx, w, probs, lse, pos,
                              ctx_img if ctx_img is not None else torch.empty(0))
        ctx.meta = (T, d, E, int(normalize), tokens_per_image, cb is not None, x.dtype,
                    ctx_bias.shape[0] if ctx_bias is not None else 0)
        ctx.mark_non_differentiable(pos, hist, offsets, xq, xs)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the index outputs
        return carrier, w, auxp, pos, hist, offsets, xq, xs

    @staticmethod
    def backward(ctx, d_xp, d_w, d_auxp, _p, _h, _o, _q, _s):
        return _RouteDispatch.backward(ctx, d_xp, d_w, d_auxp, _p, _h, _o)


class _RouteIndex(torch.autograd.Function):
    """_RouteDispatch without the row copy: the dispatch writes pos and the row
    -> token map ``tok`` (moe_route_index); a zero-stride bf16 ``carrier``
    [rows, d] stands for the routed rows in the autograd graph so that dXp
    (from _ExpertFFNGather.backward) reaches the dispatch transpose."""

    @staticmethod
    def forward(ctx, x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize, cap, rows, lb_coef, z_coef):
        T, d = x.shape
        E = wg.shape[0]
        xb = x.to(torch.bfloat16).contiguous()
        wg32 = wg.float().contiguous()
        cb = ctx_bias.float().contiguous() if ctx_bias is not None else None
        idx, w, probs, lse, lrank, bcnt, auxp = L.router_topk_fwd(xb, wg32, cb, ctx_img, tokens_per_image, k,
                                                                   normalize)
        # scan + index (+ aux losses) in one launch (moe_route_dispatch)
        pos, tok, hist, offsets, _, out3, wcoef = L.route_dispatch(bcnt, idx, lrank, w, auxp, T, E, cap, rows,
                                                                   lb_coef, z_coef)
        if out3 is None:
            out3 = torch.zeros(3, dtype=torch.float32, device=x.device)
            wcoef = torch.zeros(E + 1, dtype=torch.float32, device=x.device)
        carrier = torch.zeros((1, 1), dtype=torch.bfloat16, device=x.device).expand(max(rows, 1), d)
        ctx.save_for_backward(xb, wg32, idx, w, probs, lse, pos,
                              ctx_img if ctx_img is not None else torch.empty(0))
        ctx.meta = (T, d, E, int(normalize), tokens_per_image, cb is not None, x.dtype,
                    ctx_bias.shape[0] if ctx_bias is not None else 0)
        ctx.mark_non_differentiable(pos, hist, offsets, tok, out3, wcoef)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for the index outputs
        return carrier, w, auxp, pos, hist, offsets, tok, out3, wcoef

    @staticmethod
    def backward(ctx, d_xp, d_w, d_auxp, _p, _h, _o, _t, _a, _c):
        return _RouteDispatch.backward(ctx, d_xp, d_w, d_auxp, _p, _h, _o)[:9] + (None, None)


class _AuxFused(torch.autograd.Function):
    """The layer's weighted aux loss computed by moe_route_dispatch (out3 =
    (lb, z, lb_coef lb + z_coef z), wcoef = its gradient w.r.t. one router
    block's partials); backward = g * wcoef broadcast over the blocks."""

    @staticmethod
    def forward(ctx, auxp, out3, wcoef):
        ctx.save_for_backward(wcoef)
        ctx.nblk = auxp.shape[0]
        raw = out3[:2].clone()
        ctx.mark_non_differentiable(raw)
        ctx.set_materialize_grads(False)
        return out3[2].clone(), raw

    @staticmethod
    def backward(ctx, g, _raw):
        if g is None:
            return None, None, None
        (wcoef,) = ctx.saved_tensors
        return (g * wcoef).view(1, -1).expand(ctx.nblk, -1), None, None


def _ffn_backward(dyp, h, w1b, w2b, offsets, G, rows, xrows, tok, wdtype, s):
    """The expert FFN's backward in two paired launches:
    {dH = (dYp W2) * (H > 0), dW2 = dYp^T H, db2} then {dXp = dH W1, dW1 = dH^T Xp, db1},
    Xp = xrows (the routed rows) or xrows[tok] (token rows gathered)."""
    F, d = w1b.shape[1], w1b.shape[2]
    odt = torch.bfloat16 if wdtype == torch.bfloat16 else torch.float32
    dh, dW2, db2 = L.grouped_gemm_bwd_pair(dyp, w2b, offsets, G, rows, F, d, L.EPI_RELU_MASK, h, dyp, h,
                                           out_dtype=odt)
    dxp, dW1, db1 = L.grouped_gemm_bwd_pair(dh, w1b, offsets, G, rows, d, F, L.EPI_NONE, None, dh, xrows, tok,
                                            out_dtype=odt)
    if s != 1.0:
        for t in (dW1, db1, dW2, db2):
            t.mul_(s)
    return dxp, dW1, db1, dW2, db2


class _ExpertFFNGather(torch.autograd.Function):
    """Expert FFN whose GEMM1 reads routed row r as token row xb[tok[r]]
    (moe_grouped_gemm_gather); ``carrier`` is _RouteIndex's stand-in for the
    routed rows (its gradient is dXp)."""

    @staticmethod
    def forward(ctx, carrier, xb, tok, w1, b1, w2, b2, offsets, rows, grad_scale):
        G, F, d = w1.shape
        w1b = w1.to(torch.bfloat16).contiguous()
        w2b = w2.to(torch.bfloat16).contiguous()
        h, yp = _ffn_forward(xb, tok, w1b, b1, w2b, b2, offsets, G, rows)
        ctx.save_for_backward(xb, tok, h, w1b, w2b, offsets)
        ctx.meta = (G, rows, float(grad_scale))
        ctx.wdtype = w1.dtype if (w1.dtype == b1.dtype == w2.dtype == b2.dtype) else torch.float32
        return yp

    @staticmethod
    def backward(ctx, d_yp):
        xb, tok, h, w1b, w2b, offsets = ctx.saved_tensors
        G, rows, s = ctx.meta
        dyp = d_yp.to(torch.bfloat16).contiguous()
        dxp, dW1, db1, dW2, db2 = _ffn_backward(dyp, h, w1b, w2b, offsets, G, rows, xb, tok, ctx.wdtype, s)
        return dxp, None, None, dW1, db1, dW2, db2, None, None, None


class _ExpertFFN(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xp, w1, b1, w2, b2, offsets, rows, grad_scale):
        G, F, d = w1.shape
        w1b = w1.to(torch.bfloat16).contiguous()
        w2b = w2.to(torch.bfloat16).contiguous()
        h, yp = _ffn_forward(xp, None, w1b, b1, w2b, b2, offsets, G, rows)
        ctx.save_for_backward(xp, h, w1b, w2b, offsets)
        ctx.meta = (G, F, d, rows, float(grad_scale))
        ctx.wdtype = w1.dtype if (w1.dtype == b1.dtype == w2.dtype == b2.dtype) else torch.float32
        return yp

    @staticmethod
    def backward(ctx, d_yp):
        xp, h, w1b, w2b, offsets = ctx.saved_tensors
        G, F, d, rows, s = ctx.meta
        dyp = d_yp.to(torch.bfloat16).contiguous()
        # weight gradients written in the parameters' dtype by the kernel (bf16
        # weights: no fp32 copy + autograd cast pass)
        dxp, dW1, db1, dW2, db2 = _ffn_backward(dyp, h, w1b, w2b, offsets, G, rows, xp, None, ctx.wdtype, s)
        return dxp, dW1, db1, dW2, db2, None, None, None


class _ExpertFFNMX(torch.autograd.Function):
    """MXFP8 expert FFN (config C5; include/moe_hip.h "MXFP8 expert path").
    Forward: W1/W2 quantized per call; GEMM1 (e4m3 xq x e4m3 W1, +b1, ReLU)
    writes H as MXFP8; GEMM2 (e4m3 H x e4m3 W2, +b2) writes bf16 Yp.
    Backward: ReLU mask from the e4m3 H, dgrad through the bf16 weights,
    weight gradients against the dequantised (exact) e4m3 H and xq."""

    @staticmethod
    def forward(ctx, carrier, xq, xs, w1, b1, w2, b2, offsets, rows, grad_scale):
        G, F, d = w1.shape
        w1b = w1.to(torch.bfloat16).contiguous()
        w2b = w2.to(torch.bfloat16).contiguous()
        w1q, w1s = L.quantize_mx(w1b)
        w2q, w2s = L.quantize_mx(w2b)
        hq, hs = L.grouped_gemm_mx(xq, xs, w1q, w1s, offsets, G, rows, F, d, L.EPI_BIAS_RELU,
                                   bias=b1.float().contiguous(), out_mx=True)
        yp = L.grouped_gemm_mx(hq, hs, w2q, w2s, offsets, G, rows, d, F, L.EPI_BIAS, bias=b2.float().contiguous())
        ctx.save_for_backward(xq, xs, hq, hs, w1b, w2b, offsets)
        ctx.meta = (G, F, d, rows, float(grad_scale))
        return yp

    @staticmethod
    def backward(ctx, d_yp):
        xq, xs, hq, hs, w1b, w2b, offsets = ctx.saved_tensors
        G, F, d, rows, s = ctx.meta
        dyp = d_yp.to(torch.bfloat16).contiguous()
        dh = L.grouped_gemm(dyp, w2b, offsets, G, rows, F, d, 0, L.EPI_RELU_MASK_MX, aux=hq)
        dW2, db2 = L.grouped_gemm_wgrad_mx(dyp, hq, hs, offsets, G)
        dxp = L.grouped_gemm(dh, w1b, offsets, G, rows, d, F, 0, L.EPI_NONE)
        dW1, db1 = L.grouped_gemm_wgrad_mx(dh, xq, xs, offsets, G)
        if s != 1.0:
            for t in (dW1, db1, dW2, db2):
                t.mul_(s)
        return dxp, None, None, dW1, db1, dW2, db2, None, None, None


class _Combine(torch.autograd.Function):
    @staticmethod
    def forward(ctx, yp, w, pos, T):
        y = L.combine_fwd(yp.to(torch.bfloat16).contiguous(), pos, w, T)
        ctx.save_for_backward(yp, w, pos)
        return y

    @staticmethod
    def backward(ctx, dy):
        yp, w, pos = ctx.saved_tensors
        dyp, dw = L.combine_bwd(dy.to(torch.bfloat16).contiguous(), yp.to(torch.bfloat16).contiguous(), pos, w)
        return dyp, dw, None, None


class _AuxLoss(torch.autograd.Function):
    """lb_coef lb + z_coef z of one layer in one HIP launch (moe_aux_loss_fwd);
    backward = g * wcoef broadcast over the router blocks (one launch).  The
    raw (lb, z) ride along, detached, for logging."""

    @staticmethod
    def forward(ctx, auxp, hist, T, k, lb_coef, z_coef):
        out, wcoef = L.aux_loss_fwd(auxp.contiguous(), hist, T, k, lb_coef, z_coef)
        ctx.save_for_backward(wcoef)
        ctx.nblk = auxp.shape[0]
        raw = out[:2]
        ctx.mark_non_differentiable(raw)
        ctx.set_materialize_grads(False)
        return out[2], raw  # (views of the kernel's output: no copy)

    @staticmethod
    def backward(ctx, g, _raw):
        if g is None:
            return None, None, None, None, None, None
        (wcoef,) = ctx.saved_tensors
        return (g * wcoef).view(1, -1).expand(ctx.nblk, -1), None, None, None, None, None


class _AuxLossRaw(torch.autograd.Function):
    """(lb, z) of one layer as separate differentiable scalars from ONE HIP
    launch (moe_aux_loss_fwd with unit coefficients: wcoef = d(lb, z)/d auxp
    per column); backward = (g_lb wcoef[:E], g_z wcoef[E]) broadcast over the
    router blocks (one small op)."""

    @staticmethod
    def forward(ctx, auxp, hist, T, k):
        out, wcoef = L.aux_loss_fwd(auxp.contiguous(), hist, T, k, 1.0, 1.0)
        ctx.save_for_backward(wcoef)
        ctx.nblk = auxp.shape[0]
        ctx.set_materialize_grads(False)
        return out[0], out[1]  # (views of the kernel's output: no copies)

    @staticmethod
    def backward(ctx, g_lb, g_z):
        (wcoef,) = ctx.saved_tensors
        E = wcoef.numel() - 1
        if g_lb is None and g_z is None:
            return None, None, None, None
        if g_lb is None or g_z is None:
            zero = torch.zeros((), dtype=wcoef.dtype, device=wcoef.device)
            g_lb = zero if g_lb is None else g_lb
            g_z = zero if g_z is None else g_z
        scale = torch.cat([g_lb.reshape(1).expand(E), g_z.reshape(1)])
        return (scale * wcoef).view(1, -1).expand(ctx.nblk, -1), None, None, None


def aux_losses_hip(auxp, hist, T, k):
    """-> (lb, z), differentiable, in one launch each way (moe_aux_loss_fwd)."""
    return _AuxLossRaw.apply(auxp, hist, int(T), int(k))


def aux_loss_weighted(auxp, hist, T, k, lb_coef, z_coef):
    """-> (lb_coef lb + z_coef z (differentiable), detached (lb, z) [2])."""
    return _AuxLoss.apply(auxp, hist, int(T), int(k), float(lb_coef), float(z_coef))


def aux_losses(auxp, hist, T, k):
    E = hist.shape[0]
    f = hist.float() / float(max(T * k, 1))
    P = auxp[:, :E].sum(0) / float(max(T, 1))
    lb = E * (f * P).sum()
    z = auxp[:, E].sum() / float(max(T, 1))
    return lb, z


def route_dispatch_hip(x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize, cap, pad=0):
    """-> (xp, w, auxp, pos, hist, offsets, rows); pad > 0: fixed-capacity
    layout (rows = E pad, offsets = e pad; see _RouteDispatch)."""
    T = x.shape[0]
    E = wg.shape[0]
    rows = E * pad if pad else (T * k if cap <= 0 else min(T * k, E * cap))
    return _RouteDispatch.apply(x, wg, ctx_bias, ctx_img, int(tokens_per_image), int(k), bool(normalize), int(cap),
                                rows, int(pad)) + (rows,)


def route_dispatch_mx_hip(x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize, cap, pad=0):
    """-> (carrier, w, auxp, pos, hist, offsets, xq, xs, rows): MXFP8 dispatch."""
    T = x.shape[0]
    E = wg.shape[0]
    rows = E * pad if pad else (T * k if cap <= 0 else min(T * k, E * cap))
    return _RouteDispatchMX.apply(x, wg, ctx_bias, ctx_img, int(tokens_per_image), int(k), bool(normalize),
                                  int(cap), rows, int(pad)) + (rows,)


# MOE_FUSE_RESIDUAL=0: the residual add stays a torch add (A/B switch)
_FUSE_RESIDUAL = os.environ.get("MOE_FUSE_RESIDUAL", "1") != "0"


class _MoELayer(torch.autograd.Function):
    """The whole single-GPU bf16 routed FFN of one layer as ONE autograd node
    (SURVEY 8(a) rows a2-a7), 8 HIP launches forward + backward:
      forward  router_topk_fwd; route_dispatch (scan, index, row gates, aux
               losses); the expert FFN reading token rows through the row
               map (moe_expert_ffn_fwd: GEMM1 +b1, ReLU, GEMM2 +b2 in one
               launch); combine
      backward bwd_pair {dH = gate * (dy[token] W2) * (H > 0), dW2 = dYp^T H,
               db2} with dYp = gate * dy[token] formed inside the GEMMs (no
               combine transpose launch); bwd_pair {dXp = dH W1, dW1 = dH^T
               x[token], db1}; token_bwd_dw (gate gradient <dy, Yp>, router
               softmax / top-k / aux / z-loss backward, dx)
    plus the router weight and context-bias gradients (moe_router_wgrad: one
    launch, fixed-order sums).  Outputs: y, then (weighted=True) the
    layer's lb_coef lb + z_coef z and the detached raw (lb, z), or
    (weighted=False) lb and z as separate differentiable outputs; hist.
    residual=True (x in bf16): y = x + FFN(x) -- the caller's residual add
    folded into combine (one bf16 rounding) and its gradient into token_bwd
    (dx = dy + ...), so neither the forward add nor autograd's gradient
    accumulation for x runs as a separate launch."""

    @staticmethod
    def forward(ctx, x, wg, ctx_bias, w1, b1, w2, b2, ctx_img, tpi, k, normalize, cap, lb_coef, z_coef, weighted,
                residual=False):
        T, d = x.shape
        E = wg.shape[0]
        G, F, _ = w1.shape
        rows = T * k if cap <= 0 else min(T * k, E * cap)
        xb = x.to(torch.bfloat16).contiguous()
        wg32 = wg.float().contiguous()
        cb = ctx_bias.float().contiguous() if ctx_bias is not None else None
        idx, w, probs, lse, lrank, bcnt, auxp = L.router_topk_fwd(xb, wg32, cb, ctx_img, tpi, k, normalize)
        pos, tok, hist, offsets, gate, out3, wcoef = L.route_dispatch(bcnt, idx, lrank, w, auxp, T, E, cap, rows,
                                                                      lb_coef, z_coef, row_gate=True)
        w1b = w1.to(torch.bfloat16).contiguous()
        w2b = w2.to(torch.bfloat16).contiguous()
        h, yp = _ffn_forward(xb, tok, w1b, b1, w2b, b2, offsets, G, rows)
        y = L.combine_fwd(yp, pos, w, T, resid=xb if residual else None)
        ctx.residual = bool(residual)
        ctx.save_for_backward(xb, wg32, idx, w, probs, lse, pos, tok, gate, h, yp, w1b, w2b, offsets, wcoef,
                              ctx_img if ctx_img is not None else torch.empty(0))
        ctx.meta = (T, d, E, G, rows, int(normalize), tpi, cb is not None,
                    ctx_bias.shape[0] if ctx_bias is not None else 0, weighted)
        ctx.dtypes = (x.dtype, w1.dtype if (w1.dtype == b1.dtype == w2.dtype == b2.dtype) else torch.float32)
        ctx.mark_non_differentiable(hist)
        ctx.set_materialize_grads(False)  # no zero-filled gradients for raw / hist (backward takes None)
        # out3's elements leave as views (no copy launches); nothing writes them in place
        if weighted:
            raw = out3[:2]
            ctx.mark_non_differentiable(raw)
            return y.to(x.dtype), out3[2], raw, hist
        return y.to(x.dtype), out3[0], out3[1], hist

    @staticmethod
    def backward(ctx, dy, g_a, g_b, _h):
        (xb, wg32, idx, w, probs, lse, pos, tok, gate, h, yp, w1b, w2b, offsets, wcoef,
         ctx_img) = ctx.saved_tensors
        T, d, E, G, rows, normalize, tpi, has_ctx, C, weighted = ctx.meta
        xdtype, wdtype = ctx.dtypes
        F = w1b.shape[1]
        odt = torch.bfloat16 if wdtype == torch.bfloat16 else torch.float32
        if dy is None:
            dy = torch.zeros((T, d), dtype=torch.bfloat16, device=xb.device)
        dyb = dy.to(torch.bfloat16).contiguous()
        if _FFN_BWD2:  # two launches: dH, then {dXp, dW2, dW1} in one grid
            _, dxp, dW1, db1, dW2, db2 = L.expert_ffn_bwd(dyb, tok, gate, xb, h, w1b, w2b, offsets, G, rows,
                                                          out_dtype=odt)
        else:  # paired launches {dH, dW2}, {dXp, dW1} (A/B)
            dh, dW2, db2 = L.grouped_gemm_bwd_pair(dyb, w2b, offsets, G, rows, F, d, L.EPI_RELU_MASK, h, dyb, h,
                                                   out_dtype=odt, a_gather=tok, row_scale=gate, wx_gather=tok,
                                                   wx_scale=gate)
            dxp, dW1, db1 = L.grouped_gemm_bwd_pair(dh, w1b, offsets, G, rows, d, F, L.EPI_NONE, None, dh, xb, tok,
                                                    out_dtype=odt)
        # aux-loss gradients as device tensors (no host sync): the router
        # partials' gradient is uniform over blocks (moe_route_dispatch wcoef)
        if weighted:
            if g_a is not None:
                coef = g_a.float() * wcoef
                dprob_bias, zc = coef[:E].contiguous(), (2.0 * coef[E:E + 1]).contiguous()
            else:
                dprob_bias, zc = None, None
        else:
            # wcoef holds d lb / d partials (lb_coef = 1) and d z / d partials (z_coef = 1)
            dprob_bias = (g_a.float() * wcoef[:E]).contiguous() if g_a is not None else None
            zc = (2.0 * g_b.float() * wcoef[E:E + 1]).contiguous() if g_b is not None else None
        dx, dlogits, _ = L.token_bwd_dw(dxp, pos, probs, idx, w, dyb, yp, lse, dprob_bias, zc, wg32, normalize,
                                        dres=dyb if ctx.residual else None)
        # router weight + context-bias gradients: one HIP launch, fixed-order sums
        dwg, dcb = L.router_wgrad(dlogits, xb, ctx_img if has_ctx else None, tpi, C if has_ctx else 0)
        return (dx.to(xdtype), dwg, dcb, dW1, db1, dW2, db2) + (None,) * 9


def moe_layer_hip(x, wg, ctx_bias, w1, b1, w2, b2, ctx_img, tokens_per_image, k, normalize, cap, aux_coefs=None,
                  residual=False):
    """_MoELayer: -> (y, lb_coef lb + z_coef z, raw (lb, z), hist) with aux_coefs,
    else (y, lb, z, hist); residual=True returns x + y (fused for bf16 x)."""
    fuse = bool(residual) and x.dtype == torch.bfloat16 and _FUSE_RESIDUAL
    if aux_coefs is not None:
        out = _MoELayer.apply(x, wg, ctx_bias, w1, b1, w2, b2, ctx_img, int(tokens_per_image), int(k),
                              bool(normalize), int(cap), float(aux_coefs[0]), float(aux_coefs[1]), True, fuse)
    else:
        out = _MoELayer.apply(x, wg, ctx_bias, w1, b1, w2, b2, ctx_img, int(tokens_per_image), int(k),
                              bool(normalize), int(cap), 1.0, 1.0, False, fuse)
    if residual and not fuse:  # fp32 activations (amp): keep the residual add in x's precision
        out = (x + out[0],) + tuple(out[1:])
    return out


def route_index_hip(x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize, cap, aux_coefs=None):
    """-> (carrier, w, auxp, pos, hist, offsets, tok, out3, wcoef, rows): dispatch
    without the row copy; out3 / wcoef are the fused aux loss (aux_coefs given)."""
    T = x.shape[0]
    E = wg.shape[0]
    rows = T * k if cap <= 0 else min(T * k, E * cap)
    lb, z = aux_coefs if aux_coefs is not None else (None, None)
    return _RouteIndex.apply(x, wg, ctx_bias, ctx_img, int(tokens_per_image), int(k), bool(normalize), int(cap),
                             rows, lb, z) + (rows,)


def expert_ffn_gather_hip(carrier, xb, tok, w1, b1, w2, b2, offsets, rows, grad_scale=1.0):
    return _ExpertFFNGather.apply(carrier, xb, tok, w1, b1, w2, b2, offsets, int(rows), grad_scale)


def expert_ffn_hip(xp, w1, b1, w2, b2, offsets, rows, grad_scale=1.0):
    return _ExpertFFN.apply(xp, w1, b1, w2, b2, offsets, int(rows), grad_scale)


def expert_ffn_mx_hip(carrier, xq, xs, w1, b1, w2, b2, offsets, rows, grad_scale=1.0):
    return _ExpertFFNMX.apply(carrier, xq, xs, w1, b1, w2, b2, offsets, int(rows), grad_scale)


class _CombineRes(torch.autograd.Function):
    """y = resid + combine (one bf16 rounding, moe_combine_res_fwd): the EP
    layer's residual branch without a separate add; backward: dresid = dy."""

    @staticmethod
    def forward(ctx, yp, w, pos, T, resid):
        y = L.combine_fwd(yp.to(torch.bfloat16).contiguous(), pos, w, T, resid=resid.to(torch.bfloat16).contiguous())
        ctx.save_for_backward(yp, w, pos)
        ctx.rdtype = resid.dtype
        return y

    @staticmethod
    def backward(ctx, dy):
        yp, w, pos = ctx.saved_tensors
        dyp, dw = L.combine_bwd(dy.to(torch.bfloat16).contiguous(), yp.to(torch.bfloat16).contiguous(), pos, w)
        return dyp, dw, None, None, dy.to(ctx.rdtype)


def combine_hip(yp, w, pos, T, resid=None):
    if resid is not None:
        return _CombineRes.apply(yp, w, pos, int(T), resid)
    return _Combine.apply(yp, w, pos, int(T))


def moe_ffn_hip(x, wg, ctx_bias, w1, b1, w2, b2, ctx_img, tokens_per_image, k, normalize, cap,
                expert_dtype="bf16", aux_coefs=None, residual=False):
    """Routed expert FFN of one layer on the GPU.

    x [T, d] (tokens of ``T // tokens_per_image`` images, image-major),
    wg [E, d], ctx_bias [C, E] or None, w1 [E, F, d], b1 [E, F], w2 [E, d, F],
    b2 [E, d], ctx_img int32 [T // tokens_per_image].  expert_dtype "bf16" or
    "fp8" (MXFP8 dispatch rows and expert GEMMs, config C5).
    Returns (y bf16 [T, d], lb_raw, z_raw, hist int32 [E]); with
    aux_coefs = (lb_coef, z_coef) it returns (y, aux, (lb, z) detached, hist)
    instead, aux = lb_coef lb + z_coef z from the fused aux-loss kernel.
    residual=True: the first output is x + y (the layer's residual branch;
    fused into combine / token_bwd on the bf16 path).
    """
    if not x.is_cuda:
        raise L.MoEKernelError("moe_ffn_hip needs GPU tensors")
    if ctx_bias is not None and ctx_img is None:
        raise L.MoEKernelError("ctx_bias given without ctx_img")
    if expert_dtype not in ("bf16", "fp8"):
        raise L.MoEKernelError(f"unknown expert_dtype {expert_dtype!r}")
    T = x.shape[0]
    if expert_dtype == "fp8":
        carrier, w, auxp, pos, hist, offsets, xq, xs, rows = route_dispatch_mx_hip(
            x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize, cap)
        yp = expert_ffn_mx_hip(carrier, xq, xs, w1, b1, w2, b2, offsets, rows)
    else:
        return moe_layer_hip(x, wg, ctx_bias, w1, b1, w2, b2, ctx_img, tokens_per_image, k, normalize, cap,
                             aux_coefs, residual=residual)
    y = combine_hip(yp, w, pos, T)
    if residual:
        y = x + y.to(x.dtype)
    if aux_coefs is not None:
        aux, raw = aux_loss_weighted(auxp, hist, T, k, *aux_coefs)
        return y, aux, raw, hist
    lb, z = aux_losses(auxp, hist, T, k)
    return y, lb, z, hist
