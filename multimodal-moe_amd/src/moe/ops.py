"""autograd wrapper of the HIP MoE FFN.

``moe_ffn_hip`` runs the whole routed FFN of one layer on the GPU through
libmoe_hip.so: 6 launches forward (router, route_scan, permute, GEMM1+bias+
ReLU, GEMM2+bias, combine) and 7 backward (combine_bwd, dgrad GEMM with the
ReLU mask, wgrad GEMM (+db2), dgrad GEMM, wgrad GEMM (+db1), token_bwd, and a
plain GEMM for the router weight gradient).  Nothing is synchronised with the
host: expert offsets stay on the device and every grid is sized from host
upper bounds.
"""
from __future__ import annotations

import torch

from . import _lib as L


class _MoEFFNHip(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wg, ctx_bias, w1, b1, w2, b2, ctx_img, tokens_per_image, k, normalize, cap):
        T, d = x.shape
        E, F = w1.shape[0], w1.shape[1]
        xb = x.to(torch.bfloat16).contiguous()
        wg32 = wg.float().contiguous()
        cb = ctx_bias.float().contiguous() if ctx_bias is not None else None
        w1b = w1.to(torch.bfloat16).contiguous()
        w2b = w2.to(torch.bfloat16).contiguous()
        b1f = b1.float().contiguous()
        b2f = b2.float().contiguous()

        idx, w, probs, lse, lrank, bcnt, auxp = L.router_topk_fwd(
            xb, wg32, cb, ctx_img, tokens_per_image, k, normalize)
        rank_base, hist, offsets = L.route_scan(bcnt, cap)
        rows = T * k if cap <= 0 else min(T * k, E * cap)
        xp, pos = L.permute_fwd(xb, idx, lrank, rank_base, offsets, E, cap, rows)
        h = L.grouped_gemm(xp, w1b, offsets, E, rows, F, d, 1, L.EPI_BIAS_RELU, bias=b1f)
        yp = L.grouped_gemm(h, w2b, offsets, E, rows, d, F, 1, L.EPI_BIAS, bias=b2f)
        y = L.combine_fwd(yp, pos, w, T)

        # aux losses, raw (coefficients applied by the caller)
        f = hist.float() / float(max(T * k, 1))
        P = auxp[:, :E].sum(0) / float(max(T, 1))
        lb = E * (f * P).sum()
        z = auxp[:, E].sum() / float(max(T, 1))

        ctx.save_for_backward(xb, wg32, w1b, w2b, idx, w, probs, lse, pos, offsets, xp, h, yp, hist,
                              ctx_img if ctx_img is not None else torch.empty(0))
        ctx.meta = (T, d, E, F, k, int(normalize), rows, tokens_per_image, cb is not None,
                    x.dtype, ctx_bias.shape[0] if ctx_bias is not None else 0)
        ctx.mark_non_differentiable(hist)
        return y, lb, z, hist

    @staticmethod
    def backward(ctx, dy, g_lb, g_z, _g_hist):
        (xb, wg32, w1b, w2b, idx, w, probs, lse, pos, offsets, xp, h, yp, hist,
         ctx_img) = ctx.saved_tensors
        T, d, E, F, k, normalize, rows, tpi, has_ctx, xdtype, C = ctx.meta
        dyb = dy.to(torch.bfloat16).contiguous()
        dyp, dw = L.combine_bwd(dyb, yp, pos, w)
        dh = L.grouped_gemm(dyp, w2b, offsets, E, rows, F, d, 0, L.EPI_RELU_MASK, aux=h)
        dW2, db2 = L.grouped_gemm_wgrad(dyp, h, offsets, E)
        dxp = L.grouped_gemm(dh, w1b, offsets, E, rows, d, F, 0, L.EPI_NONE)
        dW1, db1 = L.grouped_gemm_wgrad(dh, xp, offsets, E)

        f = hist.float() / float(max(T * k, 1))
        dprob_bias = (g_lb.float() * E / float(max(T, 1))) * f
        zc = (g_z.float() * (2.0 / float(max(T, 1)))).reshape(1).contiguous() if g_z is not None else None
        dx, dlogits = L.token_bwd(dxp, pos, probs, idx, w, dw, lse, dprob_bias.contiguous(), zc,
                                  wg32, normalize)
        dwg = dlogits.t().mm(xb.float())
        dcb = None
        if has_ctx:
            per_img = dlogits.view(-1, tpi, E).sum(1)
            dcb = torch.zeros((C, E), dtype=torch.float32, device=dy.device)
            dcb.index_add_(0, ctx_img.long(), per_img)
        return (dx.to(xdtype), dwg, dcb, dW1, db1, dW2, db2, None, None, None, None, None)


def moe_ffn_hip(x, wg, ctx_bias, w1, b1, w2, b2, ctx_img, tokens_per_image, k, normalize, cap):
    """Routed expert FFN of one layer on the GPU.

    x [T, d] (tokens of ``T // tokens_per_image`` images, image-major),
    wg [E, d], ctx_bias [C, E] or None, w1 [E, F, d], b1 [E, F], w2 [E, d, F],
    b2 [E, d], ctx_img int32 [T // tokens_per_image].
    Returns (y bf16 [T, d], lb_raw, z_raw, hist int32 [E]).
    """
    if not x.is_cuda:
        raise L.MoEKernelError("moe_ffn_hip needs GPU tensors")
    if ctx_bias is not None and ctx_img is None:
        raise L.MoEKernelError("ctx_bias given without ctx_img")
    return _MoEFFNHip.apply(x, wg, ctx_bias, w1, b1, w2, b2, ctx_img, int(tokens_per_image), int(k),
                            bool(normalize), int(cap))
