"""TEST / BASELINE INFRASTRUCTURE ONLY: run the numpy oracle inside a CPU
torch model (bench.py's cpu_baseline leg and tests).  Wraps
oracle.moe_oracle.moe_forward / moe_backward as an autograd Function and
swaps it into every MoEFFN module of a model that lives on the CPU."""
from __future__ import annotations

import types

import numpy as np
import torch

from . import moe_oracle as O


class _OracleMoE(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, wg, ctx_bias, w1, b1, w2, b2, ctx_img, tpi, k, normalize, cap, mx=False):
        n = lambda t: None if t is None else t.detach().double().numpy()  # noqa: E731
        ci = None if ctx_img is None else ctx_img.numpy()
        st = O.moe_forward(n(x), n(wg), n(ctx_bias), n(w1), n(b1), n(w2), n(b2), ci, tpi, k, normalize, cap, mx=mx)
        ctx.st = st
        ctx.args = (n(x), n(wg), n(w1), n(w2), ci, tpi, 0 if ctx_bias is None else ctx_bias.shape[0], normalize)
        ctx.has_ctx = ctx_bias is not None
        f = lambda a: torch.from_numpy(np.asarray(a)).to(x.dtype)  # noqa: E731
        return f(st.y), torch.tensor(st.lb, dtype=x.dtype), torch.tensor(st.z, dtype=x.dtype)

    @staticmethod
    def backward(ctx, dy, g_lb, g_z):
        x, wg, w1, w2, ci, tpi, C, normalize = ctx.args
        g = O.moe_backward(ctx.st, x, wg, w1, w2, ci, tpi, C, dy.double().numpy(), float(g_lb), float(g_z),
                           normalize)
        f = lambda a: None if a is None else torch.from_numpy(np.asarray(a)).to(dy.dtype)  # noqa: E731
        return (f(g["dx"]), f(g["dwg"]), f(g["dctx_bias"]) if ctx.has_ctx else None, f(g["dw1"]), f(g["db1"]),
                f(g["dw2"]), f(g["db2"]), None, None, None, None, None, None)


def _oracle_forward(self, x, ctx_img):
    B, L, d = x.shape
    cfg = self.cfg
    cb = self.ctx_bias if (self.ctx_bias is not None and ctx_img is not None) else None
    y, lb, z = _OracleMoE.apply(x.reshape(B * L, d), self.wg, cb, self.w1, self.b1, self.w2, self.b2,
                                ctx_img if cb is not None else None, L, cfg.top_k, cfg.normalize,
                                cfg.capacity(B * L), cfg.expert_dtype == "fp8")
    self.last_aux = (lb, z)
    return y.view(B, L, d)


def use_oracle_moe(model: torch.nn.Module) -> int:
    """Route every MoEFFN of a CPU model through the oracle; returns the count."""
    n = 0
    for m in model.modules():
        if type(m).__name__ == "MoEFFN":
            m.forward = types.MethodType(_oracle_forward, m)
            n += 1
    return n
