"""MoEFFN: the routed expert FFN that replaces the dense FFN of the RT-DETR
AIFI encoder layer and of every decoder layer.

Parameters (fp32 masters; the GPU path computes in bf16 with fp32 accumulate):
  router.weight wg [E, d]      router.ctx_bias [C, E]  (context as additive logit bias)
  w1 [E, F, d], b1 [E, F]      w2 [E, d, F], b2 [E, d]  (nn.Linear layout per expert)
"""
from __future__ import annotations

import math

import torch
from torch import nn

from .config import MoEConfig


class MoEFFN(nn.Module):
    def __init__(self, d_model: int, cfg: MoEConfig):
        super().__init__()
        self.cfg = cfg
        E, F = cfg.num_experts, cfg.hidden
        self.d_model = d_model
        self.ep_size = max(1, cfg.ep_size)
        self.ep_group = None          # set by parallel.expert_parallel for C4
        self.wg = nn.Parameter(torch.randn(E, d_model) * cfg.router_init_std)
        self.ctx_bias = nn.Parameter(torch.randn(cfg.num_contexts, E) * cfg.ctx_init_scale) \
            if cfg.use_context else None
        bound1 = 1.0 / math.sqrt(d_model)
        bound2 = 1.0 / math.sqrt(F)
        # all E experts are initialised on every rank (same RNG stream), then an
        # expert-parallel rank keeps its slice [r E/W, (r+1) E/W)
        w1 = torch.empty(E, F, d_model).uniform_(-bound1, bound1)
        b1 = torch.empty(E, F).uniform_(-bound1, bound1)
        w2 = torch.empty(E, d_model, F).uniform_(-bound2, bound2)
        b2 = torch.empty(E, d_model).uniform_(-bound2, bound2)
        if self.ep_size > 1:
            import torch.distributed as dist

            if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() != self.ep_size:
                raise RuntimeError(f"expert parallelism over {self.ep_size} ranks needs torch.distributed "
                                   f"initialised with world size {self.ep_size} before the model is built")
            El = E // self.ep_size
            r = dist.get_rank()
            w1, b1, w2, b2 = (t[r * El:(r + 1) * El].clone() for t in (w1, b1, w2, b2))
        self.w1 = nn.Parameter(w1)
        self.b1 = nn.Parameter(b1)
        self.w2 = nn.Parameter(w2)
        self.b2 = nn.Parameter(b2)
        for p in (self.w1, self.b1, self.w2, self.b2):
            p.expert_parallel = self.ep_size > 1  # excluded from the DP all-reduce
        self.last_aux = None   # (lb_raw, z_raw) of the last forward
        self.last_aux_weighted = None  # lb_coef lb + z_coef z (GPU path: fused kernel, differentiable)
        self.last_hist = None  # int32 [E] expert histogram of the last forward
        self.last_ep_overflow = None  # EP without capacity: assignments beyond the a2a slots (device)
        self.last_tokens = 0   # T of the last forward (bench: EP exchange bytes)
        self.y_has_residual = False  # EP: the residual was folded into the combine
        self.ep_aux_weighted = None  # EP on the GPU: lb_coef lb + z_coef z from the fused kernel

    def forward(self, x: torch.Tensor, ctx_img: torch.Tensor | None, residual: bool = False) -> torch.Tensor:
        """x [B, L, d] (image-major tokens), ctx_img int [B] -> [B, L, d].
        residual=True returns x + FFN(x) (the caller's residual branch; on the
        single-GPU bf16 path fused into the combine and token_bwd kernels)."""
        B, L, d = x.shape
        cfg = self.cfg
        flat = x.reshape(B * L, d)
        T = B * L
        self.last_tokens = T
        cap = cfg.capacity(T)
        cb = self.ctx_bias if (self.ctx_bias is not None and ctx_img is not None) else None
        ci = ctx_img.to(torch.int32).contiguous() if cb is not None else None
        if self.ep_size > 1 or cfg.expert_parallel:  # C4: experts sharded over ranks, all-to-all exchange
            from .ep import moe_ffn_ep

            y, lb, z, hist = moe_ffn_ep(self, flat, cb, ci, L, cap, residual=residual,
                                        aux_coefs=(cfg.lb_coef, cfg.z_coef))
            if residual and self.y_has_residual:  # folded into the combine
                self.last_aux = (lb, z)
                self.last_aux_weighted = self.ep_aux_weighted
                self.last_hist = hist
                return y.to(x.dtype).view(B, L, d)
        elif flat.is_cuda:
            from .ops import moe_ffn_hip

            y, aux, raw, hist = moe_ffn_hip(flat, self.wg, cb, self.w1, self.b1, self.w2, self.b2,
                                            ci, L, cfg.top_k, cfg.normalize, cap, cfg.expert_dtype,
                                            aux_coefs=(cfg.lb_coef, cfg.z_coef), residual=residual)
            self.last_aux = (raw[0], raw[1])
            self.last_aux_weighted = aux
            self.last_hist = hist
            return y.to(x.dtype).view(B, L, d)
        else:
            from .eager import moe_ffn_eager

            y, lb, z, hist = moe_ffn_eager(flat, self.wg, cb, self.w1, self.b1, self.w2, self.b2,
                                           ci, L, cfg.top_k, cfg.normalize, cap, cfg.expert_dtype)
        y = y.to(x.dtype)
        if residual:
            y = flat + y
        self.last_aux = (lb, z)
        self.last_aux_weighted = getattr(self, "ep_aux_weighted", None)
        self.last_hist = hist
        return y.view(B, L, d)

    def aux_loss(self) -> torch.Tensor | None:
        if self.last_aux is None:
            return None
        if self.last_aux_weighted is not None:  # fused kernel (GPU path)
            return self.last_aux_weighted
        lb, z = self.last_aux
        return self.cfg.lb_coef * lb + self.cfg.z_coef * z
