"""One RT-DETR-MoE training step, optionally with the model's forward and
backward captured as hipGraphs (torch.cuda.make_graphed_callables).

Why graphs: a step launches ~6,000 kernels (MIOpen convolutions + BatchNorm,
~80 layers of small element-wise ops, 13 MoE launches x 7 layers, loss
terms); launched eagerly from Python the GPU idles ~40 % of the step waiting
for the host.  Captured, the model's forward and backward are one replay each.
What stays eager: the Hungarian matching (host linear_sum_assignment, one
device->host copy of all cost matrices), the batched set criterion, the
gradient all-reduce (one flat RCCL all_reduce over xGMI when world > 1),
gradient clipping and the fused AdamW update.

The captured forward keeps the MoE aux losses as an explicit graph output so
their gradients reach the router through the captured backward.
"""
from __future__ import annotations

import torch
import torch.distributed as dist
from torch import nn

from .model import RTDETRMoE


class FlatOutputs(nn.Module):
    """Model wrapper whose forward returns a flat tuple of tensors (a graph
    output signature): final, auxiliary and encoder logits/boxes + MoE aux loss."""

    def __init__(self, model: RTDETRMoE):
        super().__init__()
        self.model = model

    def forward(self, images, ctx):
        out = self.model(images, ctx)
        sets = [out] + list(out["aux_outputs"]) + [out["enc_outputs"]]
        flat = []
        for s in sets:
            flat += [s["pred_logits"], s["pred_boxes"]]
        aux = self.model.moe_aux_loss()
        flat.append(aux if aux is not None else out["pred_boxes"].sum() * 0.0)
        return tuple(flat)

    @staticmethod
    def unflatten(flat):
        pairs = [{"pred_logits": flat[i], "pred_boxes": flat[i + 1]} for i in range(0, len(flat) - 1, 2)]
        out = dict(pairs[0])
        out["aux_outputs"] = pairs[1:-1]
        out["enc_outputs"] = pairs[-1]
        return out, flat[-1]


def gemm_params(model: nn.Module):
    """Parameters that are GEMM / convolution operands: weights and biases of
    Linear, Conv2d and MultiheadAttention layers and the MoE expert weights.
    These are held in bf16 (TrainStep precision "bf16"); norms, the MoE router
    and everything else stay fp32."""
    from ..moe.layer import MoEFFN

    out, seen = [], set()
    for mod in model.modules():
        if isinstance(mod, (nn.Linear, nn.Conv2d)):
            ps = [mod.weight, mod.bias]
        elif isinstance(mod, nn.MultiheadAttention):
            ps = [mod.in_proj_weight, mod.in_proj_bias]
        elif isinstance(mod, MoEFFN):
            ps = [mod.w1, mod.b1, mod.w2, mod.b2]
        else:
            continue
        for p in ps:
            if p is not None and id(p) not in seen:
                seen.add(id(p))
                out.append(p)
    return out


class TrainStep:
    """precision (GPU):
      "bf16" (default) -- GEMM/conv operands (gemm_params) held in bf16, fp32
             master copies in the optimizer, no autocast: no per-layer weight
             casts in the forward nor grad casts in the backward (about 1,700
             cast ops per C2 step under autocast, most of the host time of an
             eager step); after backward the bf16 grads are copied into the
             masters' fp32 grads (multi-tensor copy), AdamW updates the
             masters, and the masters are copied back into the bf16 weights;
      "amp"  -- fp32 parameters under bf16 autocast.
    On CPU the model runs in fp32."""

    def __init__(self, model: RTDETRMoE, criterion, images, ctx, *, lr=1e-4, lr_backbone=1e-5,
                 weight_decay=1e-4, clip_norm=0.1, graphs=True, ddp_local=None, world=1, precision="bf16"):
        self.model = model
        self.criterion = criterion
        self.clip_norm = clip_norm
        self.world = world
        self.graphs = graphs
        self.precision = precision if images.is_cuda else "fp32"
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        self.params = [p for _, p in named]
        self.lowp, self.master = [], []
        opt_of = {id(p): p for p in self.params}  # model param -> tensor the optimizer updates
        if self.precision == "bf16":
            for p in gemm_params(model):
                p.data = p.data.to(torch.bfloat16)
                if p.requires_grad:
                    m = p.detach().float().clone()
                    m.grad = torch.zeros_like(m)
                    self.lowp.append(p)
                    self.master.append(m)
                    opt_of[id(p)] = m
        bb = [opt_of[id(p)] for n, p in named if n.startswith("backbone.")]
        rest = [opt_of[id(p)] for n, p in named if not n.startswith("backbone.")]
        self.opt_params = bb + rest
        fused = images.is_cuda
        self.opt = torch.optim.AdamW([{"params": bb, "lr": lr_backbone}, {"params": rest, "lr": lr}], lr=lr,
                                     weight_decay=weight_decay, fused=fused)
        self.flat = FlatOutputs(model)
        self.dp_params = [p for p in self.params if not getattr(p, "expert_parallel", False)]
        images = self._cast_in(images)
        if graphs:
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False, enabled=self.precision == "amp"):
                self.fn = torch.cuda.make_graphed_callables(self.flat, (images, ctx), num_warmup_iters=3,
                                                            allow_unused_input=True)
            self.ddp = None
        elif world > 1:
            from .engine import wrap_ddp

            self.ddp = wrap_ddp(self.flat, ddp_local)
            self.fn = self.ddp
        else:
            self.fn = self.flat
            self.ddp = None

    def _cast_in(self, images):
        return images.to(torch.bfloat16) if self.precision == "bf16" else images

    def _grads_to_master(self):
        src, dst = [], []
        for p, m in zip(self.lowp, self.master):
            if p.grad is None:
                m.grad.zero_()
            else:
                src.append(p.grad)
                dst.append(m.grad)
        if src:
            torch._foreach_copy_(dst, src)

    def _allreduce_grads(self):
        grads = [p.grad for p in self.dp_params if p.grad is not None]
        if not grads:
            return
        flat = torch.cat([g.reshape(-1) for g in grads])
        dist.all_reduce(flat)
        flat.div_(self.world)
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n

    def __call__(self, images, ctx, targets, num_boxes):
        for p in self.params:
            p.grad = None
        with torch.autocast(images.device.type, dtype=torch.bfloat16, enabled=self.precision == "amp",
                            cache_enabled=not self.graphs):
            flat = self.fn(self._cast_in(images), ctx)
        out, aux = FlatOutputs.unflatten(flat)
        losses = self.criterion(out, targets, num_boxes)
        loss = sum(losses.values()) + aux
        loss.backward()
        if self.graphs and self.world > 1:
            self._allreduce_grads()
        if self.lowp:
            self._grads_to_master()
        if self.clip_norm > 0:
            torch.nn.utils.clip_grad_norm_(self.opt_params, self.clip_norm, foreach=True)
        self.opt.step()
        if self.lowp:
            with torch.no_grad():
                torch._foreach_copy_(self.lowp, self.master)
        return loss.detach()
