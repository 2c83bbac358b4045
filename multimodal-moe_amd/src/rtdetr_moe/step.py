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


class TrainStep:
    def __init__(self, model: RTDETRMoE, criterion, images, ctx, *, lr=1e-4, lr_backbone=1e-5,
                 weight_decay=1e-4, clip_norm=0.1, graphs=True, ddp_local=None, world=1):
        self.model = model
        self.criterion = criterion
        self.clip_norm = clip_norm
        self.world = world
        self.graphs = graphs
        self.params = [p for p in model.parameters() if p.requires_grad]
        bb = [p for n, p in model.named_parameters() if n.startswith("backbone.") and p.requires_grad]
        rest = [p for n, p in model.named_parameters() if not n.startswith("backbone.") and p.requires_grad]
        fused = images.is_cuda
        self.opt = torch.optim.AdamW([{"params": bb, "lr": lr_backbone}, {"params": rest, "lr": lr}], lr=lr,
                                     weight_decay=weight_decay, fused=fused)
        self.flat = FlatOutputs(model)
        self.dp_params = [p for p in self.params if not getattr(p, "expert_parallel", False)]
        if graphs:
            with torch.autocast("cuda", dtype=torch.bfloat16, cache_enabled=False):
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
        self.opt.zero_grad(set_to_none=True)
        with torch.autocast(images.device.type, dtype=torch.bfloat16, enabled=images.is_cuda,
                            cache_enabled=not self.graphs):
            flat = self.fn(images, ctx)
        out, aux = FlatOutputs.unflatten(flat)
        losses = self.criterion(out, targets, num_boxes)
        loss = sum(losses.values()) + aux
        loss.backward()
        if self.graphs and self.world > 1:
            self._allreduce_grads()
        if self.clip_norm > 0:
            torch.nn.utils.clip_grad_norm_(self.params, self.clip_norm, foreach=True)
        self.opt.step()
        return loss.detach()
