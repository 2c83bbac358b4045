"""RT-DETR-MoE: PResNet-vd backbone -> HybridEncoder (AIFI with MoE FFN) ->
RT-DETR decoder (MoE FFN in every layer).  The engine behind the reference's
operator API (src/models/vision/rtdetr.py), built from a local spec string."""
from __future__ import annotations

import torch
from torch import nn

from ..moe.config import ModelSpec, parse_moe_spec
from ..moe.layer import MoEFFN
from .backbone import PResNet
from .decoder import RTDETRDecoder
from .encoder import HybridEncoder

_BACKBONE_DEPTH = {"r18": 18, "r34": 34, "r50": 50, "r101": 101}
_DEC_LAYERS = {"r18": 3, "r34": 4, "r50": 6, "r101": 6}


class RTDETRMoE(nn.Module):
    def __init__(self, spec: ModelSpec | str, num_classes: int = 1, freeze_norm: bool = True):
        super().__init__()
        if isinstance(spec, str):
            spec = parse_moe_spec(spec)
        self.spec = spec
        self.num_classes = num_classes
        depth = _BACKBONE_DEPTH[spec.backbone]
        self.backbone = PResNet(depth, return_idx=(1, 2, 3), freeze_norm=freeze_norm)
        self.encoder = HybridEncoder(in_channels=self.backbone.out_channels,
                                     strides=self.backbone.out_strides, moe=spec.moe,
                                     expansion=0.5 if depth < 50 else 1.0)
        nl = spec.num_decoder_layers or _DEC_LAYERS[spec.backbone]
        self.decoder = RTDETRDecoder(num_classes=num_classes, num_layers=nl, moe=spec.moe)

    @property
    def GFLOPs(self) -> float | None:
        """Forward GFLOPs of one 640x640 image (Ultralytics' convention):
        torch's FlopCounterMode for the dense ops + the routed expert FFNs and
        routers counted analytically (their HIP kernels are opaque to it)."""
        if getattr(self, "_gflops", None) is None:
            try:
                from torch.utils.flop_counter import FlopCounterMode

                dev = next(self.parameters()).device
                x = torch.zeros((1, 3, 640, 640), device=dev)
                saved = [m.__dict__.get("forward") for m in self.moe_layers()]
                for m in self.moe_layers():  # identity stand-in: count the dense body only
                    m.forward = (lambda x, ctx=None, residual=False: x)
                was = self.training
                self.eval()
                try:
                    with torch.no_grad(), FlopCounterMode(display=False) as fc:
                        self(x, None)
                finally:
                    for m, f in zip(self.moe_layers(), saved):
                        if f is None:
                            del m.forward
                        else:
                            m.forward = f
                    self.train(was)
                dense = fc.get_total_flops()
                moe = 0.0
                for i, m in enumerate(self.moe_layers()):
                    T = 400 if i == 0 else self.decoder.num_queries  # AIFI on S5 (20x20) / decoder queries
                    c = m.cfg
                    moe += T * (2 * m.d_model * c.num_experts + c.top_k * 4 * m.d_model * c.hidden)
                self._gflops = (dense + moe) / 1e9
            except Exception:
                return None
        return self._gflops

    @property
    def flops(self):
        return self.GFLOPs

    def train(self, mode: bool = True):
        """nn.Module.train, plus the inference re-parameterisation: entering
        eval mode folds the running-statistics BatchNorms (and each RepVgg
        block's 1x1 branch) into the convolutions (evalfold.refresh); entering
        training marks the folds stale."""
        super().train(mode)
        from . import evalfold

        if mode:
            evalfold.invalidate(self)
        else:
            evalfold.refresh(self)
        return self

    def moe_layers(self):
        return [m for m in self.modules() if isinstance(m, MoEFFN)]

    def forward(self, images: torch.Tensor, ctx_ids: torch.Tensor | None = None):
        feats = self.backbone(images)
        feats = self.encoder(feats, ctx_ids)
        return self.decoder(feats, ctx_ids)

    def moe_aux_loss(self):
        terms = [m.aux_loss() for m in self.moe_layers()]
        terms = [t for t in terms if t is not None]
        return torch.stack([t.float() for t in terms]).sum() if terms else None

    @torch.no_grad()
    def postprocess(self, outputs, orig_sizes, num_top=300):
        """Boxes in pixels (xyxy), scores, labels per image (RT-DETR postprocessor)."""
        logits = outputs["pred_logits"].float()
        boxes = outputs["pred_boxes"].float()
        B, Q, C = logits.shape
        scores = logits.sigmoid().flatten(1)
        k = min(num_top, Q * C)
        sc, idx = torch.topk(scores, k, dim=1)
        labels = idx % C
        qi = idx // C
        b = boxes.gather(1, qi[..., None].expand(-1, -1, 4))
        cx, cy, w, h = b.unbind(-1)
        xyxy = torch.stack([cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], -1)
        wh = torch.as_tensor(orig_sizes, dtype=xyxy.dtype, device=xyxy.device)  # [B, 2] (w, h)
        xyxy = xyxy * wh.repeat(1, 2)[:, None, :]
        return [{"boxes": xyxy[i], "scores": sc[i], "labels": labels[i]} for i in range(B)]
