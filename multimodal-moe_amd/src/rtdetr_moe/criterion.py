"""RT-DETR set criterion: Hungarian matching (focal class cost + L1 + GIoU),
varifocal classification loss, L1 and GIoU box losses, applied to the final
decoder output, every auxiliary decoder layer and the encoder's top-k
proposals.  (torchvision is absent in this image: the box ops are local.)"""
from __future__ import annotations

import numpy as np
import torch
from torch import nn
import torch.nn.functional as F

try:
    from scipy.optimize import linear_sum_assignment
except Exception:  # pragma: no cover
    linear_sum_assignment = None


def box_cxcywh_to_xyxy(b):
    cx, cy, w, h = b.unbind(-1)
    return torch.stack([cx - 0.5 * w, cy - 0.5 * h, cx + 0.5 * w, cy + 0.5 * h], -1)


def box_area(b):
    return (b[..., 2] - b[..., 0]).clamp(min=0) * (b[..., 3] - b[..., 1]).clamp(min=0)


def box_iou(a, b):
    """Pairwise IoU of xyxy boxes a [N,4], b [M,4] -> (iou [N,M], union)."""
    area_a, area_b = box_area(a), box_area(b)
    lt = torch.max(a[:, None, :2], b[None, :, :2])
    rb = torch.min(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    union = area_a[:, None] + area_b[None, :] - inter
    return inter / union.clamp(min=1e-9), union


def generalized_box_iou(a, b):
    iou, union = box_iou(a, b)
    lt = torch.min(a[:, None, :2], b[None, :, :2])
    rb = torch.max(a[:, None, 2:], b[None, :, 2:])
    wh = (rb - lt).clamp(min=0)
    area = wh[..., 0] * wh[..., 1]
    return iou - (area - union) / area.clamp(min=1e-9)


class HungarianMatcher(nn.Module):
    def __init__(self, cost_class=2.0, cost_bbox=5.0, cost_giou=2.0, alpha=0.25, gamma=2.0):
        super().__init__()
        self.cost_class, self.cost_bbox, self.cost_giou = cost_class, cost_bbox, cost_giou
        self.alpha, self.gamma = alpha, gamma

    @torch.no_grad()
    def forward(self, outputs, targets):
        return self.match_many([outputs], targets)[0]

    @torch.no_grad()
    def match_many(self, output_sets, targets):
        """Match several prediction sets (final, aux layers, encoder) with ONE
        device->host transfer of the stacked cost matrices."""
        sizes = [len(t["boxes"]) for t in targets]
        if sum(sizes) == 0:
            e = torch.empty(0, dtype=torch.int64)
            return [[(e, e) for _ in targets] for _ in output_sets]
        logits = torch.stack([o["pred_logits"].float() for o in output_sets])  # [S, B, Q, C]
        boxes = torch.stack([o["pred_boxes"].float() for o in output_sets])
        S, B, Q, _ = logits.shape
        prob = logits.flatten(0, 2).sigmoid()
        out_bbox = boxes.flatten(0, 2)
        tgt_ids = torch.cat([t["labels"] for t in targets])
        tgt_bbox = torch.cat([t["boxes"] for t in targets]).float()
        p = prob[:, tgt_ids]
        neg = (1 - self.alpha) * p ** self.gamma * (-(1 - p + 1e-8).log())
        pos = self.alpha * (1 - p) ** self.gamma * (-(p + 1e-8).log())
        c_class = pos - neg
        c_bbox = torch.cdist(out_bbox, tgt_bbox, p=1)
        c_giou = -generalized_box_iou(box_cxcywh_to_xyxy(out_bbox), box_cxcywh_to_xyxy(tgt_bbox))
        C = (self.cost_bbox * c_bbox + self.cost_class * c_class + self.cost_giou * c_giou)
        C = C.view(S, B, Q, -1).cpu()  # one host round trip for every set
        res = []
        for s in range(S):
            out = []
            for i, c in enumerate(C[s].split(sizes, -1)):
                if sizes[i] == 0:
                    e = torch.empty(0, dtype=torch.int64)
                    out.append((e, e))
                    continue
                r, col = linear_sum_assignment(c[i].numpy())
                out.append((torch.as_tensor(r, dtype=torch.int64), torch.as_tensor(col, dtype=torch.int64)))
            res.append(out)
        return res


class SetCriterion(nn.Module):
    def __init__(self, num_classes=1, weight_vfl=1.0, weight_bbox=5.0, weight_giou=2.0, alpha=0.75, gamma=2.0):
        super().__init__()
        self.num_classes = num_classes
        self.matcher = HungarianMatcher()
        self.w = {"loss_vfl": weight_vfl, "loss_bbox": weight_bbox, "loss_giou": weight_giou}
        self.alpha, self.gamma = alpha, gamma

    def _idx(self, indices, device):
        b = torch.cat([torch.full_like(s, i) for i, (s, _) in enumerate(indices)]).to(device)
        s = torch.cat([s for s, _ in indices]).to(device)
        return b, s

    def _losses(self, out, targets, indices, num_boxes):
        logits = out["pred_logits"].float()
        boxes = out["pred_boxes"].float()
        dev = logits.device
        bi, si = self._idx(indices, dev)
        tgt_boxes = torch.cat([t["boxes"][j] for t, (_, j) in zip(targets, indices)]).to(dev).float()
        tgt_cls = torch.cat([t["labels"][j] for t, (_, j) in zip(targets, indices)]).to(dev)
        src_boxes = boxes[bi, si]
        # boxes
        if tgt_boxes.numel():
            l1 = F.l1_loss(src_boxes, tgt_boxes, reduction="none").sum() / num_boxes
            giou = torch.diag(generalized_box_iou(box_cxcywh_to_xyxy(src_boxes), box_cxcywh_to_xyxy(tgt_boxes)))
            lg = (1 - giou).sum() / num_boxes
            ious = torch.diag(box_iou(box_cxcywh_to_xyxy(src_boxes.detach()), box_cxcywh_to_xyxy(tgt_boxes))[0])
        else:
            l1 = boxes.sum() * 0.0
            lg = boxes.sum() * 0.0
            ious = boxes.new_zeros(0)
        # varifocal
        target_classes = torch.full(logits.shape[:2], self.num_classes, dtype=torch.int64, device=dev)
        target_classes[bi, si] = tgt_cls
        target = F.one_hot(target_classes, self.num_classes + 1)[..., :-1].to(logits.dtype)
        score = torch.zeros(logits.shape[:2], dtype=logits.dtype, device=dev)
        score[bi, si] = ious.to(logits.dtype)
        target_score = score.unsqueeze(-1) * target
        pred_score = logits.sigmoid().detach()
        weight = self.alpha * pred_score.pow(self.gamma) * (1 - target) + target_score
        vfl = F.binary_cross_entropy_with_logits(logits, target_score, weight=weight, reduction="none")
        vfl = vfl.mean(1).sum() * logits.shape[1] / num_boxes
        return {"loss_vfl": vfl, "loss_bbox": l1, "loss_giou": lg}

    @staticmethod
    def _sets(outputs):
        sets = [("", outputs)] + [(f"_aux{i}", a) for i, a in enumerate(outputs.get("aux_outputs", []))]
        if "enc_outputs" in outputs:
            sets.append(("_enc", outputs["enc_outputs"]))
        return sets

    def forward_per_set(self, outputs, targets, num_boxes: float):
        """Reference formulation: one loss evaluation per prediction set."""
        losses = {}
        sets = self._sets(outputs)
        all_indices = self.matcher.match_many([o for _, o in sets], targets)
        for (suffix, out), indices in zip(sets, all_indices):
            for k, v in self._losses(out, targets, indices, num_boxes).items():
                losses[k + suffix] = v * self.w[k]
        return losses

    def forward(self, outputs, targets, num_boxes: float):
        """All prediction sets (final, auxiliary layers, encoder top-k) evaluated
        in one batched pass: the same losses as ``forward_per_set`` with ~S x
        fewer kernel launches (the step is launch-bound at these sizes)."""
        sets = self._sets(outputs)
        all_indices = self.matcher.match_many([o for _, o in sets], targets)
        logits = torch.stack([o["pred_logits"] for _, o in sets]).float()  # [S, B, Q, C]
        boxes = torch.stack([o["pred_boxes"] for _, o in sets]).float()    # [S, B, Q, 4]
        S, B, Q, C = logits.shape
        dev = logits.device
        sid, bid, qid, tid = [], [], [], []
        offs = [0]
        for t in targets:
            offs.append(offs[-1] + len(t["boxes"]))
        for s, indices in enumerate(all_indices):
            for b, (src, tgt) in enumerate(indices):
                n = len(src)
                if n:
                    sid.append(torch.full((n,), s, dtype=torch.int64))
                    bid.append(torch.full((n,), b, dtype=torch.int64))
                    qid.append(src)
                    tid.append(tgt + offs[b])
        tgt_all = torch.cat([t["boxes"] for t in targets]).to(dev).float() if offs[-1] else boxes.new_zeros((0, 4))
        cls_all = torch.cat([t["labels"] for t in targets]).to(dev) if offs[-1] else \
            torch.zeros(0, dtype=torch.int64, device=dev)
        score = torch.zeros((S, B, Q, C), dtype=logits.dtype, device=dev)
        if sid:
            idx = torch.stack([torch.cat(sid), torch.cat(bid), torch.cat(qid), torch.cat(tid)]).to(dev,
                                                                                                 non_blocking=True)
            si, bi, qi, ti = idx
            src = boxes[si, bi, qi]
            tgt = tgt_all[ti]
            sx, tx = box_cxcywh_to_xyxy(src), box_cxcywh_to_xyxy(tgt)
            iou, giou = _paired_iou_giou(sx, tx)
            l1 = torch.zeros(S, dtype=logits.dtype, device=dev).index_add_(0, si, (src - tgt).abs().sum(-1))
            lg = torch.zeros(S, dtype=logits.dtype, device=dev).index_add_(0, si, 1.0 - giou)
            score[si, bi, qi, cls_all[ti]] = iou.detach()
            onehot = torch.zeros_like(score)
            onehot[si, bi, qi, cls_all[ti]] = 1.0
        else:
            l1 = boxes.sum() * 0.0 + torch.zeros(S, device=dev)
            lg = l1.clone()
            onehot = torch.zeros_like(score)
        pred = logits.sigmoid().detach()
        weight = self.alpha * pred.pow(self.gamma) * (1 - onehot) + score
        vfl = F.binary_cross_entropy_with_logits(logits, score, weight=weight, reduction="none")
        vfl = vfl.mean(2).sum((1, 2)) * Q / num_boxes  # [S]
        l1 = l1 / num_boxes
        lg = lg / num_boxes
        losses = {}
        for s, (suffix, _) in enumerate(sets):
            losses["loss_vfl" + suffix] = vfl[s] * self.w["loss_vfl"]
            losses["loss_bbox" + suffix] = l1[s] * self.w["loss_bbox"]
            losses["loss_giou" + suffix] = lg[s] * self.w["loss_giou"]
        return losses


    def loss_padded(self, outputs, tgt_boxes, tgt_labels, n_valid, num_boxes, status):
        """Total weighted loss (differentiable scalar) and the per-set components
        {name: detached value} of ``forward_padded``, with the matching and the
        losses fused into HIP kernels (_SetLossHip).  GPU only; needs
        gamma == 2 and B*Q*C*4 bytes <= 64 KiB."""
        sets = self._sets(outputs)
        logits = torch.stack([o["pred_logits"] for _, o in sets]).float()
        boxes = torch.stack([o["pred_boxes"] for _, o in sets]).float()
        comps, _ = _SetLossHip.apply(logits, boxes, tgt_boxes, tgt_labels, n_valid, num_boxes, status, self.alpha)
        key = (comps.device, tuple(self.w.values()))
        w = getattr(self, "_wvec", None)
        if w is None or w[0] != key:
            w = (key, torch.tensor([self.w["loss_vfl"], self.w["loss_bbox"], self.w["loss_giou"]],
                                   dtype=torch.float32, device=comps.device))
            self._wvec = w
        weighted = comps * w[1]
        total = weighted.sum()
        det = weighted.detach()
        names = ["loss_vfl", "loss_bbox", "loss_giou"]
        parts = {n + suffix: det[s_, k] for s_, (suffix, _) in enumerate(sets) for k, n in enumerate(names)}
        return total, parts

    def fused_ok(self, outputs, M):
        lg = outputs["pred_logits"]
        B, Q, C = lg.shape
        return lg.is_cuda and self.gamma == 2.0 and B * Q * C * 4 <= 64 * 1024 and M <= 1024 and Q <= 4096

    def forward_padded(self, outputs, tgt_boxes, tgt_labels, n_valid, num_boxes, status=None):
        """The same losses as ``forward`` with fixed shapes and no host round
        trip, so the whole training step can be one hipGraph: targets padded to
        M per image (``tgt_boxes`` [B, M, 4] cxcywh, ``tgt_labels`` [B, M],
        ``n_valid`` int32 [B]; padding must be finite boxes), ``num_boxes`` a
        device scalar, and the Hungarian matching on the GPU
        (``rtdetr_hungarian_match``: scipy's linear_sum_assignment restated,
        same pairs).  ``status`` (int32 [1]) collects matcher failures."""
        from ..moe import _lib as L

        sets = self._sets(outputs)
        logits = torch.stack([o["pred_logits"] for _, o in sets]).float()  # [S, B, Q, C]
        boxes = torch.stack([o["pred_boxes"] for _, o in sets]).float()    # [S, B, Q, 4]
        S, B, Q, C = logits.shape
        M = tgt_boxes.shape[1]
        dev = logits.device
        tb = tgt_boxes.float()
        lab = tgt_labels.long().clamp(0, C - 1)
        valid = torch.arange(M, device=dev)[None, :] < n_valid[:, None]  # [B, M]
        m = self.matcher
        with torch.no_grad():  # matching cost (HungarianMatcher.match_many's, per image)
            p = logits.sigmoid().gather(3, lab[None, :, None, :].expand(S, B, Q, M))
            neg = (1 - m.alpha) * p ** m.gamma * (-(1 - p + 1e-8).log())
            pos = m.alpha * (1 - p) ** m.gamma * (-(p + 1e-8).log())
            c_bbox = (boxes[:, :, :, None, :] - tb[None, :, None, :, :]).abs().sum(-1)
            c_giou = -_pairwise_giou(box_cxcywh_to_xyxy(boxes)[:, :, :, None, :],
                                     box_cxcywh_to_xyxy(tb)[None, :, None, :, :])
            cost = m.cost_bbox * c_bbox + m.cost_class * (pos - neg) + m.cost_giou * c_giou
            assign = L.hungarian_match(cost.contiguous(), n_valid.to(torch.int32).contiguous(), status)
        q = assign.clamp(min=0).long()  # [S, B, M]
        mask = valid[None].expand(S, B, M).to(logits.dtype)
        src = boxes.gather(2, q[..., None].expand(S, B, M, 4))
        tgt = tb[None].expand(S, B, M, 4)
        iou, giou = _paired_iou_giou(box_cxcywh_to_xyxy(src).reshape(-1, 4), box_cxcywh_to_xyxy(tgt).reshape(-1, 4))
        iou, giou = iou.view(S, B, M), giou.view(S, B, M)
        l1 = ((src - tgt).abs().sum(-1) * mask).sum((1, 2)) / num_boxes
        lg = ((1.0 - giou) * mask).sum((1, 2)) / num_boxes
        # VFL targets: the padding writes into an extra query slot, sliced away
        qe = torch.where(valid[None], q, torch.full_like(q, Q))
        si = torch.arange(S, device=dev)[:, None, None].expand(S, B, M)
        bi = torch.arange(B, device=dev)[None, :, None].expand(S, B, M)
        ci = lab[None].expand(S, B, M)
        score = torch.zeros((S, B, Q + 1, C), dtype=logits.dtype, device=dev)
        onehot = torch.zeros_like(score)
        score.index_put_((si, bi, qe, ci), iou.detach() * mask)
        onehot.index_put_((si, bi, qe, ci), mask)
        score, onehot = score[:, :, :Q], onehot[:, :, :Q]
        pred = logits.sigmoid().detach()
        weight = self.alpha * pred.pow(self.gamma) * (1 - onehot) + score
        vfl = F.binary_cross_entropy_with_logits(logits, score, weight=weight, reduction="none")
        vfl = vfl.mean(2).sum((1, 2)) * Q / num_boxes  # [S]
        losses = {}
        for s_, (suffix, _) in enumerate(sets):
            losses["loss_vfl" + suffix] = vfl[s_] * self.w["loss_vfl"]
            losses["loss_bbox" + suffix] = l1[s_] * self.w["loss_bbox"]
            losses["loss_giou" + suffix] = lg[s_] * self.w["loss_giou"]
        return losses


class _SetLossHip(torch.autograd.Function):
    """Matching + VFL/L1/GIoU losses of all prediction sets in three HIP
    launches (rtdetr_set_criterion_match / _loss), their gradients computed in
    the same pass and scaled in the backward (rtdetr_set_criterion_loss_bwd)."""

    @staticmethod
    def forward(ctx, logits, boxes, tgt_boxes, tgt_labels, n_valid, num_boxes, status, vfl_alpha):
        from ..moe import _lib as L

        S, B, Q, C = logits.shape
        M = tgt_boxes.shape[1]
        lg, bx = logits.contiguous(), boxes.contiguous()
        tb, tl, nv = tgt_boxes.float().contiguous(), tgt_labels.to(torch.int32).contiguous(), n_valid.contiguous()
        nb = num_boxes.float().reshape(1).contiguous()
        assign = torch.empty((S, B, M), dtype=torch.int32, device=lg.device)
        s = L._stream()
        L._check(L.lib().rtdetr_set_criterion_match(lg.data_ptr(), bx.data_ptr(), tb.data_ptr(), tl.data_ptr(),
                                                    nv.data_ptr(), S, B, Q, C, M, assign.data_ptr(),
                                                    status.data_ptr(), s), "rtdetr_set_criterion_match")
        comps = torch.empty((S, 3), dtype=torch.float32, device=lg.device)
        d_lg = torch.empty_like(lg)
        d_l1 = torch.empty_like(bx)
        d_gi = torch.empty_like(bx)
        L._check(L.lib().rtdetr_set_criterion_loss(lg.data_ptr(), bx.data_ptr(), tb.data_ptr(), tl.data_ptr(),
                                                   nv.data_ptr(), assign.data_ptr(), nb.data_ptr(), float(vfl_alpha),
                                                   S, B, Q, C, M, comps.data_ptr(), d_lg.data_ptr(),
                                                   d_l1.data_ptr(), d_gi.data_ptr(), s), "rtdetr_set_criterion_loss")
        ctx.save_for_backward(d_lg, d_l1, d_gi)
        ctx.mark_non_differentiable(assign)
        return comps, assign

    @staticmethod
    def backward(ctx, g_comps, _g_assign):
        from ..moe import _lib as L

        d_lg, d_l1, d_gi = ctx.saved_tensors
        S, B, Q, C = d_lg.shape
        g = g_comps.float().contiguous()
        g_lg = torch.empty_like(d_lg)
        g_bx = torch.empty_like(d_l1)
        L._check(L.lib().rtdetr_set_criterion_loss_bwd(g.data_ptr(), S, B, Q, C, d_lg.data_ptr(), d_l1.data_ptr(),
                                                       d_gi.data_ptr(), g_lg.data_ptr(), g_bx.data_ptr(),
                                                       L._stream()), "rtdetr_set_criterion_loss_bwd")
        return g_lg, g_bx, None, None, None, None, None, None


PAD_BOX = (0.5, 0.5, 0.1, 0.1)  # finite stand-in for padded target slots (masked out of every loss)


def pad_targets(targets, M, boxes_out=None, labels_out=None, n_valid_out=None):
    """Targets (list of {"boxes" [n,4], "labels" [n]}) -> padded device tensors
    ([B, M, 4], [B, M], int32 [B]) for ``SetCriterion.forward_padded``; writes
    into the given static buffers when passed (graph replay)."""
    B = len(targets)
    dev = targets[0]["boxes"].device if B else torch.device("cpu")
    if boxes_out is None:
        boxes_out = torch.empty((B, M, 4), dtype=torch.float32, device=dev)
        labels_out = torch.empty((B, M), dtype=torch.int64, device=dev)
        n_valid_out = torch.empty(B, dtype=torch.int32, device=dev)
    counts = [len(t["boxes"]) for t in targets]
    if max(counts, default=0) > M:
        raise ValueError(f"pad_targets: {max(counts)} boxes in one image exceed the padded capacity {M}")
    boxes_out[..., :2] = PAD_BOX[0]
    boxes_out[..., 2:] = PAD_BOX[2]
    labels_out.zero_()
    for b, t in enumerate(targets):
        n = counts[b]
        if n:
            boxes_out[b, :n].copy_(t["boxes"])
            labels_out[b, :n].copy_(t["labels"])
    host = torch.tensor(counts, dtype=torch.int32)
    if n_valid_out.is_cuda:  # pinned staging: the copy does not wait for the stream
        host = host.pin_memory()
    n_valid_out.copy_(host, non_blocking=True)
    return boxes_out, labels_out, n_valid_out


def _pairwise_giou(a, b):
    """GIoU of broadcast xyxy boxes a[..., 4], b[..., 4]."""
    lt = torch.max(a[..., :2], b[..., :2])
    rb = torch.min(a[..., 2:], b[..., 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[..., 0] * wh[..., 1]
    union = box_area(a) + box_area(b) - inter
    iou = inter / union.clamp(min=1e-9)
    lt2 = torch.min(a[..., :2], b[..., :2])
    rb2 = torch.max(a[..., 2:], b[..., 2:])
    wh2 = (rb2 - lt2).clamp(min=0)
    area = wh2[..., 0] * wh2[..., 1]
    return iou - (area - union) / area.clamp(min=1e-9)


def _paired_iou_giou(a, b):
    """IoU and GIoU of paired xyxy boxes a[i], b[i]."""
    lt = torch.max(a[:, :2], b[:, :2])
    rb = torch.min(a[:, 2:], b[:, 2:])
    wh = (rb - lt).clamp(min=0)
    inter = wh[:, 0] * wh[:, 1]
    union = box_area(a) + box_area(b) - inter
    iou = inter / union.clamp(min=1e-9)
    lt2 = torch.min(a[:, :2], b[:, :2])
    rb2 = torch.max(a[:, 2:], b[:, 2:])
    wh2 = (rb2 - lt2).clamp(min=0)
    area = wh2[:, 0] * wh2[:, 1]
    return iou, iou - (area - union) / area.clamp(min=1e-9)


def targets_to_device(targets, device):
    return [{k: (v.to(device, non_blocking=True) if torch.is_tensor(v) else v) for k, v in t.items()}
            for t in targets]


def count_boxes(targets) -> int:
    return int(sum(len(t["boxes"]) for t in targets))


def as_numpy_boxes(t):
    return np.asarray(t["boxes"].detach().cpu().numpy(), dtype=np.float64)
