"""Detection metrics computed in-house (pycocotools / faster_coco_eval are
absent here).  Produces what the reference's serializer
reads from an Ultralytics metrics object (src/models/vision/yolo.py:204-300):
``results_dict`` keys ``metrics/{precision,recall,mAP50,mAP50-95}(B)``,
``box.{map50,map,mp,mr,curves,curves_results}`` and ``speed``.

AP per class: predictions matched greedily by descending score to unmatched
ground truth of the same class at IoU thresholds 0.50:0.05:0.95; AP is the
area under the monotone precision envelope sampled at 101 recall points
(COCO interpolation, pycocotools' accumulate).  P and R are reported at the confidence that maximises
the class-mean F1 (Ultralytics convention).
"""
from __future__ import annotations

from dataclasses import dataclass, field

import numpy as np

IOU_THRESHOLDS = np.linspace(0.5, 0.95, 10)


def box_iou_np(a: np.ndarray, b: np.ndarray) -> np.ndarray:
    if len(a) == 0 or len(b) == 0:
        return np.zeros((len(a), len(b)))
    lt = np.maximum(a[:, None, :2], b[None, :, :2])
    rb = np.minimum(a[:, None, 2:], b[None, :, 2:])
    wh = np.clip(rb - lt, 0, None)
    inter = wh[..., 0] * wh[..., 1]
    area_a = np.prod(np.clip(a[:, 2:] - a[:, :2], 0, None), 1)
    area_b = np.prod(np.clip(b[:, 2:] - b[:, :2], 0, None), 1)
    return inter / np.maximum(area_a[:, None] + area_b[None] - inter, 1e-9)


def match_predictions(pred_boxes, pred_scores, pred_labels, gt_boxes, gt_labels, iouv=IOU_THRESHOLDS):
    """tp [n_pred, n_thr] (bool) for one image."""
    n = len(pred_boxes)
    tp = np.zeros((n, len(iouv)), dtype=bool)
    if n == 0 or len(gt_boxes) == 0:
        return tp
    iou = box_iou_np(pred_boxes, gt_boxes)
    same = pred_labels[:, None] == gt_labels[None, :]
    order = np.argsort(-pred_scores, kind="stable")
    for ti, thr in enumerate(iouv):
        taken = np.zeros(len(gt_boxes), dtype=bool)
        for i in order:
            cand = np.where(same[i] & ~taken & (iou[i] >= thr))[0]
            if len(cand):
                j = cand[np.argmax(iou[i, cand])]
                taken[j] = True
                tp[i, ti] = True
    return tp


def _ap(recall, precision):
    """COCO 101-point AP: mean over recall thresholds r of the best precision
    at any recall >= r (0 where r is never reached)."""
    if len(recall) == 0:
        return 0.0
    env = np.flip(np.maximum.accumulate(np.flip(precision)))
    rs = np.linspace(0, 1, 101)
    inds = np.searchsorted(recall, rs, side="left")
    q = np.where(inds < len(env), env[np.minimum(inds, len(env) - 1)], 0.0)
    return float(q.mean())


def ap_per_class(tp, conf, pred_cls, target_cls, eps=1e-16):
    """Returns dict(p, r, f1, ap [nc, n_thr], classes, px, curves) over the dataset."""
    order = np.argsort(-conf, kind="stable")
    tp, conf, pred_cls = tp[order], conf[order], pred_cls[order]
    classes = np.unique(target_cls) if len(target_cls) else np.unique(pred_cls)
    nc = len(classes)
    px = np.linspace(0, 1, 1000)
    ap = np.zeros((nc, tp.shape[1]))
    p_curve = np.zeros((nc, 1000))
    r_curve = np.zeros((nc, 1000))
    pr_curve = np.zeros((nc, 1000))
    for ci, c in enumerate(classes):
        sel = pred_cls == c
        n_l = int((target_cls == c).sum())
        n_p = int(sel.sum())
        if n_p == 0 or n_l == 0:
            continue
        fpc = (1 - tp[sel]).cumsum(0)
        tpc = tp[sel].cumsum(0)
        recall = tpc / (n_l + eps)
        precision = tpc / (tpc + fpc)
        r_curve[ci] = np.interp(-px, -conf[sel], recall[:, 0], left=0)
        p_curve[ci] = np.interp(-px, -conf[sel], precision[:, 0], left=1)
        for j in range(tp.shape[1]):
            ap[ci, j] = _ap(recall[:, j], precision[:, j])
        # PR curve at IoU 0.5 on the recall grid
        mrec = np.concatenate([[0.0], recall[:, 0], [1.0]])
        mpre = np.flip(np.maximum.accumulate(np.flip(np.concatenate([[1.0], precision[:, 0], [0.0]]))))
        pr_curve[ci] = np.interp(px, mrec, mpre)
    f1 = 2 * p_curve * r_curve / (p_curve + r_curve + eps)
    i = int(np.argmax(f1.mean(0))) if nc else 0
    return dict(p=p_curve[:, i], r=r_curve[:, i], f1=f1[:, i], ap=ap, classes=classes, px=px,
                p_curve=p_curve, r_curve=r_curve, f1_curve=f1, pr_curve=pr_curve)


@dataclass
class BoxMetrics:
    """Mirror of the attributes the reference reads from ``metrics.box``."""
    mp: float = 0.0
    mr: float = 0.0
    map50: float = 0.0
    map: float = 0.0
    curves: list = field(default_factory=lambda: ["Precision-Recall(B)", "F1-Confidence(B)",
                                                  "Precision-Confidence(B)", "Recall-Confidence(B)"])
    curves_results: list = field(default_factory=list)


class DetectionEvaluator:
    """Accumulates per-image matches, then reduces to dataset metrics."""

    def __init__(self):
        self.tp, self.conf, self.pred_cls, self.target_cls = [], [], [], []

    def update(self, pred_boxes, pred_scores, pred_labels, gt_boxes, gt_labels, conf_thres=0.001):
        keep = pred_scores >= conf_thres
        pb, ps, pl = pred_boxes[keep], pred_scores[keep], pred_labels[keep]
        self.tp.append(match_predictions(pb, ps, pl, gt_boxes, gt_labels))
        self.conf.append(ps)
        self.pred_cls.append(pl)
        self.target_cls.append(gt_labels)

    def average_recall(self, max_det: int = 100) -> float:
        """COCO AR@max_det (all classes, area "all"): per image the max_det
        highest-scoring detections, recall at each IoU threshold of
        IOU_THRESHOLDS, averaged over thresholds (and classes present)."""
        n_gt = {}
        for tc in self.target_cls:
            for c in np.asarray(tc).reshape(-1).tolist():
                n_gt[int(c)] = n_gt.get(int(c), 0) + 1
        if not n_gt:
            return -1.0
        hits = {c: np.zeros(len(IOU_THRESHOLDS)) for c in n_gt}
        for tp, conf, pc in zip(self.tp, self.conf, self.pred_cls):
            order = np.argsort(-np.asarray(conf), kind="stable")[:max_det]
            for j in order:
                c = int(pc[j])
                if c in hits:
                    hits[c] += np.asarray(tp[j], dtype=np.float64)
        return float(np.mean([(hits[c] / n_gt[c]).mean() for c in n_gt]))

    def compute(self) -> BoxMetrics:
        cat = lambda xs, d: np.concatenate(xs, 0) if xs else np.zeros((0,) + d)  # noqa: E731
        tp = cat(self.tp, (len(IOU_THRESHOLDS),))
        conf = cat(self.conf, ())
        pred_cls = cat(self.pred_cls, ())
        target_cls = cat(self.target_cls, ())
        box = BoxMetrics()
        if len(target_cls) == 0:
            return box
        if len(conf) == 0:
            px = np.linspace(0, 1, 1000)
            zero = np.zeros((1, 1000))
            box.curves_results = [[px, zero, "Recall", "Precision"], [px, zero, "Confidence", "F1"],
                                  [px, zero, "Confidence", "Precision"], [px, zero, "Confidence", "Recall"]]
            return box
        r = ap_per_class(tp.astype(np.float64), conf, pred_cls, target_cls)
        box.mp = float(r["p"].mean())
        box.mr = float(r["r"].mean())
        box.map50 = float(r["ap"][:, 0].mean())
        box.map = float(r["ap"].mean())
        box.curves_results = [[r["px"], r["pr_curve"], "Recall", "Precision"],
                              [r["px"], r["f1_curve"], "Confidence", "F1"],
                              [r["px"], r["p_curve"], "Confidence", "Precision"],
                              [r["px"], r["r_curve"], "Confidence", "Recall"]]
        return box
