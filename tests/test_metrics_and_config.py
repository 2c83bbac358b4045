from __future__ import annotations

import numpy as np
import pytest


def test_map_perfect_and_shifted():
    from src.rtdetr_moe.metrics import DetectionEvaluator

    rng = np.random.default_rng(0)
    ev = DetectionEvaluator()
    ev_bad = DetectionEvaluator()
    for _ in range(5):
        n = rng.integers(1, 6)
        xy = rng.uniform(0, 500, (n, 2))
        gt = np.concatenate([xy, xy + rng.uniform(20, 80, (n, 2))], 1)
        lab = np.zeros(n, np.int64)
        ev.update(gt, np.linspace(0.9, 0.5, n), lab, gt, lab)
        ev_bad.update(gt + 15.0, np.linspace(0.9, 0.5, n), lab, gt, lab)
    m = ev.compute()
    assert m.map50 == pytest.approx(1.0, abs=1e-6) and m.map == pytest.approx(1.0, abs=1e-6)
    assert m.mp == pytest.approx(1.0) and m.mr == pytest.approx(1.0)
    b = ev_bad.compute()
    assert b.map < m.map


def _ev(images):
    """images: list of (pred_boxes, scores, labels, gt_boxes, gt_labels)."""
    from src.rtdetr_moe.metrics import DetectionEvaluator

    ev = DetectionEvaluator()
    for pb, ps, pl, gb, gl in images:
        ev.update(np.asarray(pb, float).reshape(-1, 4), np.asarray(ps, float), np.asarray(pl, np.int64),
                  np.asarray(gb, float).reshape(-1, 4), np.asarray(gl, np.int64))
    return ev.compute()


# Known answers worked by hand with the COCO rules (pycocotools evaluateImg /
# accumulate): detections sorted by score (stable, image order breaks ties),
# each matched to the best-IoU unmatched GT of its class at IoU >= t, AP the
# mean over 101 recall points of the precision envelope, classes without GT
# excluded and classes with GT but no detections scoring 0.
GT = [0.0, 0.0, 10.0, 10.0]


def test_map_duplicate_detection():
    # 0.9: IoU 0.625 with the GT (TP at t <= 0.6, FP above); 0.8: exact (FP while
    # the GT is taken, TP once the first one misses) -> AP 1 at 3 thresholds, 0.5 at 7
    m = _ev([([[0, 0, 10, 6.25], GT], [0.9, 0.8], [0, 0], [GT], [0])])
    assert m.map50 == pytest.approx(1.0)
    assert m.map == pytest.approx((3 * 1.0 + 7 * 0.5) / 10)


def test_map_score_ties_break_in_image_order():
    far = [50.0, 50.0, 60.0, 60.0]
    # image 0: FP at 0.7 and TP at 0.5; image 1: TP at 0.7 (ties the FP)
    # sorted: FP, TP, TP -> precision [0, .5, .667], recall [0, .5, 1] -> AP 2/3
    a = _ev([([far, GT], [0.7, 0.5], [0, 0], [GT], [0]), ([GT], [0.7], [0], [GT], [0])])
    assert a.map50 == pytest.approx(2 / 3) and a.map == pytest.approx(2 / 3)
    # images swapped: TP, FP, TP -> envelope 1 up to recall .5 (51 points), 2/3 after (50)
    b = _ev([([GT], [0.7], [0], [GT], [0]), ([far, GT], [0.7, 0.5], [0, 0], [GT], [0])])
    assert b.map50 == pytest.approx((51 + 50 * 2 / 3) / 101)


def test_map_crowded_duplicate_ground_truth():
    # two identical GT boxes, one detection: recall caps at 0.5 -> 51 of 101 points
    m = _ev([([GT], [0.9], [0], [GT, GT], [0, 0])])
    assert m.map50 == pytest.approx(51 / 101) and m.map == pytest.approx(51 / 101)
    assert m.mr == pytest.approx(0.5)


def test_map_multi_class_multi_image():
    g2 = [20.0, 20.0, 40.0, 30.0]
    imgs = [
        # class 0 perfect over two images
        ([GT], [0.9], [0], [GT], [0]),
        ([g2, g2], [0.8, 0.6], [0, 1], [g2, g2], [0, 1]),
        # class 1: a higher-scored FP before its TP -> AP 0.5; class 2: GT, no detections -> 0
        ([[70, 70, 80, 80], [100, 0, 110, 10]], [0.95, 0.3], [1, 1], [[100, 0, 110, 10]], [2]),
        # class 3: detections but no GT -> excluded from the mean
        ([[0, 50, 10, 60]], [0.99], [3], [], []),
    ]
    m = _ev(imgs)
    # class 1: 0.95 FP (no class-1 GT in image 2), 0.6 TP -> precision [0, .5], recall [0, 1]
    # class 2 in image 2 gets no class-2 detection -> AP 0
    assert m.map50 == pytest.approx((1.0 + 0.5 + 0.0) / 3)
    assert m.map == pytest.approx((1.0 + 0.5 + 0.0) / 3)


def test_map_empty_inputs():
    m = _ev([([], [], [], [GT], [0])])
    assert m.map == 0.0 and m.map50 == 0.0 and len(m.curves_results) == 4
    m = _ev([([GT], [0.9], [0], [], [])])  # no ground truth anywhere
    assert m.map == 0.0 and m.mp == 0.0


@pytest.mark.parametrize("spec,E,k,cf,bb", [
    ("rtdetr-r50-moe8-top2", 8, 2, 0.0, "r50"),
    ("rtdetr-r18-moe4-top1", 4, 1, 0.0, "r18"),
    ("rtdetr-r50-moe32-top4-cf1.25-fp8", 32, 4, 1.25, "r50"),
])
def test_spec_parsing(spec, E, k, cf, bb):
    from src.moe.config import parse_moe_spec

    s = parse_moe_spec(spec)
    assert (s.backbone, s.moe.num_experts, s.moe.top_k, s.moe.capacity_factor) == (bb, E, k, cf)


def test_dense_spec_and_errors():
    from src.moe.config import parse_moe_spec

    assert parse_moe_spec("rtdetr-r50").moe is None
    with pytest.raises(ValueError):
        parse_moe_spec("rtdetr-l.pt")
    with pytest.raises(ValueError):
        parse_moe_spec("rtdetr-r50-moe2-top4")


def test_capacity_formula():
    from src.moe.config import MoEConfig

    c = MoEConfig(num_experts=32, top_k=4, capacity_factor=1.25)
    assert c.capacity(14720) == 2300  # C5 enc cap at cf 1.25


def test_batched_criterion_matches_per_set():
    import torch
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.data import SyntheticZOD

    torch.manual_seed(0)
    B, Q, S = 3, 50, 4
    _, targets, _ = SyntheticZOD(batch=B, img_h=256, img_w=256, seed=3).sample()
    def mk():
        return {"pred_logits": torch.randn(B, Q, 1, requires_grad=True),
                "pred_boxes": torch.rand(B, Q, 4).mul(0.5).add(0.1).requires_grad_(True)}
    outs = [mk() for _ in range(S)]
    out = dict(outs[0], aux_outputs=outs[1:-1], enc_outputs=outs[-1])
    crit = SetCriterion()
    nb = max(1.0, float(sum(len(t["boxes"]) for t in targets)))
    a = crit(out, targets, nb)
    b = crit.forward_per_set(out, targets, nb)
    assert a.keys() == b.keys()
    for k in a:
        torch.testing.assert_close(a[k], b[k], rtol=1e-5, atol=1e-6, msg=k)
    ga = torch.autograd.grad(sum(a.values()), [o["pred_logits"] for o in outs] + [o["pred_boxes"] for o in outs])
    gb = torch.autograd.grad(sum(b.values()), [o["pred_logits"] for o in outs] + [o["pred_boxes"] for o in outs])
    for x, y in zip(ga, gb):
        torch.testing.assert_close(x, y, rtol=1e-5, atol=1e-6)
