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
