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
