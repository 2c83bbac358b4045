"""GPU Hungarian matching (csrc/matcher.hip) against scipy's
linear_sum_assignment -- the matcher the reference's RT-DETR loss runs
(Ultralytics / RT-DETRv2 HungarianMatcher).  Bit-exact: the same pairs,
including tie-heavy integer costs where many optima exist."""
from __future__ import annotations

import numpy as np
import pytest
import torch
from scipy.optimize import linear_sum_assignment

DEV = "cuda"


def _check(cost, n_valid):
    from src.moe import _lib as L

    c = torch.from_numpy(cost).to(DEV)
    nv = torch.from_numpy(n_valid).to(DEV)
    status = torch.zeros(1, dtype=torch.int32, device=DEV)
    got = L.hungarian_match(c, nv, status).cpu().numpy()
    assert int(status.item()) == 0
    S, B, Q, M = cost.shape
    for s in range(S):
        for b in range(B):
            n = int(n_valid[b])
            assert (got[s, b, n:] == -1).all()
            if n == 0:
                continue
            r, col = linear_sum_assignment(cost[s, b, :, :n])
            want = np.full(n, -1)
            want[col] = r
            np.testing.assert_array_equal(got[s, b, :n], want, err_msg=f"set {s} image {b} n={n}")


@pytest.mark.gpu
@pytest.mark.parametrize("ties", [False, True])
@pytest.mark.parametrize("Q,M", [(300, 16), (40, 40), (7, 8)])
def test_hungarian_matches_scipy(hip_lib, ties, Q, M):
    rng = np.random.default_rng(Q * 7 + M + ties)
    S, B = 3, 6
    if ties:
        cost = rng.integers(0, 4, size=(S, B, Q, M)).astype(np.float32)
    else:
        cost = rng.standard_normal((S, B, Q, M)).astype(np.float32) * 3
    n_valid = np.array([0, 1, min(Q, M), min(5, Q, M), min(M, Q) // 2, min(3, Q)], dtype=np.int32)
    _check(cost, n_valid)


@pytest.mark.gpu
def test_hungarian_rtdetr_cost(hip_lib):
    """Costs shaped like the criterion's (focal + 5 L1 + 2 GIoU), 7 sets x 8
    images x 300 queries x up to 24 boxes."""
    from src.rtdetr_moe.criterion import box_cxcywh_to_xyxy, generalized_box_iou

    g = torch.Generator().manual_seed(3)
    S, B, Q, M = 7, 8, 300, 24
    logits = torch.randn(S, B, Q, generator=g)
    boxes = torch.rand(S, B, Q, 4, generator=g) * 0.5 + 0.2
    tgt = torch.rand(B, M, 4, generator=g) * 0.5 + 0.2
    p = logits.sigmoid()
    c_cls = 0.25 * (1 - p) ** 2 * (-(p + 1e-8).log()) - 0.75 * p ** 2 * (-(1 - p + 1e-8).log())
    cost = torch.empty(S, B, Q, M)
    for s in range(S):
        for b in range(B):
            c_l1 = torch.cdist(boxes[s, b], tgt[b], p=1)
            c_giou = -generalized_box_iou(box_cxcywh_to_xyxy(boxes[s, b]), box_cxcywh_to_xyxy(tgt[b]))
            cost[s, b] = 5 * c_l1 + 2 * c_cls[s, b][:, None] + 2 * c_giou
    n_valid = np.array([0, 3, 24, 1, 17, 9, 2, 5], dtype=np.int32)
    _check(cost.numpy(), n_valid)
