"""The fused ReLU MLP heads (linear._MLPHip: grouped-GEMM bias + ReLU
epilogue forward, the ReLU mask in the next layer's data-gradient epilogue)
against the per-layer path (TokenLinear + F.relu) on the detector's shapes:
box head 256 -> 256 -> 256 -> 4 and query-position head 4 -> 512 -> 256.
Both accumulate in fp32 and round each layer's output to bf16 once, so the
outputs and gradients agree to bf16 rounding (tolerance: 2e-2 relative
Frobenius on outputs and every gradient, the dense-GEMM tolerance of the
other TokenLinear tests)."""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.mark.parametrize("dims,rows,input_grad", [((256, 256, 4, 3), 2400, True), ((4, 512, 256, 2), 2400, False),
                                                  ((256, 256, 4, 3), 77, True)])
def test_fused_mlp_matches_per_layer(hip_lib, monkeypatch, dims, rows, input_grad):
    from src.rtdetr_moe import decoder as D

    torch.manual_seed(1)
    mlp = D.MLP(*dims).to(DEV).to(torch.bfloat16)
    x = torch.randn(rows, dims[0], device=DEV).to(torch.bfloat16)
    gy = torch.randn(rows, dims[2], device=DEV).to(torch.bfloat16)
    res = []
    for fused in (True, False):
        monkeypatch.setattr(D, "_FUSED_MLP", fused)
        mlp.zero_grad(set_to_none=True)
        xi = x.clone().requires_grad_(input_grad)
        y = mlp(xi)
        (y.float() * gy.float()).sum().backward()
        grads = [p.grad.float().clone() for p in mlp.parameters()]
        res.append((y.float(), xi.grad.float() if input_grad else None, grads))
    (ya, gxa, ga), (yb, gxb, gb) = res

    def rel(a, b):
        return float((a - b).norm() / b.norm().clamp_min(1e-12))

    assert rel(ya, yb) < 2e-2
    if input_grad:
        assert rel(gxa, gxb) < 2e-2
    for a, b in zip(ga, gb):
        assert rel(a, b) < 2e-2, rel(a, b)
