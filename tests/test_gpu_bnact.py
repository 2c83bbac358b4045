"""Training-mode BatchNorm + SiLU of the HybridEncoder (fused.bn_act over
libmoe_hip's rtdetr_bn_act_fwd/_bwd) against torch.nn.BatchNorm2d in fp32 on
the same bf16 inputs.  Tolerances: y and dx are bf16 (one rounding of an fp32
value: rtol 1e-2, atol 2e-2 relative to the tensor scale); batch statistics,
running statistics, dgamma and dbeta are fp32 reductions of the same inputs
(rtol 1e-4, atol 1e-5 x scale)."""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cl(t):
    return t.to(DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def _bns(nb, C, g):
    out = []
    for _ in range(nb):
        bn = torch.nn.BatchNorm2d(C).to(DEV)
        with torch.no_grad():
            bn.weight.copy_(torch.rand(C, generator=g) + 0.5)
            bn.bias.copy_(torch.randn(C, generator=g) * 0.3)
            bn.running_mean.copy_(torch.randn(C, generator=g) * 0.1)
            bn.running_var.copy_(torch.rand(C, generator=g) + 0.5)
        out.append(bn)
    return out


@pytest.mark.parametrize("nb,act", [(1, "silu"), (2, "silu"), (1, None)])
@pytest.mark.parametrize("shape", [(2, 256, 23, 40), (8, 256, 46, 80), (3, 64, 7, 9)])
def test_bn_act_matches_torch(hip_lib, nb, act, shape):
    import copy

    from src.rtdetr_moe.fused import bn_act, bn_act_ok

    g = torch.Generator().manual_seed(hash((nb, act, shape)) % 1000)
    N, C, H, W = shape
    xs = [_cl(torch.randn(shape, generator=g) * 1.7 + 0.4) for _ in range(nb)]
    bns = _bns(nb, C, g)
    ref_bns = copy.deepcopy(bns)
    dy = _cl(torch.randn(shape, generator=g))
    assert bn_act_ok(xs, bns)
    xg = [x.clone().requires_grad_(True) for x in xs]
    y = bn_act(xg, bns, act)
    y.backward(dy)
    # fp32 reference on the same (bf16-valued) inputs
    xr = [x.float().requires_grad_(True) for x in xs]
    z = sum(bn(x) for bn, x in zip(ref_bns, xr))
    yr = F.silu(z) if act == "silu" else z
    yr.backward(dy.float())
    scale = yr.abs().max().item()
    torch.testing.assert_close(y.float(), yr.detach(), rtol=1e-2, atol=2e-2 * scale)
    for a, b in zip(xg, xr):
        s = b.grad.abs().max().item()
        torch.testing.assert_close(a.grad.float(), b.grad, rtol=1e-2, atol=2e-2 * s)
    for bn, rb in zip(bns, ref_bns):
        for name in ("running_mean", "running_var"):
            torch.testing.assert_close(getattr(bn, name), getattr(rb, name), rtol=1e-4, atol=1e-5)
        for name in ("weight", "bias"):
            ga, gb = getattr(bn, name).grad, getattr(rb, name).grad
            torch.testing.assert_close(ga, gb, rtol=1e-4, atol=1e-5 * gb.abs().max().item())


def test_bn_act_deterministic(hip_lib):
    from src.moe import _lib as L

    g = torch.Generator().manual_seed(1)
    shape = (8, 256, 92, 160)
    xs = [_cl(torch.randn(shape, generator=g)) for _ in range(2)]
    gam = [torch.rand(256, generator=g).to(DEV) + 0.5 for _ in range(2)]
    bet = [torch.randn(256, generator=g).to(DEV) for _ in range(2)]
    dy = _cl(torch.randn(shape, generator=g))
    runs = []
    for _ in range(2):
        y, saved = L.bn_act_fwd(xs, gam, bet, [None, None], [None, None], 1, 1e-5, 0.1)
        dxs, dgb = L.bn_act_bwd(dy, xs, gam, saved, 1)
        runs.append((y, saved, dxs[0], dxs[1], dgb))
    for a, b in zip(*runs):
        assert torch.equal(a, b)


def test_encoder_fused_bn_matches_unfused(hip_lib, monkeypatch):
    """One CSPRepLayer (RepVgg blocks + ConvNormLayer silu) forward/backward with
    the fused BN path vs torch's BN path: same loss and gradients within bf16
    tolerance."""
    import copy

    from src.rtdetr_moe import backbone, encoder

    torch.manual_seed(0)
    layer = encoder.CSPRepLayer(256, 256, num_blocks=3).to(DEV)
    for m in layer.modules():
        if isinstance(m, torch.nn.Conv2d):
            m.to(torch.bfloat16)
    layer = layer.to(memory_format=torch.channels_last)
    ref = copy.deepcopy(layer)
    x = _cl(torch.randn(4, 256, 46, 80))
    outs = []
    for mod, fused in ((layer, True), (ref, False)):
        monkeypatch.setattr(backbone, "_FUSED_BN", fused)
        monkeypatch.setattr(encoder, "_FUSED_BN", fused)
        xi = x.clone().requires_grad_(True)
        y = mod(xi)
        loss = (y.float() ** 2).mean()
        loss.backward()
        outs.append((y.float(), xi.grad.float(), [p.grad.float() for p in mod.parameters()]))
    (ya, ga, pa), (yb, gb, pb) = outs
    rel = lambda a, b: ((a - b).norm() / b.norm().clamp(min=1e-12)).item()  # noqa: E731
    assert rel(ya, yb) < 2e-2
    assert rel(ga, gb) < 5e-2
    for a, b in zip(pa, pb):
        assert rel(a, b) < 5e-2
