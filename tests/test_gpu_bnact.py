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


@pytest.mark.parametrize("nb,act,resid", [(1, "silu", False), (2, "silu", True), (1, None, False), (2, "silu", False)])
def test_bn_act_eval_matches_torch(hip_lib, nb, act, resid):
    """rtdetr_bn_act_eval (running statistics, branch sum, SiLU, shortcut after
    the activation) against torch's inference BatchNorm in fp32."""
    from src.rtdetr_moe.fused import bn_act_eval, bn_eval_ok

    g = torch.Generator().manual_seed(nb * 7 + int(resid))
    shape = (4, 256, 23, 40)
    xs = [_cl(torch.randn(shape, generator=g) * 1.5 + 0.3) for _ in range(nb)]
    bns = [bn.eval() for bn in _bns(nb, shape[1], g)]
    r = _cl(torch.randn(shape, generator=g)) if resid else None
    with torch.no_grad():
        assert bn_eval_ok(xs, bns)
        y = bn_act_eval(xs, bns, act, resid=r)
        z = sum(bn(x.float()) for bn, x in zip(bns, xs))
        ref = F.silu(z) if act == "silu" else z
        if resid:
            ref = ref + r.float()
    assert y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=2e-2 * ref.abs().max().item())


def test_encoder_eval_bn_matches_torch_bn(hip_lib, monkeypatch):
    """The HybridEncoder's inference forward with the one-pass HIP BatchNorms
    against torch's batch_norm + SiLU + adds: within bf16 rounding."""
    from src.rtdetr_moe import encoder, fused

    torch.manual_seed(2)
    enc = encoder.HybridEncoder().to(DEV).to(memory_format=torch.channels_last)
    for m in enc.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.3, 0.3)
            m.running_var.uniform_(0.5, 2.0)
    enc.eval()
    feats = [_cl(torch.randn(2, c, h, w)) for c, h, w in ((512, 46, 80), (1024, 23, 40), (2048, 12, 20))]
    ctx = torch.zeros(2, dtype=torch.long, device=DEV)
    outs = []
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        for on in (True, False):
            monkeypatch.setattr(fused, "_BN_EVAL", on)
            outs.append([o.float() for o in enc(feats, ctx)])
    for a, b in zip(*outs):
        torch.testing.assert_close(a, b, rtol=3e-2, atol=3e-2 * b.abs().max().item())


@pytest.mark.parametrize("ks,st,act,resid", [(3, 1, 2, True), (3, 1, 2, False), (1, 1, 0, False), (3, 2, 2, False),
                                             (1, 1, 1, False), (3, 1, 0, True)])
def test_conv_act_eval_matches_torch(hip_lib, ks, st, act, resid):
    """rtdetr_conv_fwd_act (the folded inference layers: conv + bias, ReLU /
    SiLU, the shortcut added after the activation) against fp32 torch on the
    same bf16 operands (one bf16 rounding of the conv, one of the activation,
    one of the add: rtol 1e-2, atol 2e-2 x scale)."""
    from src.rtdetr_moe.conv import conv_act_eval

    g = torch.Generator().manual_seed(ks * 10 + st + act)
    x = _cl(torch.randn(2, 256, 23, 40, generator=g))
    w = _cl(torch.randn(128, 256, ks, ks, generator=g) * (256 * ks * ks) ** -0.5)
    b = (torch.randn(128, generator=g) * 0.5).to(DEV)
    Ho, Wo = (23 - 1) // st + 1, (40 - 1) // st + 1
    r = _cl(torch.randn(2, 128, Ho, Wo, generator=g)) if resid else None
    with torch.no_grad():
        y = conv_act_eval(x, w, b, act, resid=r, st=st)
        z = F.conv2d(x.float(), w.float(), b, stride=st, padding=(ks - 1) // 2)
        ref = F.silu(z) if act == 2 else (z.relu() if act == 1 else z)
        if resid:
            ref = ref + r.float()
    assert y.shape == ref.shape and y.dtype == torch.bfloat16 and y.is_contiguous(memory_format=torch.channels_last)
    torch.testing.assert_close(y.float(), ref, rtol=1e-2, atol=2e-2 * ref.abs().max().item())


def test_encoder_eval_fold_matches_unfolded(hip_lib, monkeypatch):
    """The HybridEncoder's inference forward with every running-statistics
    BatchNorm folded into its convolution and each RepVgg block as ONE 3x3
    convolution (evalfold: the 1x1 branch in the centre tap, SiLU and the CSP
    shortcut in the epilogue) against the unfolded inference path (conv + the
    one-pass BatchNorm kernel): within bf16 rounding (the folded weights are
    rounded once to bf16)."""
    from src.rtdetr_moe import encoder, evalfold

    torch.manual_seed(3)
    enc = encoder.HybridEncoder().to(DEV).to(memory_format=torch.channels_last)
    for m in enc.modules():
        if isinstance(m, torch.nn.BatchNorm2d):
            m.running_mean.uniform_(-0.3, 0.3)
            m.running_var.uniform_(0.5, 2.0)
            m.weight.data.uniform_(0.5, 1.5)
            m.bias.data.uniform_(-0.2, 0.2)
    enc.eval()
    evalfold.refresh(enc)
    n_fold = sum(hasattr(m, "_eval_fold") for m in enc.modules())
    assert n_fold == 3 + 2 + 2 + 4 * (2 + 3), n_fold  # proj, lateral, downsample, CSP entries + RepVgg blocks
    feats = [_cl(torch.randn(2, c, h, w)) for c, h, w in ((512, 46, 80), (1024, 23, 40), (2048, 12, 20))]
    ctx = torch.zeros(2, dtype=torch.long, device=DEV)
    outs = []
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        for on in (True, False):
            monkeypatch.setattr(evalfold, "_ON", on)
            outs.append([o.float() for o in enc(feats, ctx)])
    for a, b in zip(*outs):
        assert torch.isfinite(a).all()
        torch.testing.assert_close(a, b, rtol=3e-2, atol=3e-2 * b.abs().max().item())


def test_conv_act_eval_rows_into_memory(hip_lib):
    """rtdetr_conv_fwd_act writing image b's output rows at out[b, row:row + Ho Wo]
    (the folded input projections filling the decoder memory [B, S, N] in
    place): bitwise the dense output, other rows untouched."""
    from src.rtdetr_moe.conv import conv_act_eval

    g = torch.Generator().manual_seed(5)
    x = _cl(torch.randn(3, 512, 12, 20, generator=g))
    w = _cl(torch.randn(256, 512, 1, 1, generator=g) * 512 ** -0.5)
    b = torch.randn(256, generator=g).to(DEV)
    dense = conv_act_eval(x, w, b, 0)
    mem = torch.full((3, 300, 256), 7.0, dtype=torch.bfloat16, device=DEV)
    got = conv_act_eval(x, w, b, 0, out=mem, out_row=40)
    assert got is mem
    ref = dense.flatten(2).permute(0, 2, 1)
    assert torch.equal(mem[:, 40:280], ref)
    assert (mem[:, :40] == 7).all() and (mem[:, 280:] == 7).all()
