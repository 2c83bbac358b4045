"""Frozen-BN convolution epilogues of the backbone (fused.BiasReLU /
AddBiasReLU over libmoe_hip's rtdetr_*_nhwc kernels) on the GPU.
Tolerances: the kernels are bit-exact against the same fp32 formula rounded
once to bf16; the fused backbone (BN folded into the weights, bf16) follows
the unfused one (conv, then frozen BN): its error against the same network
in fp32 is no larger than the unfused bf16 network's (relative Frobenius:
features x 1.5 + 2e-3; weight gradients, median over layers x 1.5 + 2e-3 and
every layer x 3 + 5e-3) -- the two
bf16 paths round at different points, so they are compared through the fp32
reference rather than with each other."""
from __future__ import annotations

import copy

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _cl(t):
    return t.to(DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)


def test_bias_act_and_add_bias_relu_exact(hip_lib):
    from src.moe import _lib as L

    g = torch.Generator().manual_seed(0)
    a = _cl(torch.randn(3, 64, 17, 23, generator=g))
    b = _cl(torch.randn(3, 64, 17, 23, generator=g))
    bias = torch.randn(64, generator=g).to(DEV)
    bc = bias.view(1, -1, 1, 1)
    y = L.bias_act_nhwc(a, bias, True)
    torch.testing.assert_close(y, (a.float() + bc).relu().to(torch.bfloat16), rtol=0, atol=0)
    y0 = L.bias_act_nhwc(a, bias, False)
    torch.testing.assert_close(y0, (a.float() + bc).to(torch.bfloat16), rtol=0, atol=0)
    z = L.add_bias_relu_nhwc(a, b, bias)
    torch.testing.assert_close(z, (a.float() + b.float() + bc).relu().to(torch.bfloat16), rtol=0, atol=0)
    z0 = L.add_bias_relu_nhwc(a, b, None)
    torch.testing.assert_close(z0, (a.float() + b.float()).relu().to(torch.bfloat16), rtol=0, atol=0)
    xi = a.clone()
    L.bias_act_nhwc(xi, bias, True, out=xi)  # in place
    torch.testing.assert_close(xi, y, rtol=0, atol=0)


@pytest.mark.parametrize("shape", [(3, 72, 17, 23), (8, 264, 160, 160)])
def test_epilogues_channel_walk_exact(hip_lib, shape):
    """Channel counts whose chunk count does not divide the grid stride (the
    kernels advance the channel incrementally) and a tensor large enough for
    the capped grid's multi-iteration stride, incl. relu_grad2."""
    from src.moe import _lib as L

    g = torch.Generator().manual_seed(1)
    a = _cl(torch.randn(*shape, generator=g))
    b = _cl(torch.randn(*shape, generator=g))
    bias = torch.randn(shape[1], generator=g).to(DEV)
    bc = bias.view(1, -1, 1, 1)
    torch.testing.assert_close(L.bias_act_nhwc(a, bias, True), (a.float() + bc).relu().to(torch.bfloat16),
                               rtol=0, atol=0)
    torch.testing.assert_close(L.add_bias_relu_nhwc(a, b, bias),
                               (a.float() + b.float() + bc).relu().to(torch.bfloat16), rtol=0, atol=0)
    y = L.add_bias_relu_nhwc(a, b, bias)
    got = L.relu_grad2_nhwc(a, b, y)
    ref = torch.where(y > 0, a.float() + b.float(), torch.zeros((), device=DEV)).to(torch.bfloat16)
    torch.testing.assert_close(got, ref, rtol=0, atol=0)


def _rel(a, b):
    return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))


@pytest.mark.parametrize("depth", [18, 50])
def test_folded_backbone_matches_unfolded(hip_lib, depth):
    from src.rtdetr_moe.backbone import ConvNormLayer, FrozenBatchNorm2d, PResNet

    torch.manual_seed(0)
    m = PResNet(depth)
    for mod in m.modules():
        if isinstance(mod, FrozenBatchNorm2d):
            mod.weight.uniform_(0.5, 1.5)
            mod.bias.normal_(0, 0.1)
            mod.running_mean.normal_(0, 0.1)
            mod.running_var.uniform_(0.5, 2.0)
    m32 = copy.deepcopy(m).to(DEV).to(memory_format=torch.channels_last)  # fp32, unfused
    for mod in m32.modules():
        if isinstance(mod, ConvNormLayer):
            mod.fold = False
    m = m.to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    ref = copy.deepcopy(m)
    for mod in ref.modules():
        if isinstance(mod, ConvNormLayer):
            mod.fold = False
    x = _cl(torch.randn(2, 3, 256, 320))
    outs, outs_r, outs_32 = m(x), ref(x), m32(x.float())
    for a, b, c in zip(outs, outs_r, outs_32):
        assert _rel(a, c) <= 1.5 * _rel(b, c) + 2e-3
    for o in (outs, outs_r, outs_32):
        sum(t.float().square().mean() for t in o).backward()
    ef, eu = [], []
    for (n, p), (_, q), (_, r) in zip(m.named_parameters(), ref.named_parameters(), m32.named_parameters()):
        if p.grad is not None:
            ef.append(_rel(p.grad, r.grad))
            eu.append(_rel(q.grad, r.grad))
            assert ef[-1] <= 3.0 * eu[-1] + 5e-3, (n, ef[-1], eu[-1])  # no layer grossly off
    ef, eu = torch.tensor(ef), torch.tensor(eu)
    assert float(ef.median()) <= 1.5 * float(eu.median()) + 2e-3, (float(ef.median()), float(eu.median()))


@pytest.mark.gpu
def test_relu_grad2_and_fork_backward_exact(hip_lib):
    """rtdetr_relu_grad2_nhwc == threshold_backward(g1 + g2, y) bit for bit
    (bf16 add rounds once either way), and AddBiasReLUFork's two-handle
    backward equals autograd's accumulate + mask of AddBiasReLU."""
    from src.moe import _lib as L
    from src.rtdetr_moe.fused import AddBiasReLU, AddBiasReLUFork

    g = torch.Generator().manual_seed(4)
    y = _cl(torch.randn(2, 64, 9, 13, generator=g))
    g1 = _cl(torch.randn(2, 64, 9, 13, generator=g))
    g2 = _cl(torch.randn(2, 64, 9, 13, generator=g))
    assert torch.equal(L.relu_grad2_nhwc(g1, g2, y), torch.ops.aten.threshold_backward(g1 + g2, y, 0))
    assert torch.equal(L.relu_grad2_nhwc(g1, None, y), torch.ops.aten.threshold_backward(g1, y, 0))
    a0 = _cl(torch.randn(2, 64, 9, 13, generator=g))
    b0 = _cl(torch.randn(2, 64, 9, 13, generator=g))
    bias = torch.randn(64, generator=g).to(DEV)
    w1 = _cl(torch.randn(2, 64, 9, 13, generator=g))
    w2 = _cl(torch.randn(2, 64, 9, 13, generator=g))
    grads = []
    for fork in (False, True):
        a = a0.clone().requires_grad_(True)
        b = b0.clone().requires_grad_(True)
        if fork:
            y1, y2 = AddBiasReLUFork.apply(a, b, bias)
        else:
            y1 = y2 = AddBiasReLU.apply(a, b, bias)
        ((y1 * w1).float().sum() + (y2 * w2).float().sum()).backward()
        grads.append((a.grad, b.grad))
    assert torch.equal(grads[0][0], grads[1][0]) and torch.equal(grads[0][1], grads[1][1])


def test_fold_all_matches_per_layer_fold(hip_lib):
    """PResNet's one-launch fold of the frozen BNs (rtdetr_fold_scale_multi)
    gives the per-layer fold's outputs and weight gradients, and no gradient
    for the frozen stem."""
    from src.rtdetr_moe.backbone import PResNet

    torch.manual_seed(0)
    m = PResNet(18).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    for mod in m.modules():  # non-trivial frozen statistics
        if hasattr(mod, "running_var") and not isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_var.uniform_(0.5, 2.0)
            mod.weight.uniform_(0.5, 1.5)
    x = torch.randn(2, 3, 64, 96, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = []
    for use_plan in (False, True):
        m.zero_grad(set_to_none=True)
        if not use_plan:
            m._fold_plan = type("Off", (), {"usable": lambda self: False})()
        else:
            m._fold_plan = None
        outs = m(x)
        sum(o.float().square().mean() for o in outs).backward()
        res.append(([o.detach().clone() for o in outs],
                    {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}))
    # (MIOpen's convolution kernels are not bit-reproducible call to call --
    # weight gradients use atomics -- so compare at bf16 noise level)
    assert m._fold_plan.usable() and len(m._fold_plan.layers) > 0
    for a, b in zip(res[0][0], res[1][0]):
        assert _rel(b, a) < 2e-3
    assert res[0][1].keys() == res[1][1].keys()
    assert not any(k.startswith("stem") for k in res[1][1])
    for k in res[0][1]:
        assert _rel(res[1][1][k], res[0][1][k]) < 2e-2, k


@pytest.mark.parametrize("depth", [18, 50])
def test_no_fork_switch_keeps_relu_backward(hip_lib, monkeypatch, depth):
    """MOE_BACKBONE_FORK=0 (backbone._NO_FORK) takes _block_out's autograd
    fallback; the producing convolutions must then keep their own ReLU
    backward (they skipped it and the gradients came out wrong).
    Same outputs and weight gradients as the fork path, at bf16 noise."""
    from src.rtdetr_moe import backbone as bb

    torch.manual_seed(0)
    m = bb.PResNet(depth).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    for mod in m.modules():
        if hasattr(mod, "running_var") and not isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_var.uniform_(0.5, 2.0)
            mod.weight.uniform_(0.5, 1.5)
    x = torch.randn(2, 3, 128, 160, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = []
    for no_fork in (False, True):
        monkeypatch.setattr(bb, "_NO_FORK", no_fork)
        m.zero_grad(set_to_none=True)
        outs = m(x)
        sum(o.float().square().mean() for o in outs).backward()
        res.append(([o.detach().clone() for o in outs],
                    {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}))
    for a, b in zip(res[0][0], res[1][0]):
        assert _rel(b, a) < 2e-3
    assert res[0][1].keys() == res[1][1].keys()
    for k in res[0][1]:
        assert _rel(res[1][1][k], res[0][1][k]) < 2e-2, k


def test_down_link_matches_relu_grad2(hip_lib, monkeypatch):
    """GradLink through the ResNet-D downsampling shortcuts (backbone._DOWN_LINK:
    the average-pool backward hands its gradient to branch2a's dgrad epilogue,
    which adds it and applies the block input's ReLU mask -- no relu_grad2 pass
    at the stage boundaries) == the relu_grad2 path, at bf16 noise."""
    from src.rtdetr_moe import backbone as bb

    torch.manual_seed(1)
    m = bb.PResNet(50).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    for mod in m.modules():
        if hasattr(mod, "running_var") and not isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_var.uniform_(0.5, 2.0)
            mod.weight.uniform_(0.5, 1.5)
    x = torch.randn(2, 3, 128, 160, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = []
    for down in (True, False):
        monkeypatch.setattr(bb, "_DOWN_LINK", down)
        m.zero_grad(set_to_none=True)
        outs = m(x)
        sum(o.float().square().mean() for o in outs).backward()
        res.append(([o.detach().clone() for o in outs],
                    {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}))
    for a, b in zip(res[0][0], res[1][0]):
        assert torch.equal(a, b)
    assert res[0][1].keys() == res[1][1].keys()
    for k in res[0][1]:
        assert _rel(res[0][1][k], res[1][1][k]) < 2e-2, k


@pytest.mark.parametrize("tap", [False, True])
def test_stage_outputs_with_external_consumer(hip_lib, monkeypatch, tap):
    """The backbone's returned stage outputs (C3, C4) also feed the next stage,
    whose first block finishes their gradient through a GradLink (the average
    pool of the ResNet-D shortcut hands its gradient to branch2a's dgrad
    epilogue, which adds it and applies the ReLU mask).  The encoder's
    gradient for those outputs must be masked too: with a general consumer
    (a 1x1 HIP convolution, as the encoder's input projections, then a random
    linear functional, which -- unlike a square loss -- is non-zero where the
    ReLU output is zero) the parameter gradients with the links on equal the
    link-free path (every gradient summed by autograd, one relu_grad2 pass) at
    bf16 noise.  tap: the outputs go through backbone.stage_taps (the
    encoder's hand-off of its gradient into the link, no autograd add)."""
    from src.rtdetr_moe import backbone as bb
    from src.rtdetr_moe.conv import conv_module

    torch.manual_seed(3)
    m = bb.PResNet(50).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    for mod in m.modules():
        if hasattr(mod, "running_var") and not isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_var.uniform_(0.5, 2.0)
            mod.weight.uniform_(0.5, 1.5)
    projs = [torch.nn.Conv2d(c, 64, 1, bias=False).to(DEV).to(torch.bfloat16) for c in m.out_channels]
    x = torch.randn(2, 3, 128, 160, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    rs = None
    res = []
    for links in (True, False):
        monkeypatch.setattr(bb, "_GRAD_LINK", links)
        monkeypatch.setattr(bb, "_DOWN_LINK", links)
        m.zero_grad(set_to_none=True)
        outs = m(x)
        if tap:
            outs = bb.stage_taps(outs)
        ys = [conv_module(p, o) for p, o in zip(projs, outs)]
        if rs is None:
            g = torch.Generator(device=DEV).manual_seed(7)
            rs = [torch.randn(y.shape, device=DEV, generator=g).to(torch.bfloat16) for y in ys]
        sum((y.float() * r.float()).sum() for y, r in zip(ys, rs)).backward()
        res.append({n: p.grad.float().clone() for n, p in m.named_parameters() if p.grad is not None})
    assert res[0].keys() == res[1].keys() and len(res[0]) > 0
    bad = {k: round(_rel(res[0][k], res[1][k]), 4) for k in res[0] if _rel(res[0][k], res[1][k]) >= 2e-2}
    assert not bad, bad
