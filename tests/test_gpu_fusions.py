"""Round-5 launch-floor fusions in the detector body, each checked bitwise
against the unfused torch composition it replaces (same kernels, same
statistics, only the addressing / accumulation point differs):

  * decoder._LevelMemory: the input projections' BatchNorms written straight
    into the rows of memory [B, S, d] (rtdetr_bn_act_fwd_rows) and their
    gradients read from d memory in place (rtdetr_bn_act_bwd_rows), against
    bn_act per level + flatten / permute / torch.cat;
  * decoder._ValueProjAll's query-selection rows: sel = memory[topk] * vsel
    with its gradient scatter-added into d memory in place, against the
    gather + multiply whose backward is a zero-filled scatter and a full-size
    add.
"""
from __future__ import annotations

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def test_level_memory_equals_concat(hip_lib):
    from src.rtdetr_moe.decoder import _LevelMemory
    from src.rtdetr_moe.fused import bn_act

    torch.manual_seed(0)
    B, C = 3, 256
    shapes = [(24, 40), (12, 20), (6, 10)]
    ys = [torch.randn(B, C, h, w, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
          for h, w in shapes]
    bns = [torch.nn.BatchNorm2d(C).to(DEV) for _ in shapes]
    for bn in bns:
        bn.weight.data.uniform_(0.5, 1.5)
        bn.bias.data.uniform_(-0.5, 0.5)
    S = sum(h * w for h, w in shapes)
    dmem = torch.randn(B, S, C, device=DEV).to(torch.bfloat16)
    res = []
    for fused in (True, False):
        xs = [y.detach().clone().requires_grad_(True) for y in ys]
        for bn in bns:
            bn.weight.grad = bn.bias.grad = None
            bn.running_mean.zero_()
            bn.running_var.fill_(1.0)
        if fused:
            mem = _LevelMemory.apply(bns, [None] * 3, *xs, *[bn.weight for bn in bns], *[bn.bias for bn in bns])
        else:
            proj = [bn_act([x], [bn], None) for x, bn in zip(xs, bns)]
            mem = torch.cat([f.flatten(2).permute(0, 2, 1) for f in proj], 1).contiguous()
        mem.backward(dmem)
        res.append((mem.detach().clone(), [x.grad.clone() for x in xs],
                    [t.grad.clone() for bn in bns for t in (bn.weight, bn.bias)],
                    [t.clone() for bn in bns for t in (bn.running_mean, bn.running_var)]))
    assert torch.equal(res[0][0], res[1][0])
    for k in (1, 2, 3):
        for a, b in zip(res[0][k], res[1][k]):
            assert torch.equal(a, b)


def test_value_proj_selection_rows(hip_lib):
    from src.rtdetr_moe.decoder import _ValueProjAll

    torch.manual_seed(1)
    B, S, d, n, Q = 2, 1500, 256, 3, 300
    memory = torch.randn(B, S, d, device=DEV).to(torch.bfloat16)
    ws = [(torch.randn(d, d, device=DEV) * 0.05).to(torch.bfloat16) for _ in range(n)]
    bs = [(torch.randn(d, device=DEV) * 0.05).to(torch.bfloat16) for _ in range(n)]
    topk = torch.stack([torch.randperm(S, device=DEV)[:Q] for _ in range(B)])
    vmask = (torch.rand(1, S, 1, device=DEV) > 0.1).to(torch.bfloat16)
    vsel = vmask.expand(B, -1, -1).gather(1, topk[..., None])
    gsel = torch.randn(B, Q, d, device=DEV).to(torch.bfloat16)
    G = torch.randn(B, S, n * d, device=DEV).to(torch.bfloat16)
    zero = torch.zeros((), device=DEV)
    res = []
    for fused in (True, False):
        m = memory.clone().requires_grad_(True)
        v_all, g_all, token, sel = _ValueProjAll.apply(m, torch.bfloat16, True, topk, vsel,
                                                       *[t for wb in zip(ws, bs) for t in wb])
        g_all.copy_(G)  # (the value gradients the layers' MSDA backward would have written)
        if not fused:  # the unfused selection: autograd's zero-filled scatter + add into d memory
            sel = m.gather(1, topk[..., None].expand(-1, -1, d)) * vsel
        torch.autograd.backward([sel, token], [gsel, zero], inputs=[m])
        res.append((sel.detach().clone(), m.grad.clone()))
    assert torch.equal(res[0][0], res[1][0])
    assert torch.equal(res[0][1], res[1][1])
