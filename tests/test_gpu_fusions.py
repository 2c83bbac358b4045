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


@pytest.mark.parametrize("nb", [1, 2])
def test_bn_act_resid_equals_add(hip_lib, nb):
    """fused.bn_act(..., resid=r) == bn_act(...) + r, forward and backward, bitwise
    (the CSPRep layer's bottleneck output + shortcut branch)."""
    from src.rtdetr_moe.fused import bn_act

    torch.manual_seed(2)
    shape = (2, 128, 20, 24)
    xs0 = [torch.randn(shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
           for _ in range(nb)]
    r0 = torch.randn(shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    dy = torch.randn(shape, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    bns = [torch.nn.BatchNorm2d(shape[1]).to(DEV) for _ in range(nb)]
    res = []
    for fused in (True, False):
        xs = [x.clone().requires_grad_(True) for x in xs0]
        r = r0.clone().requires_grad_(True)
        for bn in bns:
            bn.weight.grad = bn.bias.grad = None
        y = bn_act(xs, bns, "silu", resid=r) if fused else bn_act(xs, bns, "silu") + r
        y.backward(dy)
        res.append([y.detach().clone(), r.grad.clone()] + [x.grad.clone() for x in xs] +
                   [t.grad.clone() for bn in bns for t in (bn.weight, bn.bias)])
    for a, b in zip(res[0], res[1]):
        assert torch.equal(a, b)


def test_dual_linear_matches_two_linears(hip_lib):
    """linear.dual_linear (one node; x's gradient accumulated by the second
    GEMM) == two TokenLinears: outputs and weight gradients bitwise, x's
    gradient at one bf16 rounding (fp32 sum, rounded once)."""
    from src.rtdetr_moe.linear import TokenLinear, dual_linear

    torch.manual_seed(4)
    l1 = TokenLinear(256, 192).to(DEV).to(torch.bfloat16)
    l2 = TokenLinear(256, 96).to(DEV).to(torch.bfloat16)
    x0 = torch.randn(4, 300, 256, device=DEV).to(torch.bfloat16)
    g1 = torch.randn(4, 300, 192, device=DEV).to(torch.bfloat16)
    g2 = torch.randn(4, 300, 96, device=DEV).to(torch.bfloat16)
    res = []
    for fused in (True, False):
        x = x0.clone().requires_grad_(True)
        for p in list(l1.parameters()) + list(l2.parameters()):
            p.grad = None
        y1, y2 = dual_linear(x, l1, l2) if fused else (l1(x), l2(x))
        torch.autograd.backward([y1, y2], [g1, g2])
        res.append((y1.detach().clone(), y2.detach().clone(), x.grad.float().clone(),
                    [p.grad.clone() for p in list(l1.parameters()) + list(l2.parameters())]))
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])
    assert float((res[0][2] - res[1][2]).norm() / res[1][2].norm()) < 4e-3
    for a, b in zip(res[0][3], res[1][3]):
        assert torch.equal(a, b)


def test_grad_slot_two_conv_consumers(hip_lib):
    """conv.GradSlot: an activation consumed by two stats convolutions (the
    encoder's downsampling conv, then the decoder's input projection): the
    later consumer parks its data gradient, the earlier one adds it in its
    dgrad epilogue -- the input gradient equals autograd's sum at one bf16
    rounding, the weight gradients bitwise."""
    from src.rtdetr_moe.conv import GradSlot, conv_module_stats

    torch.manual_seed(5)
    ca = torch.nn.Conv2d(256, 256, 3, 2, 1, bias=False).to(DEV).to(torch.bfloat16)
    cb = torch.nn.Conv2d(256, 256, 1, bias=False).to(DEV).to(torch.bfloat16)
    x0 = torch.randn(2, 256, 46, 80, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res, rs = [], None
    for slot in (True, False):
        x = x0.clone().requires_grad_(True)
        ca.weight.grad = cb.weight.grad = None
        if slot:
            x.grad_slot = GradSlot()
        ya, pa = conv_module_stats(ca, x)
        yb, pb = conv_module_stats(cb, x)
        assert pa is not None and pb is not None
        if rs is None:
            rs = [torch.randn(y.shape, device=DEV).to(torch.bfloat16) for y in (ya, yb)]
        ((ya.float() * rs[0].float()).sum() + (yb.float() * rs[1].float()).sum()).backward()
        res.append((x.grad.float().clone(), ca.weight.grad.clone(), cb.weight.grad.clone()))
    assert float((res[0][0] - res[1][0]).norm() / res[1][0].norm()) < 4e-3
    assert torch.equal(res[0][1], res[1][1]) and torch.equal(res[0][2], res[1][2])


def test_narrow_heads_batched_after_backward(hip_lib, monkeypatch):
    """linear.DeferredWgrad's narrow heads (score head M = 1, box-head last
    layer M = 4, the query-position head's 4 -> 512 layer applied three times)
    in one rtdetr_linear_wgrad_narrow_batch launch pair == one
    rtdetr_linear_wgrad_narrow call per use summed by autograd, at bf16
    rounding (the batched sum is fp32, rounded once)."""
    from src.rtdetr_moe import linear as lin
    from src.rtdetr_moe.decoder import MLP

    torch.manual_seed(6)
    score = lin.TokenLinear(256, 1).to(DEV).to(torch.bfloat16)
    box = MLP(256, 256, 4, 3).to(DEV).to(torch.bfloat16)
    qpos = MLP(4, 512, 256, 2).to(DEV).to(torch.bfloat16)
    for m in list(box.layers) + list(qpos.layers):
        torch.nn.init.normal_(m.weight, std=0.05)
    params = list(score.parameters()) + list(box.parameters()) + list(qpos.parameters())
    t0 = torch.randn(2400, 256, device=DEV).to(torch.bfloat16)
    refs = [torch.rand(2400, 4, device=DEV).to(torch.bfloat16) for _ in range(3)]
    res = []
    for defer in (True, False):
        monkeypatch.setattr(lin, "NARROW_DEFER", [defer])
        t = t0.clone().requires_grad_(True)
        loss = (score(t).float() ** 2).sum() + (box(t).float() ** 2).sum()
        for r in refs:
            loss = loss + (qpos(r).float() * t.float()).sum()
        with lin.deferred_weight_grads() as d:
            grads = torch.autograd.grad(loss, params, allow_unused=True)
        grads = lin.merge_deferred(params, grads, d)
        res.append([g.float() for g in grads])
    for a, b in zip(res[0], res[1]):
        assert float((a - b).norm() / b.norm().clamp_min(1e-12)) < 1e-2


@pytest.mark.parametrize("pos", [False, True])
def test_layer_norm_finals_batched(hip_lib, pos):
    """LayerNorm [dgamma; dbeta] deferred to rtdetr_add_layer_norm_final_batch
    (one launch for every norm of the backward) == the per-norm final,
    bitwise (same fixed-order sum); the row gradients unchanged."""
    from src.rtdetr_moe import linear as lin
    from src.rtdetr_moe import norm

    torch.manual_seed(7)
    lns = [norm.AddLayerNorm(256).to(DEV).to(torch.bfloat16) for _ in range(3)]
    for m in lns:
        m.weight.data.uniform_(0.5, 1.5)
        m.bias.data.uniform_(-0.5, 0.5)
    a0 = torch.randn(2400, 256, device=DEV).to(torch.bfloat16)
    b0 = torch.randn(2400, 256, device=DEV).to(torch.bfloat16)
    p0 = torch.randn(2400, 256, device=DEV).to(torch.bfloat16)
    params = [t for m in lns for t in (m.weight, m.bias)]
    res = []
    for defer in (True, False):
        a = a0.clone().requires_grad_(True)
        x = a
        for m in lns:
            if pos:
                t, q = m.with_pos(x, b0, p0)
                x = t.float().sin().to(torch.bfloat16) + q
            else:
                x = m(x, b0)
        loss = (x.float() ** 2).sum()
        if defer:
            with lin.deferred_weight_grads() as d:
                grads = torch.autograd.grad(loss, params + [a], allow_unused=True)
            assert len(d.ln) == 3 and all(g is None for g in grads[:-1])
            grads = lin.merge_deferred(params + [a], grads, d)
        else:
            grads = torch.autograd.grad(loss, params + [a])
        res.append([g.clone() for g in grads])
    for g1, g2 in zip(res[0], res[1]):
        assert torch.equal(g1, g2)


def test_ranking_rows_overwrite_equals_mask(hip_lib):
    """RTDETRDecoder._enc_output_masked (linear on memory, invalid-anchor rows
    overwritten with the bias) == enc_output(valid * memory), bitwise."""
    from src.rtdetr_moe.decoder import RTDETRDecoder

    torch.manual_seed(8)
    dec = RTDETRDecoder(num_layers=1).to(DEV).to(torch.bfloat16)
    shapes = [(92, 160), (46, 80), (23, 40)]
    S = sum(h * w for h, w in shapes)
    anchors, valid = dec._anchors(shapes, torch.device(DEV), torch.float32)
    inv = dec._anchor_cache[("inv", tuple(shapes), torch.device(DEV), torch.float32)]
    assert 0 < inv.numel() < S
    memory = torch.randn(2, S, 256, device=DEV).to(torch.bfloat16)
    vmask = valid.to(memory.dtype)
    with torch.no_grad():
        ref = dec.enc_output(vmask * memory)
        got = dec._enc_output_masked(memory, inv, vmask)
    assert torch.equal(got, ref)


def test_fold_backward_batched_equals_per_tensor(hip_lib, monkeypatch):
    """backbone._FoldAll's backward (dW_l = dW'_l * scale_l for every folded
    convolution) as one rtdetr_fold_scale_batch launch == one torch.mul per
    tensor, bitwise."""
    from src.rtdetr_moe import backbone as bb

    torch.manual_seed(9)
    m = bb.PResNet(50).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    for mod in m.modules():
        if hasattr(mod, "running_var") and not isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_var.uniform_(0.5, 2.0)
            mod.weight.uniform_(0.5, 1.5)
    x = torch.randn(2, 3, 64, 96, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = []
    for batched in (True, False):
        monkeypatch.setattr(bb, "_FOLD_BWD_BATCH", batched)
        m.zero_grad(set_to_none=True)
        sum(o.float().sum() for o in m(x)).backward()
        res.append({n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None})
    assert res[0].keys() == res[1].keys() and len(res[0]) > 40
    for k in res[0]:
        assert torch.equal(res[0][k], res[1][k]), k


def _close_bf16(got, ref, what):
    """Within bf16 rounding of an fp32 reference (one rounding of a sum taken
    in another order)."""
    got, ref = got.float(), ref.float()
    assert torch.isfinite(got).all(), what
    tol = 1e-2 * ref.abs().max().item() + 1e-3
    err = (got - ref).abs().max().item()
    assert err <= tol, f"{what}: max err {err:.3e} > {tol:.3e}"


@pytest.mark.parametrize("M,K,N,relu,bias", [(2400, 256, 1, False, "bf16"), (2400, 256, 4, False, "bf16"),
                                             (5003, 256, 1, False, "fp32"), (37, 512, 8, True, None),
                                             (9, 1024, 3, False, "bf16"), (2400, 4, 512, True, "bf16"),
                                             (11, 8, 64, False, "fp32"), (0, 256, 4, False, "bf16"),
                                             # fewer lanes per row than outputs (K / 8 < N)
                                             (37, 8, 4, True, "bf16"), (9, 16, 8, False, "fp32"),
                                             (5, 8, 8, False, None), (13, 24, 7, True, "bf16")])
def test_linear_narrow_fwd_vs_fp32(hip_lib, M, K, N, relu, bias):
    """rtdetr_linear_narrow_fwd (N <= 8 outputs: lanes per row + butterfly; K
    <= 8 inputs: 8 outputs per thread) against an fp32 linear."""
    from src.moe import _lib as L

    torch.manual_seed(M + K + N)
    x = torch.randn(M, K, device=DEV).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * K ** -0.5).to(torch.bfloat16)
    b = None if bias is None else torch.randn(N, device=DEV).to(torch.bfloat16 if bias == "bf16" else torch.float32)
    y = L.linear_narrow_fwd(x, w, b, relu)
    ref = torch.nn.functional.linear(x.float(), w.float(), None if b is None else b.float())
    if relu:
        ref = ref.relu()
    assert y.shape == (M, N) and y.dtype == torch.bfloat16
    if M:
        _close_bf16(y, ref, "narrow fwd")


@pytest.mark.parametrize("M,K,N,masked", [(2400, 256, 4, True), (2400, 256, 1, False), (333, 512, 8, True),
                                          (7, 64, 3, False)])
def test_linear_narrow_dgrad_vs_fp32(hip_lib, M, K, N, masked):
    """rtdetr_linear_narrow_dgrad: g w, zeroed where the mask is <= 0 (the
    previous layer's ReLU), against fp32 (exact zeros where masked)."""
    from src.moe import _lib as L

    torch.manual_seed(M + K)
    g = torch.randn(M, N, device=DEV).to(torch.bfloat16)
    w = torch.randn(N, K, device=DEV).to(torch.bfloat16)
    mask = torch.randn(M, K, device=DEV).relu().to(torch.bfloat16) if masked else None
    gx = L.linear_narrow_dgrad(g, w, mask)
    ref = g.float() @ w.float()
    if masked:
        ref = ref * (mask.float() > 0)
        assert torch.all(gx[mask <= 0] == 0)
    _close_bf16(gx, ref, "narrow dgrad")


def test_narrow_heads_match_library_path(hip_lib, monkeypatch):
    """A decoder box head (MLP 256 -> 256 -> 256 -> 4), the query position
    head (4 -> 512 -> 256) and a score head (TokenLinear 256 -> 1) with the
    narrow kernels against the hipBLASLt + torch-ReLU composition: outputs
    and every gradient within bf16 rounding."""
    from src.rtdetr_moe import linear as lin
    from src.rtdetr_moe.decoder import MLP

    torch.manual_seed(5)
    box = MLP(256, 256, 4, 3).to(DEV).to(torch.bfloat16)
    qpos = MLP(4, 512, 256, 2).to(DEV).to(torch.bfloat16)
    score = lin.TokenLinear(256, 1).to(DEV).to(torch.bfloat16)
    x = torch.randn(8, 300, 256, device=DEV).to(torch.bfloat16)
    ref_pts = torch.rand(8, 300, 4, device=DEV).to(torch.bfloat16)
    gy = [torch.randn(8, 300, n, device=DEV).to(torch.bfloat16) for n in (4, 256, 1)]
    mods = [box, qpos, score]
    res = []
    for on in (True, False):
        monkeypatch.setattr(lin, "NARROW_LINEAR", [on])
        for m in mods:
            m.zero_grad(set_to_none=True)
        xa = x.clone().requires_grad_(True)
        outs = [box(xa), qpos(ref_pts), score(xa)]
        torch.autograd.backward(outs, gy)
        res.append(([o.detach() for o in outs], xa.grad.clone(),
                    [p.grad.clone() for m in mods for p in m.parameters()]))
    for a, b in zip(res[0][0], res[1][0]):
        _close_bf16(a, b, "head output")
    _close_bf16(res[0][1], res[1][1], "input gradient")
    for a, b in zip(res[0][2], res[1][2]):
        _close_bf16(a, b, "parameter gradient")


@pytest.mark.parametrize("rows,n,k,ties", [(8, 19320, 300, False), (8, 19320, 300, True), (3, 8400, 300, True),
                                           (2, 1000, 1000, True), (5, 700, 1, False), (1, 32768, 1024, True)])
def test_topk_rows_vs_torch(hip_lib, rows, n, k, ties):
    """rtdetr_topk_rows: the same sorted values as torch.topk; without ties the
    same indices; with ties (bf16-quantised scores) a valid top-k whose equal
    values are ordered by index and cut at the lowest indices."""
    from src.moe import _lib as L

    g = torch.Generator(device=DEV).manual_seed(n + k)
    x = torch.randn(rows, n, device=DEV, generator=g)
    if ties:
        x = x.to(torch.bfloat16).float()
    idx, val = L.topk_rows(x, k, values=True)
    ref_v, ref_i = torch.topk(x, k, dim=1)
    assert torch.equal(val, ref_v)
    assert torch.equal(torch.gather(x, 1, idx), val)
    srt = idx.sort(1).values
    assert torch.all(srt[:, 1:] != srt[:, :-1])  # distinct indices per row
    if not ties:
        assert torch.equal(idx, ref_i)
    else:
        kth = val[:, -1:]
        # every value above the cut is taken; at the cut the lowest indices are
        for r in range(rows):
            above = (x[r] > kth[r]).nonzero().flatten()
            assert set(above.tolist()) <= set(idx[r].tolist())
            eq_all = (x[r] == kth[r]).nonzero().flatten().sort().values
            eq_taken = idx[r][val[r] == kth[r]].sort().values
            assert torch.equal(eq_taken, eq_all[:eq_taken.numel()])
        # equal values ordered by index
        same = val[:, 1:] == val[:, :-1]
        assert torch.all(idx[:, 1:][same] > idx[:, :-1][same])
