"""GPU parity of the HIP multi-scale deformable attention (rtdetr_msda_fwd/bwd)
against the grid_sample formulation in float64 on the CPU (same inputs).
Tolerance: output |err| <= 1e-2 * max|ref| + 1 bf16 ulp (bf16 output);
gradients relative Frobenius error <= 2e-3 (loc, attn: fp32) and <= 1e-2
for the value gradient of a bf16 value (packed bf16 atomics)."""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,Q,H,D,P,shapes", [
    (2, 300, 8, 32, 4, [(92, 160), (46, 80), (23, 40)]),
    (1, 17, 8, 32, 4, [(5, 7), (3, 4), (2, 2)]),
    (3, 50, 4, 64, 2, [(16, 16), (8, 8)]),
])
def test_msda_matches_grid_sample(hip_lib, B, Q, H, D, P, shapes):
    from src.rtdetr_moe.decoder import deformable_attention, deformable_attention_core

    g = torch.Generator().manual_seed(0)
    S = sum(h * w for h, w in shapes)
    L = len(shapes)
    value = torch.randn(B, S, H, D, generator=g).to(torch.bfloat16).double()
    # locations spread over [-0.1, 1.1] to exercise the zero padding
    loc = (torch.rand(B, Q, H, L, P, 2, generator=g) * 1.2 - 0.1).double()
    attn = torch.softmax(torch.randn(B, Q, H, L * P, generator=g), -1).view(B, Q, H, L, P).double()
    gout = torch.randn(B, Q, H * D, generator=g).to(torch.bfloat16).double()

    v_ref, l_ref, a_ref = (t.clone().requires_grad_(True) for t in (value, loc, attn))
    ref = deformable_attention_core(v_ref, shapes, l_ref, a_ref)
    (ref * gout).sum().backward()

    dev = "cuda"
    v, lo, at = (t.to(dev).float().requires_grad_(True) for t in (value, loc, attn))
    vb = v.to(torch.bfloat16)
    vb.retain_grad()
    out = deformable_attention(vb, shapes, lo, at)
    (out.float() * gout.to(dev).float()).sum().backward()
    torch.cuda.synchronize()
    o = out.double().cpu()
    scale = ref.abs().max().item()
    err = (o - ref.detach()).abs()
    assert (err <= 1e-2 * scale + ref.detach().abs() * 2 ** -7).all(), float(err.max())
    for name, got, want in [("value", vb.grad, v_ref.grad), ("loc", lo.grad, l_ref.grad), ("attn", at.grad, a_ref.grad)]:
        got = got.double().cpu()
        rel = (got - want).norm() / want.norm().clamp(min=1e-12)
        assert rel < 2e-3 if name != "value" else rel < 1e-2, f"{name}: rel err {rel:.3e}"


def test_msda_bwd_bf16_atomics_vs_fp32(hip_lib):
    """The bf16-accumulated value gradient (rtdetr_msda_bwd_bf16) against the
    fp32-accumulated one (rtdetr_msda_bwd) on the C2 decoder shapes; the
    location / attention gradients do not depend on the accumulation."""
    from src.moe import _lib as L
    from src.rtdetr_moe.decoder import _level_tensors

    g = torch.Generator().manual_seed(1)
    shapes = [(92, 160), (46, 80), (23, 40)]
    B, Q, H, D, P = 8, 300, 8, 32, 4
    S = sum(h * w for h, w in shapes)
    dev = "cuda"
    value = torch.randn(B, S, H, D, generator=g).to(torch.bfloat16).to(dev)
    loc = torch.rand(B, Q, H, 3, P, 2, generator=g).to(dev)
    attn = torch.softmax(torch.randn(B, Q, H, 3 * P, generator=g), -1).view(B, Q, H, 3, P).to(dev)
    gout = torch.randn(B, Q, H * D, generator=g).to(torch.bfloat16).to(dev)
    st, so = _level_tensors(shapes, torch.device(dev))
    gv32, gl32, ga32 = L.msda_bwd(value, st, so, loc, attn, gout)
    gv16, gl16, ga16 = L.msda_bwd(value, st, so, loc, attn, gout, bf16_grad_value=True)
    assert gv16.dtype == torch.bfloat16
    assert torch.equal(gl16, gl32) and torch.equal(ga16, ga32)
    rel = float((gv16.float() - gv32).norm() / gv32.norm())
    assert rel < 4e-3, rel


def test_msda_fused_prep_matches_unfused(hip_lib):
    """rtdetr_msda_fused_fwd/bwd (locations + softmax formed in the kernel)
    against the unfused decoder formulation (torch prep + rtdetr_msda_*) on the
    C2 decoder shapes: output and the gradients of value, sampling offsets and
    attention logits."""
    import torch.nn.functional as F

    from src.rtdetr_moe.decoder import _MSDAFusedHip, _level_tensors, deformable_attention

    g = torch.Generator().manual_seed(2)
    shapes = [(92, 160), (46, 80), (23, 40)]
    B, Q, H, D, L, P = 4, 300, 8, 32, 3, 4
    S = sum(h * w for h, w in shapes)
    dev = "cuda"
    value = torch.randn(B, S, H, D, generator=g).to(torch.bfloat16).to(dev)
    off = (torch.randn(B, Q, H * L * P * 2, generator=g) * 2).to(torch.bfloat16).to(dev)
    logits = torch.randn(B, Q, H * L * P, generator=g).to(torch.bfloat16).to(dev)
    ref = torch.cat([torch.rand(B, Q, 2, generator=g) * 0.8 + 0.1, torch.rand(B, Q, 2, generator=g) * 0.3 + 0.02],
                    -1).to(dev)
    gout = torch.randn(B, Q, H * D, generator=g).to(torch.bfloat16).to(dev)
    scale = 0.5
    res = []
    for fused in (False, True):
        v, o, lg = (t.clone().requires_grad_(True) for t in (value, off, logits))
        if fused:
            st, so = _level_tensors(shapes, torch.device(dev))
            out = _MSDAFusedHip.apply(v, st, so, o, ref, lg, scale, L, P)
        else:
            aw = F.softmax(lg.view(B, Q, H, L * P).float(), -1).view(B, Q, H, L, P)
            r = ref[:, :, None, None, None, :]
            loc = r[..., :2] + o.view(B, Q, H, L, P, 2) / P * r[..., 2:] * scale
            out = deformable_attention(v, shapes, loc, aw)
        (out.float() * gout.float()).sum().backward()
        res.append((out.detach().float(), v.grad.float(), o.grad.float(), lg.grad.float()))
    for name, a, b in zip(("out", "value", "off", "logits"), res[0], res[1]):
        rel = float((b - a).norm() / a.norm().clamp_min(1e-12))
        assert rel < 1e-2, f"{name}: rel err {rel:.3e}"


def test_box_refine_matches_torch(hip_lib):
    """rtdetr_box_refine_fwd/bwd against the upstream decoder's two
    sigmoid(delta + inverse_sigmoid(.)) evaluations (on ref and ref.detach()),
    including references at and beyond the clamp edges."""
    from src.rtdetr_moe.decoder import _BoxRefineHip, inverse_sigmoid

    g = torch.Generator().manual_seed(3)
    dev = "cuda"
    delta0 = torch.randn(4, 300, 4, generator=g).to(torch.bfloat16).to(dev)
    ref0 = torch.rand(4, 300, 4, generator=g).to(dev)
    ref0[0, :4, 0] = torch.tensor([0.0, 1.0, 1e-7, 1.0 - 1e-7], device=dev)
    gb = torch.randn(4, 300, 4, generator=g).to(dev)
    gi = torch.randn(4, 300, 4, generator=g).to(dev)
    res = []
    for fused in (False, True):
        d = delta0.clone().requires_grad_(True)
        r = ref0.clone().requires_grad_(True)
        if fused:
            boxes, inter = _BoxRefineHip.apply(d, r, 1e-5)
        else:
            boxes = (d.float() + inverse_sigmoid(r)).sigmoid()
            inter = (d.float() + inverse_sigmoid(r.detach())).sigmoid()
        ((boxes * gb).sum() + (inter * gi).sum()).backward()
        res.append((boxes.detach(), inter.detach(), d.grad.float(), r.grad))
    for name, a, b in zip(("boxes", "inter", "d_ref"), (res[0][0], res[0][1], res[0][3]),
                          (res[1][0], res[1][1], res[1][3])):
        torch.testing.assert_close(b, a, rtol=1e-5, atol=1e-5, msg=name)
    # d_delta is bf16: torch rounds each path's gradient to bf16 and adds them
    # (two roundings), the kernel rounds their fp32 sum once
    rel = float((res[1][2] - res[0][2]).norm() / res[0][2].norm())
    assert rel < 5e-3, rel


@pytest.mark.parametrize("precision", ["bf16", "amp"])
def test_batched_value_projection_matches_per_layer(hip_lib, precision, monkeypatch):
    """The decoder's six value projections as one [B*S, 6d] GEMM
    (decoder._ValueProjAll + strided MSDA slices, value gradients accumulated in
    one shared buffer) give the per-layer path's outputs and gradients (memory,
    value_proj weights and biases, the other decoder weights) within bf16
    rounding."""
    import src.rtdetr_moe.decoder as dec
    from src.rtdetr_moe.decoder import RTDETRDecoder

    torch.manual_seed(0)
    dev = "cuda"
    shapes = [(20, 32), (10, 16), (5, 8)]
    B = 2
    from src.rtdetr_moe.step import gemm_params

    model = RTDETRDecoder(num_queries=50, num_layers=3).to(dev)
    if precision == "bf16":  # TrainStep's "bf16" precision: GEMM operands in bf16, BN / router fp32
        for p in gemm_params(model):
            p.data = p.data.to(torch.bfloat16)
    dt = torch.bfloat16 if precision == "bf16" else torch.float32
    g = torch.Generator(device=dev).manual_seed(1)
    feats = [torch.randn(B, 256, h, w, device=dev, generator=g).to(dt).requires_grad_(True) for h, w in shapes]
    ctx = torch.zeros(B, dtype=torch.int32, device=dev)
    res = []
    for batched in (False, True):
        monkeypatch.setattr(dec, "_BATCHED_VALUE", batched)
        model.zero_grad(set_to_none=True)
        for f in feats:
            f.grad = None
        model.query_override = None if not batched else model.last_topk
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=precision == "amp"):
            out = model(feats, ctx)
        loss = out["pred_logits"].float().square().sum() + out["pred_boxes"].float().sum() + sum(
            a["pred_boxes"].float().sum() for a in out["aux_outputs"])
        loss.backward()
        grads = {n: p.grad.float().clone() for n, p in model.named_parameters() if p.grad is not None}
        res.append((out["pred_logits"].detach().float(), [f.grad.float().clone() for f in feats], grads))
    torch.cuda.synchronize()
    assert "layers.0.cross_attn.value_proj.weight" in res[1][2]
    rel = lambda a, b: float((a - b).norm() / b.norm().clamp_min(1e-12))  # noqa: E731
    assert rel(res[1][0], res[0][0]) < 2e-2
    for a, b in zip(res[1][1], res[0][1]):
        assert rel(a, b) < 3e-2
    for n, gref in res[0][2].items():
        assert n in res[1][2], n
        assert rel(res[1][2][n], gref) < 5e-2, (n, rel(res[1][2][n], gref))


@pytest.mark.parametrize("D", [32, 64])
def test_msda_level_batched_kernels_match_generic(hip_lib, D):
    """The level-batched fused kernels (L = 3, P = 4: unrolled samples, one
    offsets load per group, a level's corner loads issued together) against the
    generic fused kernels (moe_set_tuning msda_generic) on the strided value
    slice the decoder uses: forward bit-identical (same arithmetic in the same
    order); offset / logit gradients within 1e-5 relative Frobenius (their
    group reductions are identical, the stores move to other lanes); the value
    gradient -- bf16 atomics, whose summation order differs -- within 1e-2."""
    from src.moe import _lib as L
    from src.rtdetr_moe.decoder import _level_tensors

    g = torch.Generator().manual_seed(5)
    shapes = [(46, 80), (23, 40), (12, 20)]
    B, Q, H, Lv, P = 2, 300, 8, 3, 4
    S = sum(h * w for h, w in shapes)
    C = 3 * H * D
    dev = "cuda"
    value_all = torch.randn(B, S, C, generator=g).to(torch.bfloat16).to(dev)
    off = (torch.randn(B, Q, H * Lv * P * 2, generator=g) * 2).to(torch.bfloat16).to(dev)
    logits = torch.randn(B, Q, H * Lv * P, generator=g).to(torch.bfloat16).to(dev)
    ref = torch.cat([torch.rand(B, Q, 2, generator=g) * 1.2 - 0.1, torch.rand(B, Q, 2, generator=g) * 0.3 + 0.02],
                    -1).to(dev)  # some locations off the map: the zero-padding corners
    gout = torch.randn(B, Q, H * D, generator=g).to(torch.bfloat16).to(dev)
    st, so = _level_tensors(shapes, torch.device(dev))
    col0 = H * D
    res = {}
    try:
        for generic in (3, 0):
            L.set_tuning("msda_generic", generic)
            out = L.msda_fused_fwd_slice(value_all, col0, H, D, st, so, off, ref, logits, 0.5, Lv, P)
            grad_all = torch.zeros(B, S, C, dtype=torch.bfloat16, device=dev)
            go, gl = L.msda_fused_bwd_slice(value_all, grad_all, col0, H, D, st, so, off, ref, logits, 0.5, Lv, P, gout)
            torch.cuda.synchronize()
            res[generic] = (out, grad_all, go, gl)
    finally:
        L.set_tuning("msda_generic", 0)
    (o3, gv3, go3, gl3), (o0, gv0, go0, gl0) = res[3], res[0]
    assert torch.equal(o3, o0)
    assert bool((gv0[..., :col0] == 0).all() and (gv0[..., col0 + H * D:] == 0).all())  # only this slice written

    def rel(a, b):
        return float((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12))

    assert rel(go0, go3) < 1e-5 and rel(gl0, gl3) < 1e-5, (rel(go0, go3), rel(gl0, gl3))
    assert rel(gv0, gv3) < 1e-2, rel(gv0, gv3)


def _vgrad_reference(value_all, col0, H, D, shapes, off, ref, logits, offset_scale, Lv, P, gout):
    """float64 value gradient of the fused MSDA slice, from the kernel's own
    location / attention formulas (fp32, same operation order) and a dense
    scatter-add on the host."""
    B, S, C = value_all.shape
    Q = off.shape[1]
    o = off.float().view(B, Q, H, Lv, P, 2)
    o = (o * (1.0 / P)).to(torch.bfloat16).float()  # bf16(off / P)
    a = torch.softmax(logits.float().view(B, Q, H, Lv * P), -1).view(B, Q, H, Lv, P)
    r = ref.float().view(B, Q, 1, 1, 1, 4)
    lx = r[..., 0] + o[..., 0] * r[..., 2] * offset_scale
    ly = r[..., 1] + o[..., 1] * r[..., 3] * offset_scale
    g = gout.double().view(B, Q, H, D).cpu()
    gv = torch.zeros(B, S, H, D, dtype=torch.float64)
    start = 0
    for l, (hl, wl) in enumerate(shapes):
        x = lx[..., l, :] * wl - 0.5
        y = ly[..., l, :] * hl - 0.5
        x0, y0 = torch.floor(x), torch.floor(y)
        fx, fy = (x - x0).double().cpu(), (y - y0).double().cpu()
        x0, y0 = x0.long().cpu(), y0.long().cpu()
        al = a[..., l, :].double().cpu()
        for c in range(4):
            xi, yi = x0 + (c & 1), y0 + (c >> 1)
            wc = (fx if c & 1 else 1 - fx) * (fy if c >> 1 else 1 - fy)
            ok = (xi >= 0) & (xi < wl) & (yi >= 0) & (yi < hl)
            row = (start + yi * wl + xi).clamp(0, S - 1)                      # [B, Q, H, P]
            wgt = (al * wc * ok).unsqueeze(-1) * g.unsqueeze(3)               # [B, Q, H, P, D]
            for b in range(B):
                for h in range(H):
                    gv[b, :, h].index_add_(0, row[b, :, h].reshape(-1), wgt[b, :, h].reshape(-1, D))
        start += hl * wl
    return gv


@pytest.mark.parametrize("D", [32, 64])
def test_msda_deterministic_value_gradient(hip_lib, D):
    """rtdetr_msda_fused_bwd_det (the decoder default): the offset / logit
    gradients equal the atomic kernel's bit for bit (the same per-sample
    code); the value gradient is bitwise repeatable, writes its whole column
    slice and nothing else, and is at least as close to a float64 reference
    as the bf16-atomic one (both rounded to bf16: <= 4e-3 relative Frobenius)."""
    from src.moe import _lib as L
    from src.rtdetr_moe.decoder import _level_tensors

    g = torch.Generator().manual_seed(7)
    shapes = [(46, 80), (23, 40), (12, 20)]
    B, Q, H, Lv, P = 2, 300, 8, 3, 4
    S = sum(h * w for h, w in shapes)
    C = 3 * H * D
    dev = "cuda"
    value_all = torch.randn(B, S, C, generator=g).to(torch.bfloat16).to(dev)
    off = (torch.randn(B, Q, H * Lv * P * 2, generator=g) * 2).to(torch.bfloat16).to(dev)
    logits = torch.randn(B, Q, H * Lv * P, generator=g).to(torch.bfloat16).to(dev)
    ref = torch.cat([torch.rand(B, Q, 2, generator=g) * 1.2 - 0.1, torch.rand(B, Q, 2, generator=g) * 0.3 + 0.02],
                    -1).to(dev)
    gout = torch.randn(B, Q, H * D, generator=g).to(torch.bfloat16).to(dev)
    st, so = _level_tensors(shapes, torch.device(dev))
    hw = [h * w for h, w in shapes]
    col0 = H * D
    runs = []
    for _ in range(2):
        grad_all = torch.full((B, S, C), 7.0, dtype=torch.bfloat16, device=dev)
        go, gl = L.msda_fused_bwd_slice_det(value_all, grad_all, col0, H, D, st, so, hw, off, ref, logits, 0.5, Lv,
                                            P, gout)
        torch.cuda.synchronize()
        runs.append((grad_all, go, gl))
    gv_a = torch.zeros(B, S, C, dtype=torch.bfloat16, device=dev)
    go_a, gl_a = L.msda_fused_bwd_slice(value_all, gv_a, col0, H, D, st, so, off, ref, logits, 0.5, Lv, P, gout)
    torch.cuda.synchronize()
    (gv, go, gl), (gv2, go2, gl2) = runs
    assert torch.equal(gv, gv2) and torch.equal(go, go2) and torch.equal(gl, gl2)  # repeatable
    assert torch.equal(go, go_a) and torch.equal(gl, gl_a)
    assert bool((gv[..., :col0] == 7.0).all() and (gv[..., col0 + H * D:] == 7.0).all())  # only the slice
    sl = gv[..., col0:col0 + H * D]
    assert not bool((sl == 7.0).any())  # every element of the slice written
    ref64 = _vgrad_reference(value_all, col0, H, D, shapes, off, ref, logits, 0.5, Lv, P, gout)
    ref64 = ref64.view(B, S, H * D)

    def rel(t):
        return float((t.double().cpu() - ref64).norm() / ref64.norm())

    e_det, e_atomic = rel(sl), rel(gv_a[..., col0:col0 + H * D])
    assert e_det <= 4e-3 and e_det <= e_atomic * 1.001 + 1e-6, (e_det, e_atomic)
