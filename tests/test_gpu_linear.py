"""GPU parity of the linear-layer bias gradient (rtdetr_bias_grad) and of
TokenLinear against nn.Linear.

Bias gradient: fp32 accumulation of bf16 gradients in a fixed order vs torch's
fp64 column sum of the same bf16 values: |err| <= 1e-5 * sum|dy| per column
(fp32 rounding of M terms), bf16 output within 1 bf16 ulp of the fp32 result.
Deterministic: two runs are bit-identical.  TokenLinear: output bit-identical
to nn.Linear (same F.linear call); input and weight gradients within 1e-2
relative Frobenius error (the same GEMMs, possibly another operand
orientation, bf16 outputs); bias gradient within the tolerance above plus its
bf16 rounding.
"""
from __future__ import annotations

import pytest
import torch
from torch import nn

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("M,N", [(1, 1), (37, 4), (300, 1), (2400, 256), (2400, 192), (2400, 96),
                                 (7360, 1024), (154560, 256), (1000, 8), (513, 2048), (100, 200)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_bias_grad(hip_lib, M, N, out_dtype):
    from src.rtdetr_moe.linear import bias_grad

    g = torch.Generator().manual_seed(M * 31 + N)
    dy = torch.randn(M, N, generator=g).to(torch.bfloat16).cuda()
    ref = dy.double().sum(0)
    tol = 1e-5 * dy.double().abs().sum(0) + 1e-30
    got = bias_grad(dy, out_dtype)
    assert got.dtype == out_dtype and got.shape == (N,)
    if out_dtype == torch.float32:
        err = (got.double() - ref).abs()
        assert bool((err <= tol).all()), float((err - tol).max())
        got2 = bias_grad(dy, out_dtype)
        assert torch.equal(got, got2)  # deterministic
    else:
        f32 = bias_grad(dy, torch.float32)
        assert torch.equal(got, f32.to(torch.bfloat16))


def test_bias_grad_unaligned_view(hip_lib):
    from src.rtdetr_moe.linear import bias_grad

    base = torch.randn(257 * 256 + 3, dtype=torch.bfloat16, device="cuda")
    dy = base[3:].view(257, 256)  # 6-B offset: not 16-B aligned
    got = bias_grad(dy, torch.float32)
    ref = dy.double().sum(0)
    assert bool(((got.double() - ref).abs() <= 1e-5 * dy.double().abs().sum(0) + 1e-30).all())


@pytest.mark.parametrize("shape,din,dout", [((8, 300, 256), 256, 256), ((2400, 256), 256, 1), ((4, 77, 256), 256, 4),
                                            ((8, 920, 256), 256, 1024), ((8, 300, 512), 512, 256),
                                            ((8, 300, 256), 256, 192), ((3, 190, 256), 256, 768)])
def test_token_linear_matches_linear(hip_lib, shape, din, dout):
    from src.rtdetr_moe.linear import TokenLinear

    torch.manual_seed(0)
    ref = nn.Linear(din, dout).cuda().to(torch.bfloat16)
    tl = TokenLinear(din, dout).cuda().to(torch.bfloat16)
    tl.load_state_dict(ref.state_dict())
    x = torch.randn(*shape, device="cuda", dtype=torch.bfloat16)
    x1 = x.clone().requires_grad_(True)
    x2 = x.clone().requires_grad_(True)
    y1, y2 = ref(x1), tl(x2)
    assert torch.equal(y1, y2)
    gy = torch.randn_like(y1)
    y1.backward(gy)
    y2.backward(gy)
    for a, b in ((x1.grad, x2.grad), (ref.weight.grad, tl.weight.grad)):  # same GEMMs, bf16 outputs
        assert float((a.double() - b.double()).norm() / b.double().norm().clamp_min(1e-30)) <= 1e-2
    gb_ref = gy.reshape(-1, dout).double().sum(0)
    tol = 1e-5 * gy.reshape(-1, dout).double().abs().sum(0) + 2.0 ** -8 * gb_ref.abs() + 1e-30
    assert tl.bias.grad.dtype == torch.bfloat16
    assert bool(((tl.bias.grad.double() - gb_ref).abs() <= tol).all())


def test_token_linear_fp32_weights_under_autocast(hip_lib):
    """amp precision: fp32 parameters, bf16 compute; the fused weight + bias
    gradient (libmoe_hip wgrad, G = 1) comes back in fp32."""
    from src.rtdetr_moe.linear import TokenLinear

    torch.manual_seed(1)
    tl = TokenLinear(256, 256).cuda()
    x = torch.randn(8, 300, 256, device="cuda", requires_grad=True)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = tl(x)
    gy = torch.randn_like(y)
    y.backward(gy)
    xb, wb, gb = x.detach().to(torch.bfloat16).double(), tl.weight.detach(), gy.to(torch.bfloat16).double()
    gw_ref = gb.reshape(-1, 256).t() @ xb.reshape(-1, 256)
    assert tl.weight.grad.dtype == torch.float32 and tl.bias.grad.dtype == torch.float32
    assert float((tl.weight.grad.double() - gw_ref).norm() / gw_ref.norm()) <= 1e-5
    torch.testing.assert_close(tl.bias.grad.double(), gb.reshape(-1, 256).sum(0), rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("K,M,N", [(512, 64, 128), (2400, 256, 256), (2400, 512, 256), (4800, 256, 256),
                                   (777, 128, 384), (65535, 64, 128)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_linear_wgrad_dense(hip_lib, K, M, N, out_dtype):
    """rtdetr_linear_wgrad (dense dW = gy^T x and db = colsum(gy) in one launch,
    the TokenLinear backward for conforming shapes) vs torch fp64 of the same
    bf16 operands: dW within 1e-5 * sum_r |gy_rm x_rn| per element (fp32 split-K
    accumulation), db within the bias tolerance above; bf16 outputs within one
    bf16 ulp of that; deterministic (bit-identical reruns)."""
    from src.moe import _lib as L

    g = torch.Generator().manual_seed(K + 7 * M + N)
    gy = torch.randn(K, M, generator=g).to(torch.bfloat16).cuda()
    x = torch.randn(K, N, generator=g).to(torch.bfloat16).cuda()
    dw, db = L.linear_wgrad(gy, x, out_dtype)
    assert dw.shape == (M, N) and db.shape == (M,) and dw.dtype == db.dtype == out_dtype
    ref_w = gy.double().t().mm(x.double())
    tol_w = 1e-5 * gy.double().abs().t().mm(x.double().abs()) + 1e-30
    ref_b = gy.double().sum(0)
    tol_b = 1e-5 * gy.double().abs().sum(0) + 1e-30
    if out_dtype == torch.bfloat16:  # + half a bf16 ulp of the result
        tol_w = tol_w + ref_w.abs() * 2.0 ** -8
        tol_b = tol_b + ref_b.abs() * 2.0 ** -8
    assert bool(((dw.double() - ref_w).abs() <= tol_w).all()), float(((dw.double() - ref_w).abs() - tol_w).max())
    assert bool(((db.double() - ref_b).abs() <= tol_b).all()), float(((db.double() - ref_b).abs() - tol_b).max())
    dw2, db2 = L.linear_wgrad(gy, x, out_dtype)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


@pytest.mark.parametrize("K,M,N", [(2400, 1, 256), (2400, 4, 256), (2400, 96, 256), (1, 1, 2), (17, 3, 130),
                                   (300, 128, 256), (4000, 5, 1024), (2400, 80, 384),
                                   (2400, 512, 4), (300, 256, 3), (1000, 130, 20), (64, 4, 3)])
@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_linear_wgrad_narrow(hip_lib, K, M, N, out_dtype):
    """rtdetr_linear_wgrad_narrow (class / box / attention-weight heads: M <=
    128 outputs, any M; transposed orientation for N <= 128 inputs) vs torch fp64 of the same bf16 operands, same
    tolerances as the dense kernel; ragged M, N not a multiple of the 128-column
    wave tile, a single row; deterministic."""
    from src.moe import _lib as L

    g = torch.Generator().manual_seed(K + 7 * M + N)
    gy = torch.randn(K, M, generator=g).to(torch.bfloat16).cuda()
    x = torch.randn(K, N, generator=g).to(torch.bfloat16).cuda()
    dw, db = L.linear_wgrad_narrow(gy, x, out_dtype)
    assert dw.shape == (M, N) and db.shape == (M,) and dw.dtype == db.dtype == out_dtype
    ref_w = gy.double().t().mm(x.double())
    tol_w = 1e-5 * gy.double().abs().t().mm(x.double().abs()) + 1e-30
    ref_b = gy.double().sum(0)
    tol_b = 1e-5 * gy.double().abs().sum(0) + 1e-30
    if out_dtype == torch.bfloat16:
        tol_w = tol_w + ref_w.abs() * 2.0 ** -8
        tol_b = tol_b + ref_b.abs() * 2.0 ** -8
    assert bool(((dw.double() - ref_w).abs() <= tol_w).all()), float(((dw.double() - ref_w).abs() - tol_w).max())
    assert bool(((db.double() - ref_b).abs() <= tol_b).all()), float(((db.double() - ref_b).abs() - tol_b).max())
    dw2, db2 = L.linear_wgrad_narrow(gy, x, out_dtype)
    assert torch.equal(dw, dw2) and torch.equal(db, db2)


@pytest.mark.parametrize("out_dtype", [torch.float32, torch.bfloat16])
def test_linear_wgrad_batch_mixed_shapes(hip_lib, out_dtype):
    """rtdetr_linear_wgrad_batch: 30 problems of mixed shapes (two launches of
    <= 24), outputs written into row slices of shared buffers, vs fp64 under
    the tolerance of test_linear_wgrad_dense; untouched rows stay untouched;
    deterministic."""
    from src.moe import _lib as L

    g = torch.Generator().manual_seed(11)
    shapes = [(2400, 256, 256), (2400, 512, 256), (2400, 192, 256), (7360, 256, 256), (777, 64, 128),
              (4800, 1024, 256), (512, 128, 384)] * 4 + [(2400, 256, 256), (65535, 64, 128)]
    jobs, refs = [], []
    for K, M, N in shapes:
        gy = torch.randn(K, M, generator=g).to(torch.bfloat16).cuda()
        x = torch.randn(K, N, generator=g).to(torch.bfloat16).cuda()
        big_w = torch.full((M + 64, N), 7.0, dtype=out_dtype, device="cuda")  # rows [32, 32 + M) are the target
        big_b = torch.full((M + 64,), 7.0, dtype=out_dtype, device="cuda")
        jobs.append((gy, x, big_w[32:32 + M], big_b[32:32 + M]))
        refs.append((big_w, big_b))
    L.linear_wgrad_batch(jobs, out_dtype)
    first = [(w.clone(), b.clone()) for w, b in refs]
    for (gy, x, dw, db), (big_w, big_b) in zip(jobs, refs):
        ref_w = gy.double().t().mm(x.double())
        tol_w = 1e-5 * gy.double().abs().t().mm(x.double().abs()) + 1e-30
        ref_b = gy.double().sum(0)
        tol_b = 1e-5 * gy.double().abs().sum(0) + 1e-30
        if out_dtype == torch.bfloat16:
            tol_w = tol_w + ref_w.abs() * 2.0 ** -8
            tol_b = tol_b + ref_b.abs() * 2.0 ** -8
        assert bool(((dw.double() - ref_w).abs() <= tol_w).all())
        assert bool(((db.double() - ref_b).abs() <= tol_b).all())
        assert bool((big_w[:32] == 7).all() and (big_w[32 + dw.shape[0]:] == 7).all())
        assert bool((big_b[:32] == 7).all() and (big_b[32 + db.shape[0]:] == 7).all())
    L.linear_wgrad_batch(jobs, out_dtype)
    for (w0, b0), (w1, b1) in zip(first, refs):
        assert torch.equal(w0, w1) and torch.equal(b0, b1)


def test_deferred_weight_grads_match_autograd(hip_lib):
    """Inside deferred_weight_grads(), TokenLinear / TokenSelfAttention weight
    and bias gradients (incl. in_proj row slices and a layer applied twice) are
    collected and computed after the backward; merged, they equal the
    per-layer path's gradients within the dense-wgrad tolerance."""
    from src.rtdetr_moe.linear import TokenLinear, TokenSelfAttention, deferred_weight_grads, merge_deferred

    torch.manual_seed(0)
    lin1 = TokenLinear(256, 512).cuda().to(torch.bfloat16)
    lin2 = TokenLinear(512, 256).cuda().to(torch.bfloat16)
    attn = TokenSelfAttention(256, 8).cuda().to(torch.bfloat16)
    params = list(lin1.parameters()) + list(lin2.parameters()) + list(attn.parameters())
    x = torch.randn(8, 300, 256, device="cuda", dtype=torch.bfloat16)
    pos = torch.randn(8, 300, 256, device="cuda", dtype=torch.bfloat16)

    def loss_fn():
        h = lin2(torch.relu(lin1(x)))
        h = lin2(torch.relu(lin1(h)))  # the same layers twice
        y = attn(h + pos, h)
        return (y.float() ** 2).mean()

    ref = torch.autograd.grad(loss_fn(), params)
    with deferred_weight_grads() as d:
        got = torch.autograd.grad(loss_fn(), params, allow_unused=True)
    assert d is not None and len(d.items) > 0
    got = merge_deferred(params, got, d)
    for p, r, gg in zip(params, ref, got):
        assert gg is not None and gg.shape == p.shape and gg.dtype == r.dtype
        err = (gg.float() - r.float()).norm() / r.float().norm().clamp_min(1e-12)
        assert float(err) < 1e-2, float(err)
