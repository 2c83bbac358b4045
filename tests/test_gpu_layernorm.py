"""GPU parity of the fused residual-add + LayerNorm (rtdetr_add_layer_norm_*,
src/rtdetr_moe/norm.py) against torch's fp32 LayerNorm of the same bf16
inputs.  Tolerances:
  out, ds (bf16): |err| <= 1 bf16 ulp of max(|got|, |ref|) + 1e-3 x RMS(ref)
    (fp32 statistics in another summation order, then one rounding);
  dgamma, dbeta: relative Frobenius error <= 1e-5 (fp32 out) / 4e-3 (bf16 out);
  repeated launches bit-identical (fixed-order partial sums, no atomics).
"""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ulp_close(got, ref, what):
    got, ref = got.double(), ref.double()
    m = torch.maximum(got.abs(), ref.abs()).clamp_min(1e-30)
    ulp = torch.exp2(torch.floor(torch.log2(m)) - 7)
    rms = ref.pow(2).mean().sqrt()
    bad = (got - ref).abs() > ulp + 1e-3 * rms
    assert not bool(bad.any()), f"{what}: {int(bad.sum())} elements beyond tolerance, max err " \
                                f"{float((got - ref).abs().max()):.3e}"


def _rel(got, ref):
    got, ref = got.double(), ref.double()
    return float((got - ref).norm() / ref.norm().clamp_min(1e-30))


@pytest.mark.parametrize("T,d", [(1, 256), (17, 128), (2400, 256), (7360, 256), (300, 512)])
@pytest.mark.parametrize("with_b", [True, False])
@pytest.mark.parametrize("wdtype", [torch.bfloat16, torch.float32])
def test_add_layer_norm_matches_torch(hip_lib, T, d, with_b, wdtype):
    from src.rtdetr_moe.norm import add_layer_norm

    g = torch.Generator(device=DEV).manual_seed(T * 7 + d)
    a = (torch.randn((T, d), device=DEV, generator=g) * 2 + 0.5).to(torch.bfloat16).requires_grad_(True)
    b = torch.randn((T, d), device=DEV, generator=g).to(torch.bfloat16).requires_grad_(True) if with_b else None
    w = (1 + 0.3 * torch.randn(d, device=DEV, generator=g)).to(wdtype).requires_grad_(True)
    bias = (0.2 * torch.randn(d, device=DEV, generator=g)).to(wdtype).requires_grad_(True)
    dout = torch.randn((T, d), device=DEV, generator=g).to(torch.bfloat16)

    out = add_layer_norm(a, b, w, bias, 1e-5)
    out.backward(dout)
    torch.cuda.synchronize()

    a32 = a.detach().float().requires_grad_(True)
    b32 = b.detach().float().requires_grad_(True) if with_b else None
    w32 = w.detach().float().requires_grad_(True)
    bias32 = bias.detach().float().requires_grad_(True)
    ref = F.layer_norm(a32 + b32 if with_b else a32, (d,), w32, bias32, 1e-5)
    ref.backward(dout.float())

    assert out.dtype == torch.bfloat16
    _ulp_close(out.float(), ref.detach(), "out")
    _ulp_close(a.grad.float(), a32.grad, "da")
    if with_b:
        assert torch.equal(a.grad, b.grad)  # d(a + b): the same gradient for both
    tol = 1e-5 if wdtype == torch.float32 else 4e-3
    assert w.grad.dtype == wdtype and bias.grad.dtype == wdtype
    assert _rel(w.grad, w32.grad) <= tol, f"dgamma rel err {_rel(w.grad, w32.grad):.2e}"
    assert _rel(bias.grad, bias32.grad) <= tol, f"dbeta rel err {_rel(bias.grad, bias32.grad):.2e}"


def test_add_layer_norm_deterministic_and_module(hip_lib):
    """Two launches give bit-identical outputs and gradients; AddLayerNorm
    (nn.LayerNorm parameters / state dict) equals the functional form and
    falls back to torch for fp32 activations."""
    from src.rtdetr_moe.norm import AddLayerNorm

    torch.manual_seed(0)
    m = AddLayerNorm(256).to(DEV)
    m.weight.data = (1 + 0.1 * torch.randn(256, device=DEV)).to(torch.bfloat16)
    m.bias.data = (0.1 * torch.randn(256, device=DEV)).to(torch.bfloat16)
    a0 = torch.randn((8, 300, 256), device=DEV).to(torch.bfloat16)
    b0 = torch.randn((8, 300, 256), device=DEV).to(torch.bfloat16)
    dout = torch.randn((8, 300, 256), device=DEV).to(torch.bfloat16)
    res = []
    for _ in range(2):
        a, b = a0.clone().requires_grad_(True), b0.clone().requires_grad_(True)
        m.zero_grad(set_to_none=True)
        y = m(a, b)
        y.backward(dout)
        res.append((y, a.grad, m.weight.grad, m.bias.grad))
    for x, z in zip(*res):
        assert torch.equal(x, z)
    assert set(m.state_dict()) == {"weight", "bias"}
    y32 = AddLayerNorm(256).to(DEV)(a0.float(), b0.float())  # fp32: torch path
    ref = F.layer_norm(a0.float() + b0.float(), (256,))
    assert torch.allclose(y32, ref, atol=1e-6)


def test_add_layer_norm_rejects_bad_shapes(hip_lib):
    from src.moe import _lib as L

    lib = L.lib()
    x = torch.zeros((4, 192), dtype=torch.bfloat16, device=DEV)
    w = torch.ones(192, dtype=torch.bfloat16, device=DEV)
    out = torch.empty_like(x)
    st = torch.empty(4, device=DEV)
    rc = lib.rtdetr_add_layer_norm_fwd(x.data_ptr(), None, w.data_ptr(), w.data_ptr(), 1, 4, 192, 1e-5,
                                       out.data_ptr(), st.data_ptr(), st.data_ptr(), L._stream())
    assert rc != 0 and b"d must be" in lib.moe_last_error()


@pytest.mark.parametrize("wdtype", [torch.float32, torch.bfloat16])
def test_add_layer_norm_with_pos_matches_separate_add(hip_lib, wdtype):
    """AddLayerNorm.with_pos (t and t + pos from one launch, the two gradients
    of t summed inside the LayerNorm backward) == LayerNorm(a + b) followed by
    a separate `t + pos`, outputs and every gradient bit for bit (the kernel
    sums the two bf16 gradients in bf16 exactly as autograd's accumulation)."""
    from src.rtdetr_moe import norm as N

    torch.manual_seed(4)
    ln = N.AddLayerNorm(256).cuda().to(wdtype)
    with torch.no_grad():
        ln.weight.add_(torch.randn_like(ln.weight) * 0.1)
        ln.bias.add_(torch.randn_like(ln.bias) * 0.1)
    a, b, pos = (torch.randn(8, 300, 256, device="cuda").to(torch.bfloat16) for _ in range(3))
    g1, g2 = (torch.randn(8, 300, 256, device="cuda").to(torch.bfloat16) for _ in range(2))
    res = []
    for fused in (True, False):
        aa, bb, pp = (t.clone().requires_grad_(True) for t in (a, b, pos))
        if fused:
            t, q = ln.with_pos(aa, bb, pp)
            assert q.grad_fn.name() == "_AddLayerNormPosBackward"
        else:
            t = ln(aa, bb)
            q = t + pp
        grads = torch.autograd.grad((t, q), (aa, bb, pp, ln.weight, ln.bias), (g1, g2))
        res.append((t, q) + grads)
    torch.cuda.synchronize()
    for x, y in zip(*res):
        assert torch.equal(x, y)
