"""HIP multi-head self-attention (csrc/attn.hip: rtdetr_attn_fwd / _bwd) vs a
plain PyTorch fp32 reference of the same op on the same bf16 inputs.

Shapes: the C2 encoder (AIFI, 920 tokens per image, batch 8) and decoder (300
queries), plus ragged lengths that leave partial 64-row tiles (1, 7, 65, 130)
and a single image.  8 heads x 32 dims, q and k read in place from one fused
[B, L, 2d] projection output.

Tolerance (stated): outputs and input gradients are bf16; the kernel rounds
P (and dS) to bf16 before the second product like every flash-attention
kernel, so per element |err| <= 2e-2 max|ref| and relative Frobenius error
<= 1e-2 against fp32 math on the same bf16 operands.  Repeated launches are
bitwise identical (no atomics)."""
from __future__ import annotations

import math

import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
H, DH = 8, 32
D = H * DH


def _ref(qk, v):
    B, L, _ = qk.shape
    q, k = qk.float().split(D, -1)
    heads = lambda t: t.reshape(B, L, H, DH).transpose(1, 2)  # noqa: E731
    s = heads(q) @ heads(k).transpose(-1, -2) / math.sqrt(DH)
    o = torch.softmax(s, -1) @ heads(v.float())
    return o.transpose(1, 2).reshape(B, L, D)


def _check(got, ref, what):
    got, ref = got.float(), ref.float()
    assert torch.isfinite(got).all(), what
    err = (got - ref).abs().max().item()
    scale = ref.abs().max().item()
    rel = ((got - ref).norm() / ref.norm().clamp(min=1e-30)).item()
    assert err <= 2e-2 * scale + 1e-6, f"{what}: max err {err:.3e} vs max|ref| {scale:.3e}"
    # relative Frobenius, with an absolute floor for outputs that vanish in exact
    # math (L = 1: dS = P (dP - delta) = 0, the kernel returns rounding noise)
    assert (got - ref).norm().item() <= 1e-2 * ref.norm().item() + 1e-6 * got.numel() ** 0.5, \
        f"{what}: relative Frobenius {rel:.3e}"
    return rel


@pytest.mark.parametrize("B,L", [(8, 920), (8, 300), (1, 1), (2, 7), (2, 65), (1, 130), (1, 920)])
def test_attention_fwd_bwd_vs_fp32(hip_lib, B, L):
    from src.rtdetr_moe.linear import self_attention_hip

    g = torch.Generator(device=DEV).manual_seed(B * 1000 + L)
    qk = (torch.randn(B, L, 2 * D, device=DEV, generator=g) * 1.5).to(torch.bfloat16)
    v = torch.randn(B, L, D, device=DEV, generator=g).to(torch.bfloat16)
    do = torch.randn(B, L, D, device=DEV, generator=g).to(torch.bfloat16)
    a = qk.clone().requires_grad_(True)
    b = v.clone().requires_grad_(True)
    o = self_attention_hip(a, b, H)
    o.backward(do)
    ra = qk.float().requires_grad_(True)
    rb = v.float().requires_grad_(True)
    ro = _ref(ra, rb)
    ro.backward(do.float())
    torch.cuda.synchronize()
    _check(o, ro, "o")
    _check(a.grad[..., :D], ra.grad[..., :D], "dq")
    _check(a.grad[..., D:], ra.grad[..., D:], "dk")
    _check(b.grad, rb.grad, "dv")
    # repeatable bit for bit
    a2 = qk.clone().requires_grad_(True)
    b2 = v.clone().requires_grad_(True)
    o2 = self_attention_hip(a2, b2, H)
    o2.backward(do)
    torch.cuda.synchronize()
    assert torch.equal(o, o2) and torch.equal(a.grad, a2.grad) and torch.equal(b.grad, b2.grad)


def test_token_self_attention_matches_multihead_attention(hip_lib):
    """TokenSelfAttention on the GPU (HIP attention, bf16) vs
    nn.MultiheadAttention in fp32 on the CPU with the same parameters
    (q = k = x + pos, v = x): output and parameter gradients."""
    from src.rtdetr_moe.linear import TokenSelfAttention

    torch.manual_seed(0)
    B, L = 2, 300
    m = TokenSelfAttention(D, H)
    ref = torch.nn.MultiheadAttention(D, H, batch_first=True)
    ref.load_state_dict(m.state_dict())
    x = torch.randn(B, L, D)
    pos = torch.randn(B, L, D) * 0.5
    dy = torch.randn(B, L, D)
    y_ref, _ = ref(x + pos, x + pos, x, need_weights=False)
    y_ref.backward(dy)
    mg = m.to(DEV)
    xg = x.to(DEV).to(torch.bfloat16)
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = mg(xg + pos.to(DEV).to(torch.bfloat16), xg)
    y.float().backward(dy.to(DEV))
    torch.cuda.synchronize()
    _check(y.cpu(), y_ref.detach(), "y")
    for n, p in mg.named_parameters():
        rp = dict(ref.named_parameters())[n]
        rel = ((p.grad.float().cpu() - rp.grad).norm() / rp.grad.norm().clamp(min=1e-30)).item()
        assert rel <= 2e-2, f"{n}: relative Frobenius {rel:.3e}"
