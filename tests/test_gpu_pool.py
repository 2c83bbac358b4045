"""GPU parity of the ResNet-D shortcut pooling (rtdetr_avgpool2x2_nhwc_fwd/_bwd)
against torch's AvgPool2d(2, 2) on the same channels_last bf16 input.

Bar: forward within 1 bf16 ulp of torch (fp32 window sum x 0.25, one rounding;
torch may sum the four terms in another order), backward bit-exact (0.25 * g is
exact in bf16)."""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("B,C,H,W", [(1, 8, 2, 2), (2, 64, 6, 10), (8, 256, 184, 320), (3, 1024, 46, 80), (1, 24, 4, 2)])
def test_avgpool2x2_matches_torch(hip_lib, B, C, H, W):
    from src.rtdetr_moe.backbone import _AvgPool2x2, avg_pool_2x2

    g = torch.Generator().manual_seed(B * C + H)
    x = torch.randn(B, C, H, W, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=torch.channels_last)
    x1 = x.clone().requires_grad_(True)
    x2 = x.clone().requires_grad_(True)
    ref = F.avg_pool2d(x1.float(), 2, 2, 0, ceil_mode=True)
    got = avg_pool_2x2(x2)
    assert got.grad_fn is not None and "AvgPool2x2" in type(got.grad_fn).__name__
    assert got.is_contiguous(memory_format=torch.channels_last) and got.shape == ref.shape
    ulp = ref.abs() * 2.0 ** -8 + 1e-30
    assert bool(((got.float() - ref).abs() <= ulp).all())
    gy = torch.randn(got.shape, generator=g).to(torch.bfloat16).cuda()
    got.backward(gy)
    gref = (gy.float().repeat_interleave(2, 2).repeat_interleave(2, 3) * 0.25).to(torch.bfloat16)
    assert torch.equal(x2.grad, gref)
    assert x2.grad.is_contiguous(memory_format=torch.channels_last)
    _ = _AvgPool2x2  # the HIP path, not the reshape-mean fallback


@pytest.mark.parametrize("B,C,H,W", [(1, 8, 1, 1), (2, 64, 7, 10), (8, 64, 368, 640), (1, 16, 5, 3), (3, 32, 2, 2)])
def test_stem_maxpool_matches_torch(hip_lib, B, C, H, W):
    """rtdetr_maxpool3x3s2_nhwc_fwd vs nn.MaxPool2d(3, 2, 1): bit-exact (a max
    of bf16 values), odd and even sizes, 1x1 input, NaN propagation."""
    from torch import nn

    from src.rtdetr_moe.backbone import stem_max_pool

    g = torch.Generator().manual_seed(B * C + H * W)
    x = torch.randn(B, C, H, W, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=torch.channels_last)
    if H * W > 4:
        x[0, 3, H // 2, W // 2] = float("nan")
    pool = nn.MaxPool2d(3, 2, 1)
    ref = pool(x)
    got = stem_max_pool(x, pool)
    assert got.grad_fn is None and got.is_contiguous(memory_format=torch.channels_last) and got.shape == ref.shape
    assert torch.equal(torch.isnan(got), torch.isnan(ref))
    assert torch.equal(got.nan_to_num(0.0), ref.nan_to_num(0.0))


@pytest.mark.parametrize("B,Ch,Cl,Hh,Wh,H,W", [(1, 8, 8, 1, 1, 2, 2), (2, 256, 256, 23, 40, 46, 80),
                                              (8, 256, 256, 46, 80, 92, 160), (2, 16, 24, 3, 5, 5, 9),
                                              (1, 8, 16, 4, 4, 7, 8)])
def test_upcat_matches_interpolate_cat(hip_lib, B, Ch, Cl, Hh, Wh, H, W):
    """rtdetr_upcat_nhwc_fwd / _bwd vs F.interpolate(x2, nearest) + crop +
    torch.cat: forward and dlow bit-exact, dhigh (2x2 block sums, fp32, one
    rounding) within one bf16 ulp of the fp32 sums; odd (cropped) levels."""
    from src.rtdetr_moe.encoder import _UpCat, up_cat

    g = torch.Generator().manual_seed(B * Ch + H * W)
    cl = torch.channels_last
    high = torch.randn(B, Ch, Hh, Wh, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=cl)
    low = torch.randn(B, Cl, H, W, generator=g).to(torch.bfloat16).cuda().contiguous(memory_format=cl)
    h1, l1 = high.clone().requires_grad_(True), low.clone().requires_grad_(True)
    h2, l2 = high.clone().requires_grad_(True), low.clone().requires_grad_(True)
    up = F.interpolate(h1, scale_factor=2.0, mode="nearest")[..., :H, :W]
    ref = torch.cat([up, l1], dim=1)
    got = up_cat(h2, l2)
    assert "UpCat" in type(got.grad_fn).__name__ and got.is_contiguous(memory_format=cl)
    assert torch.equal(got, ref)
    gy = torch.randn(ref.shape, generator=g).to(torch.bfloat16).cuda()
    ref.backward(gy)
    got.backward(gy)
    assert torch.equal(l2.grad, l1.grad)
    g32 = gy[:, :Ch].float()
    pad = torch.zeros(B, Ch, 2 * Hh, 2 * Wh, device="cuda")
    pad[..., :H, :W] = g32
    sums = pad.view(B, Ch, Hh, 2, Wh, 2).sum((3, 5))
    assert bool(((h2.grad.float() - sums).abs() <= sums.abs() * 2.0 ** -8 + 1e-30).all())
    _ = _UpCat
