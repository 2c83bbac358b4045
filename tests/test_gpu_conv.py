"""HIP implicit-GEMM convolutions (csrc/conv.hip) vs a plain PyTorch fp32
reference of the same op (F.conv2d on the same bf16 operands, upcast):
forward, data gradient and weight gradient, 1x1 and 3x3, stride 1 with
"same" padding, and 3x3 stride 2 (padding 1), NHWC bf16.

Forward tiles of 64, 128 and 256 pixels (rtdetr_conv_set_tuning "conv_bm"),
weight-gradient rings of 2, 3 and 4 stages ("conv_wg_stages"), 1 / 3 /
automatic pixel slices ("conv_wg_splits"), the data gradient with the weight
flipped into a workspace and read in place ("conv_dgrad_flip"), and the
automatic choices.  Shapes: the C2 encoder's RepVGG convolutions (256 -> 256 at 23x40, batch 8),
a ResNet bottleneck shape (128 channels), channel-asymmetric layers
(stride 2: the ResNet-D stage entries and the encoder's downsampling layers,
odd input sizes included),
(512 -> 128, 128 -> 256), 64-channel inputs / outputs (ResNet stage 1: the
64-wide tiles), odd spatial sizes (7 x 9: the partial 128-pixel tile and every
padding case) and a single image.

Tolerance (stated): bf16 outputs of fp32 accumulations over K = KS^2 Cin
(up to 4,608 terms), so relative Frobenius error <= 1e-2 and per element
|err| <= 2e-2 max|ref|; the weight gradient's pixel slices are summed in a
fixed order, so repeated launches are bitwise identical."""
from __future__ import annotations

import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _check(got, ref, what):
    got, ref = got.float(), ref.float()
    assert torch.isfinite(got).all(), what
    err = (got - ref).abs().max().item()
    rel = ((got - ref).norm() / ref.norm().clamp(min=1e-30)).item()
    assert err <= 2e-2 * ref.abs().max().item() + 1e-6, f"{what}: max err {err:.3e}"
    assert rel <= 1e-2, f"{what}: relative Frobenius {rel:.3e}"


_KNOBS = {"auto": {}, "bm64_wg2_flip": dict(conv_bm=64, conv_wg_stages=2, conv_dgrad_flip=1),
          "bm128_wg3_inplace": dict(conv_bm=128, conv_wg_stages=3, conv_dgrad_flip=0, conv_wg_splits=3),
          "bm256_wg4_flip": dict(conv_bm=256, conv_wg_stages=4, conv_dgrad_flip=1, conv_wg_splits=1),
          "zero_rows": dict(conv_dgrad_phase=0), "zero_rows_inplace": dict(conv_dgrad_phase=0, conv_dgrad_flip=0),
          "big8w_flip": dict(conv_big=1, conv_dgrad_flip=1), "big8w_inplace": dict(conv_big=1, conv_dgrad_flip=0),
          # the A operand in registers (128-row tiles), flipped / in-place weights, zero-row stride-2 dgrad
          "areg_flip": dict(conv_areg=1, conv_bm=128, conv_dgrad_flip=1),
          "areg_inplace": dict(conv_areg=1, conv_bm=128, conv_dgrad_flip=0),
          "areg_zero_rows": dict(conv_areg=1, conv_bm=128, conv_dgrad_phase=0),
          # 32-deep K-tiles, ring depth 2 / 3 / 4 (128- and 64-row tiles)
          "k32_s2_flip": dict(conv_k32=1, conv_dgrad_flip=1), "k32_s3_inplace": dict(conv_k32=2, conv_dgrad_flip=0),
          "k32_s4_bm64": dict(conv_k32=3, conv_bm=64), "k32_s2_zero_rows": dict(conv_k32=1, conv_dgrad_phase=0),
          "k32_off": dict(conv_k32=0),
          # the halo-staged 3x3 stride-1 kernel (256 x 128 / 128 x 128 tiles; the flipped-weight data gradient)
          "halo256_flip": dict(conv_halo=1, conv_dgrad_flip=1), "halo128_flip": dict(conv_halo=2, conv_dgrad_flip=1),
          "halo256_inplace": dict(conv_halo=1, conv_dgrad_flip=0), "halo_off": dict(conv_halo=0),
          # the 256 x 256 eight-phase kernel (N % 256 == 0 and an even K-tile count; else the default tiles)
          "ph8_flip": dict(conv_8ph=1, conv_dgrad_flip=1), "ph8_off": dict(conv_8ph=0)}
_DEFAULTS = dict(conv_bm=0, conv_wg_stages=0, conv_dgrad_flip=-1, conv_wg_splits=0, conv_dgrad_phase=1, conv_big=0,
                 conv_areg=0, conv_k32=-1, conv_halo=-1, conv_8ph=-1)


@pytest.mark.parametrize("knobs", list(_KNOBS))
@pytest.mark.parametrize("B,C,N,H,W,ks", [(8, 256, 256, 23, 40, 3), (8, 256, 256, 23, 40, 1), (2, 128, 128, 46, 80, 3),
                                          (2, 512, 128, 7, 9, 1), (2, 128, 256, 7, 9, 3), (1, 256, 512, 5, 3, 3),
                                          # 64-channel tiles (ResNet stage 1): output, input and both
                                          (2, 64, 64, 23, 40, 3), (2, 256, 64, 7, 9, 1), (2, 64, 256, 11, 13, 1),
                                          (1, 64, 128, 5, 3, 3), (2, 128, 64, 9, 7, 3),
                                          # one-row / one-column images, a row wider than the halo tile
                                          (2, 64, 128, 1, 7, 3), (3, 64, 128, 6, 1, 3), (2, 128, 128, 3, 300, 3)])
def test_conv_fwd_bwd_vs_fp32(hip_lib, B, C, N, H, W, ks, knobs):
    for k, v in _KNOBS[knobs].items():
        assert hip_lib.rtdetr_conv_set_tuning(k.encode(), v) == 0
    try:
        _conv_case(B, C, N, H, W, ks)
    finally:
        for k, v in _DEFAULTS.items():
            hip_lib.rtdetr_conv_set_tuning(k.encode(), v)


def test_conv_large_auto_paths(hip_lib):
    """A stride-8 encoder shape: the automatic choices there (flipped-weight
    data gradient, a non-multiple-of-8 slice count) against fp32."""
    assert hip_lib.rtdetr_conv_dgrad_workspace(8, 92, 160, 256, 256, 3) > 0
    assert hip_lib.rtdetr_conv_dgrad_workspace(8, 23, 40, 256, 256, 3) == 0
    _conv_case(4, 256, 256, 92, 160, 3)


@pytest.mark.parametrize("knobs", ["auto", "bm64_wg2_flip", "bm128_wg3_inplace", "zero_rows", "zero_rows_inplace",
                                   "big8w_flip", "big8w_inplace", "areg_flip", "areg_inplace", "areg_zero_rows",
                                   "k32_s2_flip", "k32_s3_inplace", "k32_s4_bm64", "k32_s2_zero_rows"])
@pytest.mark.parametrize("B,C,N,H,W", [(2, 128, 128, 46, 80), (8, 256, 256, 23, 40), (2, 64, 128, 11, 13),
                                       (1, 256, 512, 5, 3), (2, 128, 64, 7, 9), (4, 256, 256, 92, 160)])
def test_conv_stride2_vs_fp32(hip_lib, B, C, N, H, W, knobs):
    """3x3 stride-2 convolutions (padding 1, even and odd input sizes):
    forward, the data gradient (per parity class over its valid taps, or all
    nine taps with zero rows) and the strided weight gradient."""
    for k, v in _KNOBS[knobs].items():
        assert hip_lib.rtdetr_conv_set_tuning(k.encode(), v) == 0
    try:
        _conv_case(B, C, N, H, W, 3, stride=2)
    finally:
        for k, v in _DEFAULTS.items():
            hip_lib.rtdetr_conv_set_tuning(k.encode(), v)


def _conv_case(B, C, N, H, W, ks, stride=1):
    from src.rtdetr_moe.conv import _ConvHIP, hip_conv_ok

    g = torch.Generator(device=DEV).manual_seed(B + C + N + H + ks)
    x = torch.randn(B, C, H, W, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(N, C, ks, ks, device=DEV, generator=g) * (C * ks * ks) ** -0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    gy = torch.randn(B, N, Ho, Wo, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert hip_conv_ok(x, w, stride, (ks - 1) // 2)
    xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
    y = _ConvHIP.apply(xa, wa, None, False, False, False, None, stride)
    assert y.shape == (B, N, Ho, Wo) and y.is_contiguous(memory_format=torch.channels_last)
    gx, gw = torch.autograd.grad(y, (xa, wa), gy)
    xr, wr = x.float().requires_grad_(True), w.float().requires_grad_(True)
    yr = F.conv2d(xr, wr, None, stride, (ks - 1) // 2)
    gxr, gwr = torch.autograd.grad(yr, (xr, wr), gy.float())
    torch.cuda.synchronize()
    _check(y, yr, "y")
    _check(gx, gxr, "dx")
    _check(gw, gwr, "dw")
    y2 = _ConvHIP.apply(xa, wa, None, False, False, False, None, stride)
    gx2, gw2 = torch.autograd.grad(y2, (xa, wa), gy)
    torch.cuda.synchronize()
    assert torch.equal(y, y2) and torch.equal(gx, gx2) and torch.equal(gw, gw2)


def test_conv_dispatch_rules(hip_lib):
    """Only the covered convolutions take the HIP kernels."""
    from src.rtdetr_moe.conv import hip_conv_ok

    x = torch.zeros(1, 256, 8, 8, device=DEV, dtype=torch.bfloat16)
    w3 = torch.zeros(256, 256, 3, 3, device=DEV, dtype=torch.bfloat16)
    w1 = torch.zeros(256, 256, 1, 1, device=DEV, dtype=torch.bfloat16)
    assert hip_conv_ok(x, w3, 1, 1) and hip_conv_ok(x, w3, 2, 1) and not hip_conv_ok(x, w3, 1, 0)
    assert hip_conv_ok(x, w1, 1, 0) and not hip_conv_ok(x, w1, 2, 0) and not hip_conv_ok(x, w3, 3, 1)
    assert not hip_conv_ok(x.float(), w3.float(), 1, 1)
    assert hip_conv_ok(torch.zeros(1, 64, 8, 8, device=DEV, dtype=torch.bfloat16),
                       torch.zeros(64, 64, 3, 3, device=DEV, dtype=torch.bfloat16), 1, 1)
    assert not hip_conv_ok(torch.zeros(1, 32, 8, 8, device=DEV, dtype=torch.bfloat16),
                           torch.zeros(64, 32, 3, 3, device=DEV, dtype=torch.bfloat16), 1, 1)


@pytest.mark.parametrize("ks,halo", [(1, 0), (3, 0), (3, 1), (3, 2)])
def test_conv_fused_epilogues_match_separate_kernels(hip_lib, ks, halo):
    """The forward epilogue relu((conv + resid) + bias) and the dgrad's ReLU
    mask equal the separate kernels they replace (rtdetr_add_bias_relu_nhwc,
    rtdetr_bias_act_nhwc, threshold_backward) bit for bit."""
    from src.moe import _lib as L
    from src.rtdetr_moe import conv as C

    g = torch.Generator(device=DEV).manual_seed(5 + ks)
    B, Ci, Co, H, W = 2, 256, 128, 11, 13
    cl = dict(memory_format=torch.channels_last)
    x = torch.randn(B, Ci, H, W, device=DEV, generator=g).to(torch.bfloat16).contiguous(**cl)
    w = (torch.randn(Co, Ci, ks, ks, device=DEV, generator=g) * (Ci * ks * ks) ** -0.5).to(torch.bfloat16).contiguous(**cl)
    bias = torch.randn(Co, device=DEV, generator=g) * 0.3
    resid = torch.randn(B, Co, H, W, device=DEV, generator=g).to(torch.bfloat16).contiguous(**cl)
    assert hip_lib.rtdetr_conv_set_tuning(b"conv_halo", halo) == 0
    try:
        plain = C._fwd(x, w)
        assert torch.equal(C._fwd(x, w, bias, resid, True), L.add_bias_relu_nhwc(plain, resid, bias))
        assert torch.equal(C._fwd(x, w, bias, None, True), L.bias_act_nhwc(plain.clone(), bias, True))
        gy = torch.randn(B, Co, H, W, device=DEV, generator=g).to(torch.bfloat16).contiguous(**cl)
        xr = torch.relu(x)  # a ReLU output feeding the convolution
        gx_m, gw_m = C._bwd(xr, w, gy, True, True, True)
        gx, gw = C._bwd(xr, w, gy, True, True, False)
        torch.cuda.synchronize()
        assert torch.equal(gx_m, torch.ops.aten.threshold_backward(gx, xr, 0)) and torch.equal(gw_m, gw)
    finally:
        hip_lib.rtdetr_conv_set_tuning(b"conv_halo", -1)


@pytest.mark.parametrize("cin,width,stride,shortcut", [(512, 128, 1, True), (256, 128, 2, False), (1024, 256, 1, True),
                                                      (64, 64, 1, False), (256, 64, 1, True)])
def test_bottleneck_fused_matches_unfused(hip_lib, cin, width, stride, shortcut):
    """A frozen-BN ResNet bottleneck with the fused convolution epilogues
    (MOE_CONV_EPI, default) against the separate bias / add / ReLU kernels:
    output handles, input gradient and every weight gradient bitwise equal
    (stride 2 / projection shortcut: the mixed fused + MIOpen case)."""
    from src.rtdetr_moe import backbone as BB

    torch.manual_seed(3)
    blk = BB.BottleNeck(cin, width, stride, shortcut, True).to(DEV)
    blk = blk.to(torch.bfloat16).to(memory_format=torch.channels_last)
    with torch.no_grad():
        for m in blk.modules():
            if isinstance(m, BB.FrozenBatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 2.0)
                m.bias.uniform_(-0.3, 0.3)
    x0 = torch.randn(2, cin, 24, 40, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g1 = torch.randn(2, width * 4, 24 // stride, 40 // stride, device=DEV).to(torch.bfloat16)
    g2 = torch.randn_like(g1)
    res = []
    for fused in (True, False):
        BB._FUSED_EPI = fused
        try:
            x = x0.clone().requires_grad_(True)
            # the MIOpen layer (stride 2) on deterministic solvers, so the comparison is bitwise
            with torch.backends.cudnn.flags(enabled=True, benchmark=False, deterministic=True):
                y1, y2 = blk(x)
                params = [p for p in blk.parameters() if p.requires_grad]
                grads = torch.autograd.grad([y1, y2], [x] + params, [g1.contiguous(memory_format=torch.channels_last),
                                                                   g2.contiguous(memory_format=torch.channels_last)])
            torch.cuda.synchronize()
            res.append((y1.detach().clone(), [gg.clone() for gg in grads]))
        finally:
            BB._FUSED_EPI = True
    (ya, ga), (yb, gb) = res
    assert torch.equal(ya, yb)
    for u, v in zip(ga, gb):
        assert torch.equal(u, v)


@pytest.mark.parametrize("cin,width", [(256, 64), (512, 128)])
def test_block_chain_grad_link_matches_unfused(hip_lib, cin, width):
    """Two identity-shortcut bottlenecks chained as PResNet chains them: the
    first block's output gradient is finished in the second block's branch2a
    dgrad epilogue (GradLink: + the shortcut gradient, ReLU mask) instead of
    rtdetr_relu_grad2 -- bitwise equal to the unfused chain."""
    from src.rtdetr_moe import backbone as BB

    torch.manual_seed(4)
    blks = torch.nn.ModuleList([BB.BottleNeck(cin, width, 1, True, True) for _ in range(2)]).to(DEV)
    blks = blks.to(torch.bfloat16).to(memory_format=torch.channels_last)
    with torch.no_grad():
        for m in blks.modules():
            if isinstance(m, BB.FrozenBatchNorm2d):
                m.running_mean.uniform_(-0.2, 0.2)
                m.running_var.uniform_(0.5, 2.0)
                m.bias.uniform_(-0.3, 0.3)
    x0 = torch.randn(2, cin, 16, 24, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g1 = torch.randn(2, cin, 16, 24, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g2 = torch.randn_like(g1)
    res = []
    for fused in (True, False):
        BB._FUSED_EPI = fused
        try:
            x = x0.clone().requires_grad_(True)
            y, ys = blks[0](x)
            z1, z2 = blks[1](y, ys)
            params = [p for p in blks.parameters() if p.requires_grad]
            grads = torch.autograd.grad([z1, z2], [x] + params, [g1, g2])
            torch.cuda.synchronize()
            res.append((z1.detach().clone(), [gg.clone() for gg in grads]))
        finally:
            BB._FUSED_EPI = True
    (za, ga), (zb, gb) = res
    assert torch.equal(za, zb)
    for u, v in zip(ga, gb):
        assert torch.equal(u, v)


@pytest.mark.parametrize("B,C,N,H,W", [(2, 128, 128, 46, 80), (2, 64, 128, 11, 13), (1, 256, 512, 5, 3)])
def test_conv_stride2_dgrad_classes_match_zero_rows(hip_lib, B, C, N, H, W):
    """The parity-class data gradient sums the same nonzero products in the
    same order as the all-taps zero-row form: bitwise equal, with the fused
    add + ReLU-mask epilogue scattered to the class pixels."""
    from src.rtdetr_moe import conv as CV

    g = torch.Generator(device=DEV).manual_seed(H * W + C)
    cl = dict(memory_format=torch.channels_last)
    x = torch.relu(torch.randn(B, C, H, W, device=DEV, generator=g)).to(torch.bfloat16).contiguous(**cl)
    w = (torch.randn(N, C, 3, 3, device=DEV, generator=g) * (9 * C) ** -0.5).to(torch.bfloat16).contiguous(**cl)
    gy = torch.randn(B, N, (H + 1) // 2, (W + 1) // 2, device=DEV, generator=g).to(torch.bfloat16).contiguous(**cl)
    add = torch.randn(B, C, H, W, device=DEV, generator=g).to(torch.bfloat16).contiguous(**cl)
    outs = []
    for phase in (1, 0):
        assert hip_lib.rtdetr_conv_set_tuning(b"conv_dgrad_phase", phase) == 0
        try:
            outs.append(CV._bwd(x, w, gy, True, False, True, add, 2)[0])
        finally:
            hip_lib.rtdetr_conv_set_tuning(b"conv_dgrad_phase", 1)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])


@pytest.mark.parametrize("alt", ["conv_big:1", "conv_k32:1", "conv_k32:2", "conv_k32:3", "conv_8ph:1"])
@pytest.mark.parametrize("ks", [3, 1])
@pytest.mark.parametrize("stride", [1, 2])
@pytest.mark.parametrize("flip", [1, 0])
def test_conv_big_tile_bit_exact(hip_lib, stride, flip, alt, ks):
    """The 8-wave 256 x 128 tile ("conv_big"), the 32-deep K-tiles
    ("conv_k32", one k-step per stage) and the 256 x 256 eight-phase kernel
    ("conv_8ph") run every output element's K loop in
    the same order as the 4-wave 128 x 128 tile: forward and data gradient bit
    for bit equal (128-channel shapes; 64-channel outputs keep the 64-wide
    tiles)."""
    knob, val = alt.split(":")
    if ks == 1 and stride == 2:
        pytest.skip("1x1 convolutions run at stride 1")
    from src.rtdetr_moe.conv import _ConvHIP

    g = torch.Generator(device=DEV).manual_seed(11 + stride)
    B, C, N, H, W = 4, 256, 256, 46, 80
    x = torch.randn(B, C, H, W, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(N, C, ks, ks, device=DEV, generator=g) * (C * ks * ks) ** -0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
    gy = torch.randn(B, N, Ho, Wo, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = []
    try:
        assert hip_lib.rtdetr_conv_set_tuning(b"conv_dgrad_flip", flip) == 0
        for v in (0, int(val)):
            assert hip_lib.rtdetr_conv_set_tuning(knob.encode(), v) == 0
            xa, wa = x.clone().requires_grad_(True), w.clone().requires_grad_(True)
            y = _ConvHIP.apply(xa, wa, None, False, False, False, None, stride)
            gx, = torch.autograd.grad(y, (xa,), gy)
            torch.cuda.synchronize()
            res.append((y, gx))
    finally:
        for k, v in _DEFAULTS.items():
            hip_lib.rtdetr_conv_set_tuning(k.encode(), v)
    assert torch.equal(res[0][0], res[1][0]) and torch.equal(res[0][1], res[1][1])


def test_batched_flip_matches_per_call_flip(hip_lib):
    """rtdetr_conv_weight_flip_multi + rtdetr_conv_dgrad_preflipped (conv.batched_flips, GraphedStep) give
    bitwise the data gradient of the per-call flip, for two weights of different shapes in one table."""
    from src.moe import _lib as L
    from src.rtdetr_moe import conv as Cv

    dev = torch.device("cuda")
    torch.manual_seed(3)
    cases = [(8, 256, 256, 92, 160, 3), (8, 512, 256, 92, 160, 1)]
    ws, gs, xs = [], [], []
    for B, C, N, H, W, ks in cases:
        assert L.lib().rtdetr_conv_dgrad_workspace(B, H, W, C, N, ks) > 0  # shapes that flip
        ws.append((torch.randn(N, C, ks, ks, device=dev) * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last))
        xs.append(torch.randn(B, C, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
        gs.append(torch.randn(B, N, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
    ref = [Cv._bwd(x, w, g, True, False, False)[0] for x, w, g in zip(xs, ws, gs)]
    Cv._FLIP_REG.clear()
    Cv._FLIP_TABLE[:] = [None, 0, 0, 0]
    try:
        with Cv.batched_flips(dev):  # registers (per-call flips into the persistent buffers)
            first = [Cv._bwd(x, w, g, True, False, False)[0] for x, w, g in zip(xs, ws, gs)]
        assert len(Cv._FLIP_REG) == 2
        for bufs in Cv._FLIP_REG.values():
            bufs.zero_()  # the batched flip must rewrite them
        with Cv.batched_flips(dev):  # one multi-flip launch, then the preflipped data gradients
            second = [Cv._bwd(x, w, g, True, False, False)[0] for x, w, g in zip(xs, ws, gs)]
        torch.cuda.synchronize()
        for r, a, b in zip(ref, first, second):
            assert torch.equal(r, a) and torch.equal(r, b)
    finally:
        Cv._FLIP_REG.clear()
        Cv._FLIP_TABLE[:] = [None, 0, 0, 0]


@pytest.mark.parametrize("C,N,H,W", [(256, 256, 46, 80), (256, 128, 23, 40)])
def test_conv_pair_matches_two_convolutions(hip_lib, C, N, H, W):
    """conv.conv_pair (RepVgg 3x3 + 1x1 on one input, one autograd node whose
    second data gradient adds the first in its epilogue) == two separate HIP
    convolutions: outputs and weight gradients bitwise, the input gradient
    within one bf16 rounding of autograd's bf16 sum of the two."""
    from src.rtdetr_moe import conv as Cv

    torch.manual_seed(5)
    dev = torch.device("cuda")
    c1 = torch.nn.Conv2d(C, N, 3, 1, 1, bias=False).to(dev, torch.bfloat16).to(memory_format=torch.channels_last)
    c2 = torch.nn.Conv2d(C, N, 1, 1, 0, bias=False).to(dev, torch.bfloat16).to(memory_format=torch.channels_last)
    x = torch.randn(4, C, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    g1, g2 = (torch.randn(4, N, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
              for _ in range(2))
    outs = []
    for pair in (True, False):
        xa = x.clone().requires_grad_(True)
        y1, y2 = Cv.conv_pair(c1, c2, xa) if pair else (Cv.conv_module(c1, xa), Cv.conv_module(c2, xa))
        assert (y1.grad_fn.name() == "_ConvHIPPairBackward") == pair
        grads = torch.autograd.grad((y1, y2), (xa, c1.weight, c2.weight), (g1, g2))
        outs.append((y1, y2) + grads)
    torch.cuda.synchronize()
    (a1, a2, ax, aw1, aw2), (b1, b2, bx, bw1, bw2) = outs
    assert torch.equal(a1, b1) and torch.equal(a2, b2) and torch.equal(aw1, bw1) and torch.equal(aw2, bw2)
    d = (ax.float() - bx.float()).abs()
    assert d.max().item() <= 2 ** -7 * bx.float().abs().max().item()


@pytest.mark.parametrize("B,C,N,H,W,ks,st", [(8, 256, 256, 92, 160, 1, 1), (8, 256, 256, 46, 80, 3, 2),
                                             (8, 256, 256, 92, 160, 3, 1),  # the 8-phase kernel: 256-row partials
                                             (2, 128, 256, 23, 40, 3, 1), (1, 64, 128, 7, 9, 1, 1)])
def test_conv_fwd_stats_partials(hip_lib, B, C, N, H, W, ks, st):
    """rtdetr_conv_fwd_stats: the output equals rtdetr_conv_fwd's bit for bit,
    and its per-row-block partials are the column sums and sums of squares of
    that bf16 output (fp64 reference; ragged last block, 64- and 128-row
    tiles, stride 2)."""
    from src.rtdetr_moe import conv as Cv

    torch.manual_seed(B + C + H)
    dev = torch.device("cuda")
    x = torch.randn(B, C, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(N, C, ks, ks, device=dev) * 0.05).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    nblk = Cv._stats_blocks(x, w, st)
    assert nblk > 0
    part = torch.full((nblk, 2, N), float("nan"), device=dev)
    y = Cv._fwd_stats(x, w, part, st)
    y0 = Cv._fwd(x, w, st=st)
    torch.cuda.synchronize()
    assert torch.equal(y, y0)
    rows = -(-y.shape[0] * y.shape[2] * y.shape[3] // nblk)
    yf = y.permute(0, 2, 3, 1).reshape(-1, N).double()
    for blk in (0, nblk - 1):
        seg = yf[blk * rows:(blk + 1) * rows]
        assert torch.allclose(part[blk, 0].double(), seg.sum(0), rtol=1e-5, atol=1e-3)
        assert torch.allclose(part[blk, 1].double(), (seg * seg).sum(0), rtol=1e-5, atol=1e-3)
    tot = part.double().sum(0)
    assert torch.allclose(tot[0], yf.sum(0), rtol=1e-5, atol=1e-2)
    assert torch.allclose(tot[1], (yf * yf).sum(0), rtol=1e-5, atol=1e-2)


def test_bn_act_with_conv_stats_matches_stats_pass(hip_lib):
    """ConvNormLayer / RepVgg with the BatchNorm statistics from the conv
    epilogue (MOE_CONV_BN_STATS, default) vs the separate statistics pass:
    the same outputs up to the statistics' summation order, the same running
    statistics and gradients to fp32 rounding."""
    import copy

    from src.rtdetr_moe import conv as Cv
    from src.rtdetr_moe.encoder import RepVggBlock

    torch.manual_seed(11)
    dev = torch.device("cuda")
    blk = RepVggBlock(256, 256).to(dev).to(memory_format=torch.channels_last)
    for m in blk.modules():
        if isinstance(m, torch.nn.Conv2d):
            m.to(torch.bfloat16)
    blk.train()
    x = torch.randn(4, 256, 46, 80, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    gy = torch.randn(4, 256, 46, 80, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    res = []
    for on in (True, False):
        b = copy.deepcopy(blk)
        Cv._STATS_ON = on
        try:
            xa = x.clone().requires_grad_(True)
            y = b(xa)
            g = torch.autograd.grad(y, [xa] + [p for p in b.parameters()], gy)
        finally:
            Cv._STATS_ON = True
        res.append((y, g, [t.clone() for t in (b.conv1.norm.running_mean, b.conv1.norm.running_var,
                                                   b.conv2.norm.running_mean, b.conv2.norm.running_var)]))
    torch.cuda.synchronize()
    (ya, ga, ra), (yb, gb, rb) = res
    assert (ya.float() - yb.float()).abs().max().item() <= 2 ** -6 * yb.float().abs().max().item()
    for a, b in zip(ra, rb):
        assert torch.allclose(a, b, rtol=1e-5, atol=1e-6)
    for a, b in zip(ga, gb):
        assert ((a.float() - b.float()).norm() / b.float().norm().clamp_min(1e-12)).item() < 1e-2


@pytest.mark.parametrize("B,H,W,st", [(2, 64, 96, 2), (1, 37, 50, 2), (2, 20, 24, 1)])
def test_conv3x3_direct_stem_vs_fp32(hip_lib, B, H, W, st):
    """rtdetr_conv3x3_direct_fwd (the stem's 3 -> 32 layer, bias + ReLU, odd
    sizes, NCHW- and channels_last-strided weights) against fp32."""
    from src.moe import _lib as L

    g = torch.Generator(device=DEV).manual_seed(H + W)
    x = torch.randn(B, 3, H, W, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(32, 3, 3, 3, device=DEV, generator=g) * 0.3).to(torch.bfloat16)
    b = torch.randn(32, device=DEV, generator=g)
    ref = torch.nn.functional.conv2d(x.float(), w.float(), b, st, 1).relu()
    for wl in (w, w.contiguous(memory_format=torch.channels_last)):
        y = L.conv3x3_direct_fwd(x, wl, b, st, True)
        assert y.shape == ref.shape and y.is_contiguous(memory_format=torch.channels_last)
        _check(y, ref, "direct stem conv")


@pytest.mark.parametrize("C,N,ks,st", [(32, 32, 3, 1), (32, 64, 3, 1), (32, 96, 1, 1), (64, 32, 3, 2), (96, 64, 3, 1)])
def test_conv_fwd_32_channel_multiples(hip_lib, C, N, ks, st):
    """The implicit-GEMM forward on 32-channel multiples (32-deep K-tiles, a
    partial last output-channel tile), with the bias + ReLU epilogue, against
    fp32."""
    from src.rtdetr_moe.conv import _fwd

    g = torch.Generator(device=DEV).manual_seed(C + N + ks)
    B, H, W = 2, 23, 41
    x = torch.randn(B, C, H, W, device=DEV, generator=g).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w = (torch.randn(N, C, ks, ks, device=DEV, generator=g) * (C * ks * ks) ** -0.5).to(torch.bfloat16)
    w = w.contiguous(memory_format=torch.channels_last)
    b = torch.randn(N, device=DEV, generator=g)
    y = _fwd(x, w, b, None, True, st)
    ref = torch.nn.functional.conv2d(x.float(), w.float(), b, st, (ks - 1) // 2).relu()
    _check(y, ref, "32-channel conv fwd")


def test_stem_hip_matches_modules(hip_lib, monkeypatch):
    """PResNet's frozen stem on libmoe_hip (direct 3 -> 32, implicit GEMMs
    for 32 -> 32 -> 64 with the folded shift + ReLU in the epilogue) against
    the modules (MIOpen + the bias/ReLU kernel): within bf16 rounding."""
    from src.rtdetr_moe import backbone as bb

    torch.manual_seed(3)
    m = bb.PResNet(50).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    for mod in m.stem.modules():
        if hasattr(mod, "running_var") and not isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_var.uniform_(0.5, 2.0)
            mod.running_mean.uniform_(-0.2, 0.2)
    x = torch.randn(2, 3, 96, 160, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    with torch.no_grad():
        for mode in (2, 1, 0):
            monkeypatch.setattr(bb, "_STEM_HIP", mode)
            assert m._stem_hip_ok(x) == (mode > 0)
            outs.append(m._stem(x))
    _check(outs[0], outs[2], "stem (all HIP)")
    _check(outs[1], outs[2], "stem (direct first layer)")
    # the evaluation forward's case: fp32 input (and fp32 weights) under bf16 autocast
    m32 = bb.PResNet(50).to(DEV).to(memory_format=torch.channels_last)
    m32.load_state_dict(m.state_dict())
    x32 = x.float().contiguous(memory_format=torch.channels_last)
    outs = []
    with torch.no_grad(), torch.autocast("cuda", dtype=torch.bfloat16):
        for mode in (2, 0):
            monkeypatch.setattr(bb, "_STEM_HIP", mode)
            assert m32._stem_hip_ok(x32) == (mode > 0)
            outs.append(m32._stem(x32))
    assert outs[0].dtype == torch.bfloat16
    _check(outs[0], outs[1], "stem under autocast")


def test_wgrad_reduce_batch_matches_per_call(hip_lib):
    """rtdetr_conv_wgrad_part + ONE rtdetr_conv_wgrad_reduce_batch over weights of different shapes and slice
    counts (conv.deferred_wgrads) == rtdetr_conv_wgrad per weight, bitwise; a batch of 1..48, 16-B checks."""
    from src.moe import _lib as L
    from src.rtdetr_moe import conv as Cv

    dev = torch.device("cuda")
    torch.manual_seed(5)
    cases = [(8, 128, 128, 92, 160, 3, 1), (8, 512, 256, 23, 40, 1, 1), (2, 64, 64, 46, 80, 3, 2),
             (4, 256, 128, 23, 40, 3, 1), (1, 64, 128, 9, 7, 1, 1)]
    xs, ws, gs = [], [], []
    for B, C, N, H, W, ks, st in cases:
        Ho, Wo = (H + 2 * (ks // 2) - ks) // st + 1, (W + 2 * (ks // 2) - ks) // st + 1
        xs.append(torch.randn(B, C, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
        ws.append((torch.randn(N, C, ks, ks, device=dev) * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last))
        gs.append(torch.randn(B, N, Ho, Wo, device=dev).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last))
    ref = [Cv._bwd(x, w, g, False, True, False, st=c[6])[1] for x, w, g, c in zip(xs, ws, gs, cases)]
    with Cv.deferred_wgrads():
        got = [Cv._bwd(x, w, g, False, True, False, st=c[6])[1] for x, w, g, c in zip(xs, ws, gs, cases)]
        assert len(Cv._WG_PENDING[0]) == len(cases)
    assert Cv._WG_PENDING[0] is None
    torch.cuda.synchronize()
    for c, r, a in zip(cases, ref, got):
        assert torch.equal(r, a), c
    # argument checks (no launch)
    import ctypes

    one = (ctypes.c_void_p * 1)(None)
    ns = (ctypes.c_int * 1)(1)
    nw = (ctypes.c_longlong * 1)(4)
    cv = lambda a: ctypes.cast(a, ctypes.c_void_p)  # noqa: E731
    assert L.lib().rtdetr_conv_wgrad_reduce_batch(1, cv(one), cv(ns), cv(nw), cv(one), 1, None) != 0
    assert L.lib().rtdetr_conv_wgrad_reduce_batch(49, cv(one), cv(ns), cv(nw), cv(one), 1, None) != 0


def test_deferred_wgrads_backbone_bitwise(hip_lib):
    """A PResNet-50 backward (frozen-BN folds: _FoldAll's backward flushes the pending sums first) with every
    convolution's weight-gradient reduction deferred and batched == the per-convolution reductions, bitwise,
    for every parameter gradient."""
    from src.rtdetr_moe import conv as Cv
    from src.rtdetr_moe.backbone import PResNet

    torch.manual_seed(0)
    m = PResNet(50).to(DEV).to(torch.bfloat16).to(memory_format=torch.channels_last)
    for mod in m.modules():
        if hasattr(mod, "running_var") and not isinstance(mod, torch.nn.BatchNorm2d):
            mod.running_var.uniform_(0.5, 2.0)
            mod.weight.uniform_(0.5, 1.5)
    x = torch.randn(2, 3, 128, 160, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    params = [p for p in m.parameters() if p.requires_grad]
    res = []
    for defer in (False, True):
        outs = m(x)
        loss = sum((o.float() * torch.linspace(-1, 1, o.numel(), device=DEV).view_as(o)).sum() for o in outs)
        with Cv.deferred_wgrads(enabled=defer):
            grads = torch.autograd.grad(loss, params, allow_unused=True)
        torch.cuda.synchronize()
        res.append([None if g is None else g.clone() for g in grads])
    n = 0
    for p, a, b in zip(params, res[0], res[1]):
        assert (a is None) == (b is None)
        if a is not None:
            assert torch.equal(a, b)
            n += 1
    assert n > 20, n
