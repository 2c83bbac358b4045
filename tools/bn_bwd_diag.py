"""Diagnostic (GPU box): conv1x1 + training BatchNorm backward on bf16
channels_last activations -- MIOpen (nn.BatchNorm2d) vs libmoe_hip bn_act --
against fp32 CPU, at the decoder input_proj shapes."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "multimodal-moe_amd"))
import torch  # noqa: E402

from src.rtdetr_moe.fused import bn_act, bn_act_ok  # noqa: E402


def rel(a, b):
    return float((a.float().cpu() - b.float()).norm() / b.float().norm())


for shape, mean in (((1, 256, 92, 160), 0.0), ((1, 256, 23, 40), 0.0), ((1, 256, 92, 160), 3.0), ((1, 256, 23, 40), 3.0),
                    ((1, 256, 23, 40), 10.0), ((8, 256, 46, 80), 3.0)):
    g = torch.Generator().manual_seed(0)
    x = torch.randn(shape, generator=g).abs() * (1.0 if mean else 1.0) + mean
    w = torch.randn(256, shape[1], 1, 1, generator=g) / 16 + (0.02 if mean else 0.0)
    dy = torch.randn(shape, generator=g)
    # reference fp32 CPU
    xr = x.clone().requires_grad_(True)
    bnr = torch.nn.BatchNorm2d(256)
    yr = bnr(torch.nn.functional.conv2d(xr, w))
    yr.backward(dy)
    res = {}
    for mode in ("miopen", "hip"):
        xg = x.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_(True)
        wg = w.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        bn = torch.nn.BatchNorm2d(256).cuda()
        c = torch.nn.functional.conv2d(xg, wg)
        if mode == "miopen":
            y = bn(c)
        else:
            assert bn_act_ok([c], [bn])
            y = bn_act([c], [bn], None)
        y.backward(dy.cuda().to(torch.bfloat16).contiguous(memory_format=torch.channels_last))
        torch.cuda.synchronize()
        res[mode] = (rel(y.detach(), yr.detach()), rel(xg.grad, xr.grad), rel(bn.weight.grad, bnr.weight.grad))
    print(shape, "mean", mean, {k: [round(v, 4) for v in vals] for k, vals in res.items()}, "(y, dx, dgamma rel err)")
