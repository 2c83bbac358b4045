"""Diagnostic: a stride-2 3x3 convolution (MIOpen) forward + backward captured
in a hipGraph, warm-up and capture on the same stream (A) or on different
streams (B); replays on two inputs and compares the weight gradient with the
eager one (finite, relative error).

  python tools/miopen_graph_probe.py
"""
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "multimodal-moe_amd")):
    sys.path.insert(0, p)
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
os.environ.setdefault("MIOPEN_USER_DB_PATH", str(ROOT / "multimodal-moe_amd" / "miopen_db"))
import torch  # noqa: E402

import src.rtdetr_moe  # noqa: E402,F401  (the engine's MIOpen settings)

torch.backends.cudnn.benchmark = True
dev = torch.device("cuda", 0)


def run(same_stream, cin, cout, h, w, zero_grad_in_graph):
    torch.manual_seed(0)
    conv = torch.nn.Conv2d(cin, cout, 3, stride=2, padding=1, bias=False).to(dev).to(torch.bfloat16)
    conv = conv.to(memory_format=torch.channels_last)
    xs = [torch.randn(1, cin, h, w, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
          for _ in range(2)]
    ref = []
    for x in xs:
        g, = torch.autograd.grad(conv(x).float().square().sum(), [conv.weight])
        ref.append(g.float().clone())
    sx = xs[0].clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            g, = torch.autograd.grad(conv(sx).float().square().sum(), [conv.weight])
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph, stream=side if same_stream else None):
        g, = torch.autograd.grad(conv(sx).float().square().sum(), [conv.weight])
    out = []
    for i in (0, 1, 0, 1):
        sx.copy_(xs[i])
        graph.replay()
        torch.cuda.synchronize()
        e = float((g.float() - ref[i]).norm() / ref[i].norm())
        out.append((bool(torch.isfinite(g).all()), round(e, 5)))
    return out


for shape in [(256, 256, 64, 80), (64, 128, 128, 160), (128, 256, 64, 80)]:
    for same in (True, False):
        print("same_stream" if same else "diff_stream", shape, run(same, *shape, False), flush=True)
