"""Diagnostic: eager vs hipGraph-captured forward of the small test model
(tests/test_gpu_step.py::_setup), per fusion switch, plus the first training
losses of an eager and a whole-step-graph TrainStep.

    python tools/graph_eager_diag.py > gpurun_out/diag.jsonl
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT), str(ROOT / "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from test_gpu_step import _setup  # noqa: E402


def forward_diff():
    from src.rtdetr_moe.step import FlatOutputs, gemm_params

    model, crit, images, targets, ctx = _setup(seed=6)
    for p in gemm_params(model):
        p.data = p.data.to(torch.bfloat16)
    flat = FlatOutputs(model)
    x = images.to(torch.bfloat16)
    out_e = [t.detach().clone() for t in flat(x, ctx)]
    out_e2 = [t.detach().clone() for t in flat(x, ctx)]
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(2):
            flat(x, ctx)
    torch.cuda.current_stream().wait_stream(s)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        out_g = flat(x, ctx)
    g.replay()
    torch.cuda.synchronize()
    d_rep = max(float((a.float() - b.float()).abs().max()) for a, b in zip(out_e, out_e2))
    d_gr = [float((a.float() - b.detach().float()).abs().max()) for a, b in zip(out_e, out_g)]
    return d_rep, max(d_gr), d_gr


def first_losses():
    from src.rtdetr_moe.step import TrainStep

    runs = {}
    for whole in (False, True):
        model, crit, images, targets, ctx = _setup(seed=6)
        nb = max(1.0, float(sum(len(t["boxes"]) for t in targets)))
        step = TrainStep(model, crit, images, ctx, graphs=whole, world=1, precision="bf16", lr=1e-3,
                         targets=targets if whole else None, num_boxes=nb)
        runs[whole] = [float(step(images, ctx, targets, nb)) for _ in range(2)]
    return runs[False], runs[True]


def main():
    from src.moe import ops
    from src.rtdetr_moe import norm

    for fl, fr in [(1, 1), (0, 1), (1, 0), (0, 0)]:
        norm._FUSED_LN = bool(fl)
        ops._FUSE_RESIDUAL = bool(fr)
        d_rep, d_max, d_all = forward_diff()
        eager, graph = first_losses()
        print(json.dumps({"fused_ln": fl, "fuse_residual": fr, "eager_repeat_maxdiff": d_rep,
                          "graph_vs_eager_maxdiff": d_max, "per_output": [round(v, 6) for v in d_all],
                          "loss_eager": eager, "loss_graph": graph}), flush=True)


if __name__ == "__main__":
    main()
