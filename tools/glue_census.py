"""Census of the torch (non-libmoe_hip) elementwise / copy / concatenation /
fill ops in one eager C2 training step, attributed to this repository's
source: each op large enough to matter (>= 100k elements) is logged by a
TorchDispatchMode with its shapes and the nearest repository frame of the
Python stack -- or, for ops the autograd engine issues (gradient
accumulation, built-in backward formulas), the autograd node running and the
forward line that created it (anomaly mode keeps the forward traceback).
Finds the adds, copies and fills that the graphed step replays around the HIP
kernels (launch floor).

  python tools/glue_census.py [--workload c2] > census.txt
"""
from __future__ import annotations

import argparse
import collections
import os
import sys
import traceback

import torch
from torch.utils._python_dispatch import TorchDispatchMode

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "multimodal-moe_amd"))

import bench  # noqa: E402  (WORKLOADS, build_model)

WATCH = ("add", "add_", "cat", "copy_", "mul", "mul_", "fill_", "zero_", "clone", "_to_copy", "index_add_",
         "scatter_add_", "scatter_add", "index_put_", "sub", "where", "threshold_backward", "new_zeros", "zeros_like",
         "sum", "div", "neg", "slice_backward", "select_backward", "masked_fill_", "gather", "scatter")
MIN_NUMEL = int(os.environ.get("CENSUS_MIN_NUMEL", "100000"))


def _where():
    for fr in reversed(traceback.extract_stack()[:-3]):
        f = fr.filename
        if ("/src/" in f or f.endswith("bench.py")) and "glue_census" not in f:
            return f"{f.split('multimodal-moe_amd/')[-1]}:{fr.lineno} {fr.name}"
    node = torch._C._current_autograd_node()
    if node is not None:
        tb = node.metadata.get("traceback_") if hasattr(node, "metadata") else None
        line = "?"
        if tb:
            text = "".join(tb) if isinstance(tb, list) else str(tb)
            for ln in reversed(text.splitlines()):
                if "/src/" in ln and "File" in ln:
                    line = ln.strip().split("multimodal-moe_amd/")[-1]
                    break
        return f"[bwd {node.name()}] fwd {line}"
    return "[engine]"


class Census(TorchDispatchMode):
    def __init__(self):
        super().__init__()
        self.rows = collections.Counter()

    def __torch_dispatch__(self, func, types, args=(), kwargs=None):
        out = func(*args, **(kwargs or {}))
        name = func.overloadpacket.__name__
        if name in WATCH:
            ts = [a for a in list(args) + list((kwargs or {}).values()) if isinstance(a, torch.Tensor)]
            for a in args:
                if isinstance(a, (list, tuple)):
                    ts += [t for t in a if isinstance(t, torch.Tensor)]
            outs = [o for o in (out if isinstance(out, (tuple, list)) else [out]) if isinstance(o, torch.Tensor)]
            big = max([t.numel() for t in ts + outs] or [0])
            if big >= MIN_NUMEL and any(t.is_cuda for t in ts + outs):
                shapes = tuple(tuple(t.shape) for t in ts)[:3]
                self.rows[(name, shapes, big, _where())] += 1
        return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--workload", default="c2")
    args = ap.parse_args()
    from src.moe import _lib as L
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.data import SyntheticZOD
    from src.rtdetr_moe.step import TrainStep

    L.lib()
    wl = bench.WORKLOADS[args.workload]
    device = torch.device("cuda", 0)
    model = bench.build_model(wl["spec"].format(N=1), device, 1)
    images, targets, ctx = SyntheticZOD(batch=wl["batch"], img_h=720, img_w=1280, seed=1000).sample()
    images = images.to(device).contiguous(memory_format=torch.channels_last)
    ctx = ctx.to(device)
    targets = [{k: v.to(device) for k, v in t.items()} for t in targets]
    nb = float(sum(len(t["boxes"]) for t in targets))
    step = TrainStep(model, SetCriterion(num_classes=1), images, ctx, graphs=False, world=1, precision="bf16")
    for _ in range(2):
        step(images, ctx, targets, nb)
    torch.cuda.synchronize()
    census = Census()
    with torch.autograd.detect_anomaly(check_nan=False), census:
        step(images, ctx, targets, nb)
        torch.cuda.synchronize()
    rows = sorted(census.rows.items(), key=lambda kv: -kv[0][2] * kv[1])
    print(f"# ops >= {MIN_NUMEL} elements in one eager step: {sum(census.rows.values())}")
    for (name, shapes, big, where), n in rows:
        print(f"{n:3d}x {big / 1e6:7.2f}M {name:18s} {str(shapes)[:70]:70s} {where}")


if __name__ == "__main__":
    main()
