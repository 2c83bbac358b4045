"""Attribute the C2 training step's GPU time to PyTorch ops (with input shapes).

Builds the bench.py workload, runs warm-up steps, then profiles `--steps`
steps with torch.profiler and writes two tables to --out:
  * ops by self device time (grouped by op name and input shapes),
  * kernels by device time.
    python tools/torch_prof.py --out gpurun_out/tprof.txt
"""
from __future__ import annotations

import argparse
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=2)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--out", default="gpurun_out/tprof.txt")
    ap.add_argument("--spec", default="rtdetr-r50-moe8-top2")
    ap.add_argument("--batch", type=int, default=8)
    a = ap.parse_args()

    import bench
    from src.moe import _lib as L
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.data import SyntheticZOD
    from src.rtdetr_moe.step import TrainStep

    L.lib()
    bench.heartbeat()
    torch.backends.cudnn.benchmark = True  # as bench.py (--conv-search)
    dev = torch.device("cuda", 0)
    model = bench.build_model(a.spec, dev, 1)
    data = SyntheticZOD(batch=a.batch, img_h=720, img_w=1280, seed=1000)
    images, targets, ctx = data.sample()
    images = images.to(dev).contiguous(memory_format=torch.channels_last)
    ctx = ctx.to(dev)
    targets = [{k: v.to(dev) for k, v in t.items()} for t in targets]
    nb = max(1.0, float(sum(len(t["boxes"]) for t in targets)))
    step = TrainStep(model, SetCriterion(num_classes=1), images, ctx, graphs=False, world=1)
    for _ in range(a.warmup):
        step(images, ctx, targets, nb)
    torch.cuda.synchronize()
    acts = [torch.profiler.ProfilerActivity.CPU, torch.profiler.ProfilerActivity.CUDA]
    with torch.profiler.profile(activities=acts, record_shapes=True) as prof:
        for _ in range(a.steps):
            step(images, ctx, targets, nb)
        torch.cuda.synchronize()
    out = Path(a.out)
    out.parent.mkdir(parents=True, exist_ok=True)
    ka = prof.key_averages(group_by_input_shape=True)
    with open(out, "w") as f:
        f.write(f"# {a.steps} profiled steps of {a.spec} batch {a.batch}\n")
        f.write(ka.table(sort_by="self_device_time_total", row_limit=80, max_name_column_width=60,
                         max_shapes_column_width=100))
        f.write("\n\n# by op name\n")
        f.write(prof.key_averages().table(sort_by="device_time_total", row_limit=80, max_name_column_width=60))
    print(f"wrote {out}")


if __name__ == "__main__":
    main()
