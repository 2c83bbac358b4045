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
    ap.add_argument("--single-ctx", action="store_true", help="single-context batches (bench.py c4)")
    ap.add_argument("--glue-shapes", action="store_true",
                    help="record shapes: glue ops (adds, casts, fills) grouped by input shape")
    ap.add_argument("--stacks", action="store_true",
                    help="also attribute glue ops (casts, adds, fills, ReLU backward) to source lines")
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
    data = SyntheticZOD(batch=a.batch, img_h=720, img_w=1280, seed=1000, single_context=0 if a.single_ctx else None)
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
    cfg = torch._C._profiler._ExperimentalConfig(verbose=True) if a.stacks else None
    with torch.profiler.profile(activities=acts, record_shapes=a.glue_shapes or not a.stacks, with_stack=a.stacks,
                                experimental_config=cfg) as prof:
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
        if a.glue_shapes:
            f.write("\n\n# glue ops by input shape (count per step, device ms per step)\n")
            rows = [(e.device_time_total / 1e3 / a.steps, e.count / a.steps, e.key, str(e.input_shapes)[:150])
                    for e in ka if e.key in GLUE]
            rows.sort(key=lambda r: -r[0])
            f.write("\n".join(f"{t:8.3f} ms {c:7.1f}/step  {n:26s} {sh}" for t, c, n, sh in rows[:80]) + "\n")
        if a.stacks:
            f.write("\n\n# glue ops by source line (count per step, device ms per step)\n")
            f.write(glue_by_line(prof, a.steps))
    print(f"wrote {out}")


GLUE = {"aten::_to_copy", "aten::copy_", "aten::add", "aten::add_", "aten::fill_", "aten::zero_", "aten::zeros",
        "aten::threshold_backward", "aten::mul", "aten::mul_", "aten::sum", "aten::cat", "aten::clone",
        "aten::contiguous", "aten::div", "aten::sub", "aten::where", "aten::index", "aten::index_put_"}


def glue_by_line(prof, steps):
    rows = []
    for e in prof.key_averages(group_by_stack_n=12):
        if e.key not in GLUE:
            continue
        frames = [fr for fr in (e.stack or []) if "rtdetr_moe" in fr or "/moe/" in fr or "models/" in fr]
        src = " <- ".join(fr.split("src/")[-1] for fr in frames[:3]) or "(autograd engine)"
        rows.append((e.device_time_total / 1e3 / steps, e.count / steps, e.key, src))
    rows.sort(key=lambda r: -r[0])
    return "\n".join(f"{t:8.3f} ms {c:7.1f}/step  {n:26s} {src}" for t, c, n, src in rows[:80]) + "\n"


if __name__ == "__main__":
    main()
