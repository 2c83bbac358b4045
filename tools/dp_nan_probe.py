"""Diagnostic: single-process whole-step graph replays of the DP test's model
on two images; reports NaN gradients per parameter and re-captures."""
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "multimodal-moe_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from src.rtdetr_moe.criterion import SetCriterion  # noqa: E402
from src.rtdetr_moe.data import SyntheticZOD  # noqa: E402
from src.rtdetr_moe.model import RTDETRMoE  # noqa: E402
from src.rtdetr_moe.step import TrainStep  # noqa: E402

dev = torch.device("cuda", 0)
prec = sys.argv[1] if len(sys.argv) > 1 else "bf16"


def data(rank):
    images, targets, ctx = SyntheticZOD(batch=1, img_h=256, img_w=256, seed=11 + rank).sample(dev)
    return images.contiguous(memory_format=torch.channels_last), [{k: v.to(dev) for k, v in t.items()} for t in targets], ctx


torch.manual_seed(0)
model = RTDETRMoE("rtdetr-r18-moe4-top2-dec2").to(dev).to(memory_format=torch.channels_last)
images, targets, ctx = data(0)
step = TrainStep(model, SetCriterion(num_classes=1), images, ctx, graphs=True, world=1, lr=1e-3, precision=prec,
                 targets=targets, num_boxes=2.0)
names = [n for n, p in model.named_parameters() if p.requires_grad]
for it in range(2):
    for r in range(2):
        images, targets, ctx = data(r)
        step.stepper(step._cast_in(images), ctx, targets, 2.0)
        torch.cuda.synchronize()
        bad = [n for n, g in zip(names, step.stepper.static_grads) if not torch.isfinite(g.float()).all()]
        print(f"iter {it} rank-image {r} boxes {[len(t['boxes']) for t in targets]} M {step.stepper.M} "
              f"captures {step.stepper.captures} loss {float(step.stepper.static_loss):.4f} nonfinite {len(bad)} "
              f"{bad[:6]}", flush=True)
