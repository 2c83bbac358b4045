"""Diagnostic: gradients of one GraphedStep replay vs the eager step's
(same weights and inputs); prints the parameters that differ most."""
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parents[1] / "multimodal-moe_amd"))
import torch  # noqa: E402

from src.rtdetr_moe.criterion import SetCriterion, pad_targets  # noqa: E402
from src.rtdetr_moe.data import SyntheticZOD  # noqa: E402
from src.rtdetr_moe.model import RTDETRMoE  # noqa: E402
from src.rtdetr_moe.step import FlatOutputs, TrainStep  # noqa: E402

DEV = "cuda"
torch.manual_seed(0)
model = RTDETRMoE("rtdetr-r18-moe4-top2").to(DEV).to(memory_format=torch.channels_last)
images, targets, ctx = SyntheticZOD(batch=2, img_h=256, img_w=320, seed=6).sample(DEV)
images = images.contiguous(memory_format=torch.channels_last)
targets = [{k: v.to(DEV) for k, v in t.items()} for t in targets]
nb = max(1.0, float(sum(len(t["boxes"]) for t in targets)))
crit = SetCriterion(num_classes=1)
step = TrainStep(model, crit, images, ctx, graphs=True, world=1, precision="bf16", lr=1e-3, targets=targets,
                 num_boxes=nb)
names = {id(p): n for n, p in model.named_parameters()}
gl = float(step.stepper(step._cast_in(images), ctx, targets, nb))
gg = [g.detach().float().clone() for g in step.stepper.static_grads]
flat = FlatOutputs(model)
for mode in ("host", "padded"):
    out, aux = FlatOutputs.unflatten(flat(step._cast_in(images), ctx))
    if mode == "host":
        losses = crit(out, targets, nb)
    else:
        tb, tl, nv = pad_targets(targets, 16)
        losses = crit.forward_padded(out, tb, tl, nv, torch.tensor(nb, device=DEV))
    loss = sum(losses.values()) + aux
    eg = torch.autograd.grad(loss, step.params, allow_unused=True)
    print(f"{mode}: eager loss {float(loss):.6f} graph loss {gl:.6f}")
    rows = []
    for p, a, b in zip(step.params, gg, eg):
        b = torch.zeros_like(a) if b is None else b.float()
        err = float((a - b).norm() / max(float(b.norm()), 1e-12))
        rows.append((err, names.get(id(p), "?"), float(a.norm()), float(b.norm())))
    rows.sort(reverse=True)
    for r in rows[:12]:
        print(f"  rel {r[0]:.3e}  {r[1]}  |graph| {r[2]:.4e} |eager| {r[3]:.4e}")
