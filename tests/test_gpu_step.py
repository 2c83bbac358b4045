"""TrainStep on the GPU in both precisions (bench.py's step), small model."""
from __future__ import annotations

import pytest
import torch

DEV = "cuda"


def _setup():
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.data import SyntheticZOD
    from src.rtdetr_moe.model import RTDETRMoE

    torch.manual_seed(0)
    model = RTDETRMoE("rtdetr-r18-moe4-top2").to(DEV).to(memory_format=torch.channels_last)
    images, targets, ctx = SyntheticZOD(batch=2, img_h=256, img_w=320, seed=3).sample(DEV)
    images = images.contiguous(memory_format=torch.channels_last)
    targets = [{k: v.to(DEV) for k, v in t.items()} for t in targets]
    return model, SetCriterion(num_classes=1), images, targets, ctx


@pytest.mark.gpu
@pytest.mark.parametrize("precision", ["bf16", "amp"])
def test_train_step_precisions(hip_lib, precision):
    from src.rtdetr_moe.step import TrainStep

    model, crit, images, targets, ctx = _setup()
    w0 = model.decoder.dec_score_head[0].weight.detach().float().clone()
    step = TrainStep(model, crit, images, ctx, graphs=False, world=1, precision=precision, lr=1e-3)
    losses = [float(step(images, ctx, targets, 4.0)) for _ in range(4)]
    torch.cuda.synchronize()
    assert all(torch.isfinite(torch.tensor(losses))), losses
    assert min(losses[1:]) < losses[0], losses  # same batch: the loss must go down
    w1 = model.decoder.dec_score_head[0].weight
    assert not torch.equal(w1.detach().float(), w0)
    if precision == "bf16":
        assert w1.dtype == torch.bfloat16
        for p, m in zip(step.lowp, step.master):  # bf16 weights are the rounded masters
            assert torch.equal(p.detach(), m.to(torch.bfloat16))


@pytest.mark.gpu
def test_graphed_step_matches_eager(hip_lib):
    """GraphedModel (forward + backward hipGraphs, static gradient buffers)
    follows the eager step: same losses over a few steps from the same init."""
    from src.rtdetr_moe.step import TrainStep

    runs = {}
    for graphs in (False, True):
        model, crit, images, targets, ctx = _setup()
        step = TrainStep(model, crit, images, ctx, graphs=graphs, world=1, precision="bf16", lr=1e-3)
        runs[graphs] = [float(step(images, ctx, targets, 4.0)) for _ in range(3)]
    torch.cuda.synchronize()
    eager, graph = runs[False], runs[True]
    assert min(graph[1:]) < graph[0], graph
    for a, b in zip(eager, graph):
        assert abs(a - b) <= 2e-2 * max(1.0, abs(a)), (eager, graph)
