"""Graph-mode data parallelism on the GPU (bench.py's default N>1 path):
two processes on the same GPU (gloo for the gradient all-reduce, since RCCL
wants one device per rank), each runs TrainStep with the forward/backward
hipGraphs -- or the whole step as one graph (GraphedStep, bench's default) --
on its own image.  After the steps both ranks hold identical
weights, and the first step's loss matches a single-process eager step on
the same image."""
from __future__ import annotations

import os
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _worker(rank, world, port, out, whole):
    for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT)):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.data import SyntheticZOD
    from src.rtdetr_moe.model import RTDETRMoE
    from src.rtdetr_moe.step import TrainStep

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RTDETRMoE("rtdetr-r18-moe4-top2-dec2").to(dev).to(memory_format=torch.channels_last)
    images, targets, ctx = SyntheticZOD(batch=1, img_h=256, img_w=256, seed=11 + rank).sample(dev)
    images = images.contiguous(memory_format=torch.channels_last)
    targets = [{k: v.to(dev) for k, v in t.items()} for t in targets]
    step = TrainStep(model, SetCriterion(num_classes=1), images, ctx, graphs=True, world=world, lr=1e-3,
                     targets=targets if whole else None, num_boxes=2.0)
    assert (step.stepper is not None) == whole
    losses = [float(step(images, ctx, targets, 2.0)) for _ in range(2)]
    torch.cuda.synchronize()
    w = torch.cat([p.detach().float().reshape(-1) for p in model.parameters()]).cpu()
    torch.save({"w": w, "losses": losses}, out / f"r{rank}.pt")
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("whole", [False, True], ids=["fwd_bwd_graphs", "whole_step_graph"])
def test_graph_mode_data_parallel_two_ranks(hip_lib, tmp_path, whole):
    port = 29500 + os.getpid() % 1000 + (7 if whole else 0)
    mp.start_processes(_worker, args=(2, port, tmp_path, whole), nprocs=2, join=True, start_method="spawn")
    r0, r1 = torch.load(tmp_path / "r0.pt"), torch.load(tmp_path / "r1.pt")
    assert torch.equal(r0["w"], r1["w"]), "ranks diverged after the graph-mode all-reduce"
    assert all(torch.isfinite(torch.tensor(r0["losses"] + r1["losses"])))
