"""The captured training graph is ONE chain ("Graph capture").

A graph with parallel branches makes the HIP runtime give its exec parallel
streams; round 3's captures on torch's separate capture stream held 109-127
fork nodes and, late in a long process, segfaulted inside hipGraphLaunch
(profiles/r03/graphs/).  Captured on the warm-up stream every graph is a
single chain: 1 root, 0 forks, 0 joins -- asserted here for bench.py's
whole-step graph (forward + criterion with the GPU matcher + backward) and
the two-graph mode, so any side-stream overlap added later is a visible,
tested decision.  Topology from hipGraphGetEdges (tools/graph_topology.py)."""
from __future__ import annotations

import sys
from pathlib import Path

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = Path(__file__).resolve().parents[1]


@pytest.mark.parametrize("spec,whole", [("rtdetr-r50-moe8-top2", True), ("rtdetr-r18-moe4-top1", False),
                                        ("rtdetr-r18-moe32-top4-cf1.25-fp8", True)])
def test_captured_step_graph_is_one_chain(hip_lib, monkeypatch, spec, whole):
    sys.path.insert(0, str(ROOT / "tools"))
    import graph_topology as gt

    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.data import SyntheticZOD
    from src.rtdetr_moe.model import RTDETRMoE
    from src.rtdetr_moe.step import TrainStep

    monkeypatch.setattr(torch.cuda, "CUDAGraph", gt._KeptGraph)
    n0 = len(gt.DUMPED)
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RTDETRMoE(spec).to(dev).to(memory_format=torch.channels_last)
    images, targets, ctx = SyntheticZOD(batch=2, img_h=256, img_w=320, seed=3).sample(dev)
    images = images.contiguous(memory_format=torch.channels_last)
    targets = [{k: v.to(dev) for k, v in t.items()} for t in targets]
    step = TrainStep(model, SetCriterion(num_classes=1), images, ctx, targets=targets if whole else None,
                     graphs=True, world=1, precision="bf16", lr=1e-3)
    assert torch.isfinite(step(images, ctx, targets, 4.0))
    torch.cuda.synchronize()
    graphs = gt.DUMPED[n0:]
    assert len(graphs) == (1 if whole else 2)
    for g in graphs:
        topo = gt.topology(g)
        assert topo["nodes"] > 100
        assert topo["roots"] == 1 and topo["forks"] == 0 and topo["joins"] == 0, topo
    del gt.DUMPED[n0:]
