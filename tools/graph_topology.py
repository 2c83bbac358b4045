"""Topology of the captured training graphs (diagnostic, GPU box).

Captures TrainStep's graphs (two-graph GraphedModel and the whole-step
GraphedStep) for a small model, keeps the hipGraph_t and reports node count,
roots, fork nodes (more than one successor) and joins from hipGraphGetEdges.  A stream-captured graph with no cross-stream fork/join is a
single chain: 1 root, 0 forks; parallel branches make the HIP runtime give
the graph exec parallel streams.

  python tools/graph_topology.py [--spec rtdetr-r18-moe32-top4-cf1.25-fp8] [--out gpurun_out/topo]
"""
from __future__ import annotations

import argparse
import collections
import ctypes
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "multimodal-moe_amd")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

DUMPED = []
_Orig = torch.cuda.CUDAGraph


class _KeptGraph(_Orig):
    """CUDAGraph that keeps its hipGraph_t after instantiation (raw_cuda_graph)."""

    def __new__(cls, keep_graph=True):
        g = super().__new__(cls, keep_graph=True)
        DUMPED.append(g)
        return g

    def __init__(self, keep_graph=True):
        try:
            super().__init__(keep_graph=True)
        except TypeError:
            super().__init__(True)


def topology(g):
    """Nodes, roots, forks and joins of the captured hipGraph (hipGraphGetEdges)."""
    hip = ctypes.CDLL(str(Path(torch.__file__).parent / "lib" / "libamdhip64.so"))
    graph = ctypes.c_void_p(g.raw_cuda_graph())
    n = ctypes.c_size_t(0)
    assert hip.hipGraphGetNodes(graph, None, ctypes.byref(n)) == 0
    nodes = (ctypes.c_void_p * n.value)()
    assert hip.hipGraphGetNodes(graph, nodes, ctypes.byref(n)) == 0
    ne = ctypes.c_size_t(0)
    assert hip.hipGraphGetEdges(graph, None, None, ctypes.byref(ne)) == 0
    fr = (ctypes.c_void_p * max(ne.value, 1))()
    to = (ctypes.c_void_p * max(ne.value, 1))()
    assert hip.hipGraphGetEdges(graph, fr, to, ctypes.byref(ne)) == 0
    succ, pred = collections.defaultdict(set), collections.defaultdict(set)
    for i in range(ne.value):
        succ[fr[i]].add(to[i])
        pred[to[i]].add(fr[i])
    ids = list(nodes)
    types = {}
    for nd in ids:
        t = ctypes.c_int(-1)
        hip.hipGraphNodeGetType(ctypes.c_void_p(nd), ctypes.byref(t))
        types[nd] = t.value
    roots = [x for x in ids if not pred[x]]
    forks = [x for x in ids if len(succ[x]) > 1]
    joins = [x for x in ids if len(pred[x]) > 1]
    order = {x: i for i, x in enumerate(ids)}
    return {"nodes": len(ids), "edges": ne.value, "roots": len(roots), "forks": len(forks), "joins": len(joins),
            "node_types": dict(collections.Counter(types.values())),
            "forks_at": [(order[x], types[x], len(succ[x])) for x in forks[:12]],
            "roots_at": [(order[x], types[x]) for x in roots[:12]]}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spec", default="rtdetr-r18-moe32-top4-cf1.25-fp8")
    ap.add_argument("--out", default=str(ROOT / "gpurun_out" / "topo"))
    a = ap.parse_args()
    out = Path(a.out)
    out.mkdir(parents=True, exist_ok=True)
    torch.cuda.CUDAGraph = _KeptGraph
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.data import SyntheticZOD
    from src.rtdetr_moe.model import RTDETRMoE
    from src.rtdetr_moe.step import TrainStep

    dev = torch.device("cuda", 0)
    for mode in ("graphed_model", "whole_step"):
        torch.manual_seed(0)
        model = RTDETRMoE(a.spec).to(dev).to(memory_format=torch.channels_last)
        images, targets, ctx = SyntheticZOD(batch=2, img_h=256, img_w=320, seed=3).sample(dev)
        images = images.contiguous(memory_format=torch.channels_last)
        targets = [{k: v.to(dev) for k, v in t.items()} for t in targets]
        n0 = len(DUMPED)
        step = TrainStep(model, SetCriterion(num_classes=1), images, ctx,
                         targets=targets if mode == "whole_step" else None, graphs=True, world=1,
                         precision="bf16", lr=1e-3)
        float(step(images, ctx, targets, 4.0))
        torch.cuda.synchronize()
        for i, g in enumerate(DUMPED[n0:]):
            print(mode, i, topology(g), flush=True)
        del step, model


if __name__ == "__main__":
    main()
