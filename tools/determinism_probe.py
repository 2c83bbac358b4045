"""Which kernel makes the RT-DETR-MoE forward / backward non-repeatable?

Runs the eager forward of the same model, weights and images several times
after warm-up with a forward hook on EVERY module (outputs and inputs
recorded in call order), and reports per repeat the first module whose output
differs bitwise from the first run's while its inputs are bitwise identical --
i.e. the module that itself is non-deterministic -- plus every such module.
Then the backward: parameter gradients of repeated forward+backward passes
with fixed output gradients, listing the parameters whose gradients differ.

    python tools/determinism_probe.py [--spec rtdetr-r50-moe8-top2 --batch 2 --h 736 --w 1280]
"""
from __future__ import annotations

import argparse
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
os.environ.setdefault("MIOPEN_USER_DB_PATH", str(ROOT / "multimodal-moe_amd" / "miopen_db"))

import torch  # noqa: E402


def _tensors(x):
    if torch.is_tensor(x):
        return [x]
    if isinstance(x, (list, tuple)):
        return [t for v in x for t in _tensors(v)]
    if isinstance(x, dict):
        return [t for v in x.values() for t in _tensors(v)]
    return []


class Recorder:
    def __init__(self, model):
        self.calls = []
        self.on = False
        self.handles = []
        for name, mod in model.named_modules():
            self.handles.append(mod.register_forward_hook(self._hook(name, type(mod).__name__)))

    def _hook(self, name, cls):
        def fn(mod, inp, out):
            if self.on:
                self.calls.append((name, cls, [t.detach().clone() for t in _tensors(inp)],
                                   [t.detach().clone() for t in _tensors(out)]))
        return fn

    def run(self, f):
        self.calls = []
        self.on = True
        try:
            out = f()
        finally:
            self.on = False
        return out, self.calls


def _same(a, b):
    return len(a) == len(b) and all(x.shape == y.shape and torch.equal(x, y) for x, y in zip(a, b))


def _maxdiff(a, b):
    d = 0.0
    for x, y in zip(a, b):
        if x.shape == y.shape and x.is_floating_point():
            d = max(d, float((x.float() - y.float()).abs().max()))
        elif not torch.equal(x, y):
            d = float("inf")
    return d


def compare(ref, got):
    first, culprits = None, {}
    for (n, c, ia, oa), (_, _, ib, ob) in zip(ref, got):
        if _same(oa, ob):
            continue
        rec = {"module": n, "class": c, "inputs_identical": _same(ia, ib), "out_maxdiff": _maxdiff(oa, ob)}
        if first is None:
            first = rec
        if rec["inputs_identical"]:
            culprits.setdefault(c, []).append(n)
    return first, {c: (len(v), v[:4]) for c, v in culprits.items()}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--spec", default="rtdetr-r18-moe4-top2")
    ap.add_argument("--batch", type=int, default=2)
    ap.add_argument("--h", type=int, default=256)
    ap.add_argument("--w", type=int, default=320)
    ap.add_argument("--repeats", type=int, default=3)
    ap.add_argument("--benchmark", action="store_true", help="torch.backends.cudnn.benchmark (bench.py's setting)")
    ap.add_argument("--deterministic", action="store_true",
                    help="torch.backends.cudnn.deterministic: MIOpen's deterministic convolution solvers only")
    a = ap.parse_args()
    from src.rtdetr_moe.data import SyntheticZOD
    from src.rtdetr_moe.model import RTDETRMoE
    from src.rtdetr_moe.step import FlatOutputs, gemm_params

    torch.backends.cudnn.benchmark = a.benchmark
    torch.backends.cudnn.deterministic = a.deterministic
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    model = RTDETRMoE(a.spec).to(dev).to(memory_format=torch.channels_last)
    for p in gemm_params(model):
        p.data = p.data.to(torch.bfloat16)
    images, _, ctx = SyntheticZOD(batch=a.batch, img_h=a.h, img_w=a.w, seed=6).sample(dev)
    x = images.contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
    flat = FlatOutputs(model)
    for _ in range(2):  # warm-up: convolution search, caches
        flat(x, ctx)
    torch.cuda.synchronize()
    rec = Recorder(model)
    runs = []
    for _ in range(a.repeats):
        with torch.no_grad():
            _, calls = rec.run(lambda: flat(x, ctx))
        torch.cuda.synchronize()
        runs.append(calls)
    for i in range(1, a.repeats):
        first, culprits = compare(runs[0], runs[i])
        print(json.dumps({"probe": "forward", "spec": a.spec, "deterministic": a.deterministic, "repeat": i, "n_calls": len(runs[0]),
                          "first_diff": first, "nondeterministic_modules": culprits}), flush=True)
    runs = None
    for h in rec.handles:
        h.remove()
    # backward: fixed output gradients, repeated forward + backward
    params = [p for p in model.parameters() if p.requires_grad]
    names = [n for n, p in model.named_parameters() if p.requires_grad]
    grads = []
    gen = torch.Generator(device=dev).manual_seed(1)
    gouts = None
    for _ in range(a.repeats):
        out = flat(x, ctx)
        if gouts is None:
            gouts = [torch.randn(o.shape, device=dev, generator=gen).to(o.dtype) if o.requires_grad else None
                     for o in out]
        pairs = [(o, g) for o, g in zip(out, gouts) if g is not None]
        gs = torch.autograd.grad([o for o, _ in pairs], params, [g for _, g in pairs], allow_unused=True)
        torch.cuda.synchronize()
        grads.append([None if g is None else g.detach().clone() for g in gs])
    for i in range(1, a.repeats):
        diff = []
        for n, g0, g1 in zip(names, grads[0], grads[i]):
            if g0 is None or g1 is None or torch.equal(g0, g1):
                continue
            rel = float((g0.float() - g1.float()).norm() / g0.float().norm().clamp(min=1e-30))
            diff.append((n, rel))
        print(json.dumps({"probe": "backward", "spec": a.spec, "deterministic": a.deterministic, "repeat": i, "n_params": len(names),
                          "n_differ": len(diff), "differ_in_backward_order": diff[::-1][:40],
                          "max_rel": max((r for _, r in diff), default=0.0)}), flush=True)


if __name__ == "__main__":
    main()
