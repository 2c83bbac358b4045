"""The RCCL branches of the multi-GPU design on one
MI355X, over a world-1 ``nccl`` (= RCCL) process group.

Every multi-rank test elsewhere talks over gloo, which stages device tensors
through the host (src/moe/ep.py ``_a2a``, optim.py ``_collective``).  The
driver's ``bench.py --gpus 8`` takes the other branch: ``dist.all_to_all_single``
on device tensors captured INSIDE the step hipGraph (C4) and
``reduce_scatter_tensor`` / ``all_gather_into_tensor`` after the graph replay
(C3, ``optim.ShardedDPAdamW``).  A world-1 RCCL group executes exactly that
code -- communicator set-up, graph capture of the collective, stream ordering
against the replayed graph -- with a single rank, so the result must equal the
identity exchange / the single-process optimizer:

* C4: an ``-ep1`` model whose expert-parallel layers exchange over the RCCL
  group, trained for several replays of the whole-step graph, against the
  same model with the identity exchange (no process group): same losses and
  same weights (bitwise when the step is deterministic, else within the
  identity run's own replay spread).
* C3: ``ShardedDPAdamW`` (zero=True at world 1) over RCCL, against the same
  optimizer over a world-1 gloo group (host-staged collectives, identical
  arithmetic: bitwise) and against the replicated ``FlatAdamW``
  (tolerance: the clip norm's partial sums are ordered differently).
Anchor: /root/reference/src/models/vision/rtdetr.py:89 (multi-GPU through the
``device`` string)."""
from __future__ import annotations

import socket
from contextlib import contextmanager

import pytest
import torch
import torch.distributed as dist

DEV = "cuda"


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


@contextmanager
def _world1(backend):
    from src.rtdetr_moe.step import rccl_env, release_graphs

    kw = {"device_id": torch.device("cuda", 0)} if backend == "nccl" else {}
    release_graphs()  # earlier tests' unreachable graphs go before the communicator exists
    rccl_env()
    dist.init_process_group(backend, init_method=f"tcp://127.0.0.1:{_port()}", rank=0, world_size=1, **kw)
    try:
        yield dist.group.WORLD
    finally:
        release_graphs()  # graphs holding captured RCCL kernels must go before the communicator
        dist.destroy_process_group()


def _setup(spec, seed=6):
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.data import SyntheticZOD
    from src.rtdetr_moe.model import RTDETRMoE

    torch.manual_seed(0)
    model = RTDETRMoE(spec).to(DEV).to(memory_format=torch.channels_last)
    images, targets, ctx = SyntheticZOD(batch=2, img_h=256, img_w=320, seed=seed).sample(DEV)
    images = images.contiguous(memory_format=torch.channels_last)
    targets = [{k: v.to(DEV) for k, v in t.items()} for t in targets]
    nb = max(1.0, float(sum(len(t["boxes"]) for t in targets)))
    return model, SetCriterion(num_classes=1), images, targets, ctx, nb


def _weights(model):
    return torch.cat([p.detach().float().reshape(-1) for p in model.parameters()]).cpu()


def _rel(a, b):
    return float((a - b).norm()) / max(float(b.norm()), 1e-30)


# ---------------------------------------------------------------------------
# C4: the EP all-to-all over RCCL, captured in the whole-step hipGraph
# ---------------------------------------------------------------------------
EP_SPEC = "rtdetr-r18-moe8-top2-ep1"
STEPS = 4


def _ep_run(group, calls=None):
    from src.rtdetr_moe.step import TrainStep

    model, crit, images, targets, ctx, nb = _setup(EP_SPEC)
    layers = model.moe_layers()
    assert layers and all(m.cfg.expert_parallel and m.ep_size == 1 for m in layers)
    for m in layers:
        m.ep_group = group
    step = TrainStep(model, crit, images, ctx, graphs=True, world=1, precision="bf16", lr=1e-3,
                     targets=targets, num_boxes=nb)
    assert step.stepper is not None  # forward + criterion + backward as ONE graph
    losses = [float(step(images, ctx, targets, nb)) for _ in range(STEPS)]
    torch.cuda.synchronize()
    return losses, _weights(model)


@pytest.mark.gpu
def test_ep_all_to_all_rccl_captured_in_step_graph(hip_lib, monkeypatch):
    """dist.all_to_all_single over RCCL inside the captured step graph ==
    the identity exchange, over STEPS replays (forward dispatch / combine and
    their backward transposes in every MoE layer)."""
    seen = {"eager": 0, "captured": 0}
    real = dist.all_to_all_single

    def counting(out, inp, *a, **kw):
        seen["captured" if torch.cuda.is_current_stream_capturing() else "eager"] += 1
        return real(out, inp, *a, **kw)

    ref_losses, ref_w = _ep_run(None)  # identity exchange (no process group)
    monkeypatch.setattr(dist, "all_to_all_single", counting)
    with _world1("nccl") as g:
        assert dist.get_backend(g) == "nccl"
        losses, w = _ep_run(g)
    # warm-up (eager, creates the communicator) and capture both went through RCCL;
    # per layer: counts + dispatch + combine forward, two transposes backward
    assert seen["eager"] > 0 and seen["captured"] > 0, seen
    assert all(torch.isfinite(torch.tensor(losses))), losses
    assert min(losses[1:]) < losses[0], losses
    if losses == ref_losses and torch.equal(w, ref_w):
        return
    # not bitwise: bound by the identity path's own replay spread
    ref2_losses, ref2_w = _ep_run(None)
    spread_w = _rel(ref2_w, ref_w)
    spread_l = max(abs(a - b) / max(1.0, abs(a)) for a, b in zip(ref_losses, ref2_losses))
    assert _rel(w, ref_w) <= 3 * spread_w + 1e-6, (_rel(w, ref_w), spread_w)
    for a, b in zip(ref_losses, losses):
        assert abs(a - b) / max(1.0, abs(a)) <= 3 * spread_l + 1e-6, (ref_losses, losses, spread_l)


# ---------------------------------------------------------------------------
# C3: ShardedDPAdamW's RCCL reduce-scatter / all-gather after the graph replay
# ---------------------------------------------------------------------------
DP_SPEC = "rtdetr-r18-moe4-top2-dec2"


def _dp_run(zero, grads_check=False):
    from src.rtdetr_moe.step import TrainStep

    model, crit, images, targets, ctx, nb = _setup(DP_SPEC)
    step = TrainStep(model, crit, images, ctx, graphs=True, world=1, precision="bf16", lr=1e-3,
                     targets=targets, num_boxes=nb, zero=zero)
    assert step.stepper is not None
    assert (type(step.opt).__name__ == "ShardedDPAdamW") == zero
    losses = [float(step(images, ctx, targets, nb))]
    torch.cuda.synchronize()
    if grads_check:
        # world 1: the reduce-scattered slice IS the fp32 widening of the
        # graph's static gradients (one rank's sum), bitwise
        red = step.opt.reduced_grads()
        by_id = {id(p): g for p, g in zip(step.params, step.stepper.static_grads)}
        n = 0
        for i, v in red.items():
            g = by_id[id(step.opt.params[i])]
            if g is not None:
                assert torch.equal(v, g.float()), f"reduce-scattered gradient {i} differs"
                n += 1
        assert n > 10, n
    coef = step.opt.coef.cpu().clone()
    w1 = _weights(model)  # after one update
    losses += [float(step(images, ctx, targets, nb)) for _ in range(STEPS - 1)]
    torch.cuda.synchronize()
    return losses, _weights(model), coef, w1


@pytest.mark.gpu
def test_sharded_dp_adamw_rccl_world1(hip_lib, monkeypatch):
    calls = {"rs": 0, "ag": 0}
    rs, ag = dist.reduce_scatter_tensor, dist.all_gather_into_tensor

    def c_rs(*a, **kw):
        calls["rs"] += 1
        return rs(*a, **kw)

    def c_ag(*a, **kw):
        calls["ag"] += 1
        return ag(*a, **kw)

    monkeypatch.setattr(dist, "reduce_scatter_tensor", c_rs)
    monkeypatch.setattr(dist, "all_gather_into_tensor", c_ag)
    with _world1("nccl") as g:
        assert dist.get_backend(g) == "nccl"
        r_losses, r_w, r_coef, r_w1 = _dp_run(True, grads_check=True)
    assert calls["rs"] >= STEPS and calls["ag"] >= 2 * STEPS, calls  # RCCL branch taken every step
    with _world1("gloo"):
        g_losses, g_w, g_coef, _ = _dp_run(True)
    # same arithmetic, host-staged transport: bitwise
    assert r_losses == g_losses, (r_losses, g_losses)
    assert torch.equal(r_coef, g_coef)
    assert torch.equal(r_w, g_w)
    # the replicated optimizer (no process group): the clip norm's partial sums
    # are formed in another order, so the first update agrees to fp32 rounding
    # (a few bf16 weights one rounding apart).  Later losses are not compared:
    # on this random-init model the 300 selected queries are near-tied
    # (test_gpu_step.py::test_whole_step_graph_matches_eager), so any
    # difference in the weights grows along the trajectory.
    f_losses, f_w, f_coef, f_w1 = _dp_run(False)
    assert abs(float(r_coef[0]) - float(f_coef[0])) <= 1e-5 * float(f_coef[0]), (r_coef, f_coef)
    assert f_losses[0] == r_losses[0], (f_losses, r_losses)  # same initial weights, same graph
    assert _rel(r_w1, f_w1) <= 1e-4, _rel(r_w1, f_w1)
    assert all(torch.isfinite(torch.tensor(r_losses)))
