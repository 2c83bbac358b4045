"""Multi-rank paths on the GPU, rehearsed as two processes
sharing one MI355X: RCCL wants one device per rank, so these ranks talk over
gloo (the flat gradient all-reduce and the norm partials on device tensors;
the expert-parallel all-to-all staged through the host, src/moe/ep.py).

* C3 data parallelism, bench.py's default execution (the whole step as ONE
  hipGraph; ZeRO-1 by default -- optim.ShardedDPAdamW: one fp32
  reduce-scatter, AdamW on the rank's 1/W slice, one bf16 all-gather -- and
  the flat fp32 all-reduce + FlatAdamW with inv_world as the MOE_ZERO=0
  A/B path; both are tested): after one step
  the reduced gradient equals the mean of single-process graph-mode gradients
  of the two ranks' images, the clip norm is the norm of that mean, and both
  ranks hold identical weights.  The comparison is with the per-rank mean, not
  with one pass over the union of the images: the trainable encoder
  BatchNorm and the MoE load-balance loss are per-rank batch statistics under
  data parallelism (no SyncBN), exactly as in DDP.
* C4 expert parallelism: the HIP EP layer at world 2 (16 experts, 8 per rank)
  reproduces the single-GPU 16-expert layer on each rank's tokens -- with
  lossless slots, and with slots below the skewed load (the capacity-factor
  layer's drops, the overflow count) --, and an
  ``-ep2`` model trained for two steps keeps its replicated weights
  bit-identical across ranks (the clip norm sums the expert shards over the
  EP group).
Anchor: /root/reference/src/models/vision/rtdetr.py:83-94 (multi-GPU via the
``device`` string)."""
from __future__ import annotations

import os
import socket
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
NB = 2.0  # num_boxes normaliser shared by both ranks (the engine all-reduces it)


def _port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _init(rank, world, port):
    for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT)):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("gloo", rank=rank, world_size=world)


def _data(rank, dev):
    from src.rtdetr_moe.data import SyntheticZOD

    images, targets, ctx = SyntheticZOD(batch=1, img_h=256, img_w=256, seed=11 + rank).sample(dev)
    images = images.contiguous(memory_format=torch.channels_last)
    return images, [{k: v.to(dev) for k, v in t.items()} for t in targets], ctx


def _model(spec, dev):
    from src.rtdetr_moe.model import RTDETRMoE

    torch.manual_seed(0)
    return RTDETRMoE(spec).to(dev).to(memory_format=torch.channels_last)


# ---------------------------------------------------------------------------
# C3: whole-step graph data parallelism == mean of single-process gradients
# ---------------------------------------------------------------------------
DP_SPEC = "rtdetr-r18-moe4-top2-dec2"


def _dp_worker(rank, world, port, out, precision, zero):
    os.environ["MOE_ZERO"] = "1" if zero else "0"  # read when step.py is imported (below)
    _init(rank, world, port)
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.step import TrainStep

    dev = torch.device("cuda", 0)
    model = _model(DP_SPEC, dev)
    images, targets, ctx = _data(rank, dev)
    step = TrainStep(model, SetCriterion(num_classes=1), images, ctx, graphs=True, world=world, lr=1e-3,
                     precision=precision, targets=targets, num_boxes=NB)
    assert step.stepper is not None
    assert (step.reducer is None) == zero and (type(step.opt).__name__ == "ShardedDPAdamW") == zero
    step(images, ctx, targets, NB)
    torch.cuda.synchronize()
    names = {id(p): n for n, p in model.named_parameters()}
    if zero:  # the reduce-scattered slices, gathered (test helper)
        red = step.opt.reduced_grads()
        mean = {names[id(step.opt.params[i])]: (v.float() / world).cpu() for i, v in red.items()}
    else:
        mean = {names[id(p)]: (v.float() / world).cpu() for p, v in zip(step.dp_params, step.reducer.views)}
    coef = step.opt.coef.cpu().clone()  # [norm of the mean gradient, applied scale] of step 1
    losses = [float(step(images, ctx, targets, NB))]
    torch.cuda.synchronize()
    w = torch.cat([p.detach().float().reshape(-1) for p in model.parameters()]).cpu()
    torch.save({"g": mean, "coef": coef, "w": w, "losses": losses}, out / f"r{rank}.pt")
    dist.destroy_process_group()


@pytest.mark.gpu
@pytest.mark.parametrize("precision,zero", [("bf16", True), ("amp", True), ("bf16", False)])
def test_whole_step_graph_dp_equals_single_process_mean(hip_lib, tmp_path, precision, zero):
    """zero: the sharded optimizer (reduce-scatter, AdamW on 1/world of the
    state, all-gather; optim.ShardedDPAdamW, the default); else the flat
    all-reduce + replicated FlatAdamW (MOE_ZERO=0)."""
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.step import TrainStep

    mp.start_processes(_dp_worker, args=(2, _port(), tmp_path, precision, zero), nprocs=2, join=True,
                       start_method="spawn")
    r0, r1 = torch.load(tmp_path / "r0.pt"), torch.load(tmp_path / "r1.pt")
    assert torch.equal(r0["w"], r1["w"]), "ranks diverged after the graph-mode all-reduce"
    assert torch.equal(r0["coef"], r1["coef"])
    assert all(torch.isfinite(torch.tensor(r0["losses"] + r1["losses"])))

    # single process, same graph-mode step at world 1, one replay per rank's image
    dev = torch.device("cuda", 0)
    model = _model(DP_SPEC, dev)
    images, targets, ctx = _data(0, dev)
    step = TrainStep(model, SetCriterion(num_classes=1), images, ctx, graphs=True, world=1, lr=1e-3,
                     precision=precision, targets=targets, num_boxes=NB)
    names = [n for n, p in model.named_parameters() if p.requires_grad]  # TrainStep.params order
    means = []
    for _ in range(2):  # two independent replays of both images: the backward's own run-to-run spread
        per_rank = []
        for r in range(2):
            images, targets, ctx = _data(r, dev)
            step.stepper(step._cast_in(images), ctx, targets, NB)
            torch.cuda.synchronize()
            per_rank.append([g.float().clone() for g in step.stepper.static_grads])
        assert len(names) == len(per_rank[0])
        means.append({n: ((a + b) / 2).cpu() for n, a, b in zip(names, *per_rank)})
    ref, ref2 = means

    def rel_err(got):
        d2 = sum(float((got[n] - ref[n]).norm()) ** 2 for n in got)
        return d2 ** 0.5 / sum(float(ref[n].norm()) ** 2 for n in got) ** 0.5

    # Since round 4 the whole backward has fixed-order sums (the deformable-
    # attention value gradient included: rtdetr_msda_fused_bwd_det), so two
    # single-process replays of the same images are bitwise equal, and with two
    # ranks the reduced sum a + b is one fp32 addition either way round: the
    # data-parallel mean must then EQUAL the single-process mean.  If a replay
    # spread shows up (MOE_DET_MSDA=0: bf16 atomics in arrival order), the mean
    # must sit within 3x that spread (+1e-3).
    floor = rel_err({n: ref2[n] for n in r0["g"]})
    tot = rel_err(r0["g"])
    if floor == 0.0 and os.environ.get("MOE_DET_MSDA", "1") != "0":
        diff = [n for n in r0["g"] if not torch.equal(r0["g"][n], ref[n])]
        assert not diff, f"DP mean differs from the single-process mean in {len(diff)} tensors, e.g. {diff[:4]} ({tot:.3e})"
    assert tot <= 3.0 * floor + 1e-3, f"DP vs single-process mean {tot:.3e}, replay spread {floor:.3e}"
    norm_ref = sum(float(ref[n].norm()) ** 2 for n in r0["g"]) ** 0.5
    assert abs(float(r0["coef"][0]) - norm_ref) <= (3.0 * floor + 1e-3) * norm_ref, (float(r0["coef"][0]), norm_ref)


# ---------------------------------------------------------------------------
# C4: the HIP expert-parallel layer over two ranks
# ---------------------------------------------------------------------------
E_EP, K_EP, TPI = 16, 2, 150


def _ep_inputs(rank, dev):
    g = torch.Generator().manual_seed(200 + rank)
    x = torch.randn(4, TPI, 256, generator=g).to(dev).to(torch.bfloat16)
    ctx = torch.full((4,), rank, dtype=torch.int32, device=dev)  # one context bin per rank (C4)
    dy = torch.randn(4, TPI, 256, generator=g).to(dev)
    return x, ctx, dy


def _ep_loss(layer, y, dy, ep):
    return (y.float() * dy).sum() + 10.0 * layer.aux_loss()


def _ep_layer_worker(rank, world, port, out, epcf=0.0):
    _init(rank, world, port)
    from src.moe.config import MoEConfig
    from src.moe.layer import MoEFFN

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    # epcf 0: lossless slots; epcf 1: S = T k / E rows per (source, expert),
    # below the skewed load, with no lossless budget: the receive path drops
    layer = MoEFFN(256, MoEConfig(num_experts=E_EP, top_k=K_EP, ep_size=world, expert_parallel=True,
                                   ep_capacity_factor=epcf, ep_lossless_mb=0.0)).to(dev)
    x, ctx, dy = _ep_inputs(rank, dev)
    x.requires_grad_(True)
    y = layer(x, ctx)
    _ep_loss(layer, y, dy, True).backward()
    torch.cuda.synchronize()
    res = {"y": y.detach().float().cpu(), "dx": x.grad.float().cpu(), "hist": layer.last_hist.cpu(),
           "overflow": int(layer.last_ep_overflow)}
    for n in ("wg", "ctx_bias"):  # replicated: DP mean
        g = getattr(layer, n).grad.clone()
        dist.all_reduce(g)
        res["d" + n] = (g / world).cpu()
    for n in ("w1", "b1", "w2", "b2"):  # local shard, already scaled by 1/W (ep_grad_scale)
        res["d" + n] = getattr(layer, n).grad.float().cpu()
    torch.save(res, out / f"ep{rank}.pt")
    dist.destroy_process_group()


def _close(a, b, what):
    torch.testing.assert_close(a, b, rtol=2e-2, atol=2e-2, msg=lambda m: f"{what}: {m}")
    assert (a - b).norm() <= 1e-2 * b.norm(), f"{what}: relative Frobenius {(a - b).norm() / b.norm():.3e}"


@pytest.mark.gpu
@pytest.mark.parametrize("epcf", [0.0, 1.0], ids=["lossless", "overflow"])
def test_hip_ep_layer_two_ranks_matches_single_gpu(hip_lib, tmp_path, epcf):
    """The HIP expert-parallel layer over 2 ranks (moe_ep_compaction, the
    scattering FFN, the paired backward writing the received layout) against
    the single-GPU 16-expert layer on each rank's tokens: lossless slots, and
    slots of T k / E rows per (source, expert) -- the lossy layout the C4
    encoder runs -- where the reference layer has capacity factor 1.0 on the
    rank's own tokens (the same slot-major drops) and the reported overflow is
    sum_e max(hist_e - S, 0)."""
    from src.moe.config import MoEConfig
    from src.moe.layer import MoEFFN

    W = 2
    mp.start_processes(_ep_layer_worker, args=(W, _port(), tmp_path, epcf), nprocs=W, join=True,
                       start_method="spawn")
    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    # all 16 experts, fused single-GPU path; capacity factor epcf emulates the slots
    ref = MoEFFN(256, MoEConfig(num_experts=E_EP, top_k=K_EP, capacity_factor=epcf)).to(dev)
    sums = None
    El = E_EP // W
    overflow = 0
    for r in range(W):
        got = torch.load(tmp_path / f"ep{r}.pt")
        x, ctx, dy = _ep_inputs(r, dev)
        x.requires_grad_(True)
        ref.zero_grad(set_to_none=True)
        y = ref(x, ctx)
        _ep_loss(ref, y, dy, False).backward()
        torch.cuda.synchronize()
        assert torch.equal(got["hist"], ref.last_hist.cpu())
        T = x.shape[0] * x.shape[1]
        S = ref.cfg.capacity(T) if epcf > 0 else T
        assert got["overflow"] == int((ref.last_hist.long().cpu() - S).clamp(min=0).sum())
        overflow += got["overflow"]
        _close(got["y"], y.detach().float().cpu(), f"rank {r} y")
        _close(got["dx"], x.grad.float().cpu(), f"rank {r} dx")
        g = {n: getattr(ref, n).grad.float().cpu().clone() for n in ("wg", "ctx_bias", "w1", "b1", "w2", "b2")}
        sums = g if sums is None else {n: sums[n] + g[n] for n in g}
    assert (overflow > 0) == (epcf > 0), overflow  # the skewed single-context batches overflow T k / E slots
    for r in range(W):
        got = torch.load(tmp_path / f"ep{r}.pt")
        for n in ("wg", "ctx_bias"):
            _close(got["d" + n], sums[n] / W, f"rank {r} d{n}")
        for n in ("w1", "b1", "w2", "b2"):
            _close(got["d" + n], sums[n][r * El:(r + 1) * El] / W, f"rank {r} d{n}")


EP_SPEC = "rtdetr-r18-moe4-top2-ep2-dec1"


def _ep_model_worker(rank, world, port, out):
    _init(rank, world, port)
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.step import TrainStep

    dev = torch.device("cuda", 0)
    model = _model(EP_SPEC, dev)
    images, targets, ctx = _data(rank, dev)
    step = TrainStep(model, SetCriterion(num_classes=1), images, ctx, graphs=False, world=world, lr=1e-3,
                     targets=targets, num_boxes=NB)
    losses = [float(step(images, ctx, targets, NB)) for _ in range(2)]
    torch.cuda.synchronize()
    sd = {n: p.detach().float().cpu().clone() for n, p in model.named_parameters()}
    torch.save({"sd": sd, "losses": losses, "norm": float(step.opt.coef[0])}, out / f"m{rank}.pt")
    dist.destroy_process_group()


@pytest.mark.gpu
def test_ep2_model_replicated_weights_stay_identical(hip_lib, tmp_path):
    mp.start_processes(_ep_model_worker, args=(2, _port(), tmp_path), nprocs=2, join=True, start_method="spawn")
    m0, m1 = torch.load(tmp_path / "m0.pt"), torch.load(tmp_path / "m1.pt")
    assert all(torch.isfinite(torch.tensor(m0["losses"] + m1["losses"])))
    assert m0["norm"] == m1["norm"]  # one global clip norm
    n_exp = 0
    for n, v in m0["sd"].items():
        if n.rsplit(".", 1)[-1] in ("w1", "b1", "w2", "b2") and ".ffn." in n:
            n_exp += 1
            assert not torch.equal(v, m1["sd"][n]), n  # different expert shards
        else:
            assert torch.equal(v, m1["sd"][n]), f"replicated weight {n} diverged across EP ranks"
    assert n_exp == 8
