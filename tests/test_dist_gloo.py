"""Multi-process data parallelism on CPU (gloo, world size 2): the DDP-averaged
gradients of the RT-DETR-MoE step equal the single-process gradients of the
same two images, and every rank holds identical gradients."""
from __future__ import annotations

import os
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]


def _batch():
    from src.rtdetr_moe.data import SyntheticZOD

    return SyntheticZOD(batch=2, img_h=128, img_w=128, seed=5).sample()


def _loss(model, images, targets, ctx, nb):
    from src.rtdetr_moe.criterion import SetCriterion

    out = model(images, ctx)
    return sum(SetCriterion()(out, targets, nb).values())


def _model():
    from src.rtdetr_moe.model import RTDETRMoE

    torch.manual_seed(0)
    m = RTDETRMoE("rtdetr-r18-moe4-top1-dec1")
    for mod in m.modules():  # eval-mode BN: per-rank batch statistics would differ from the full batch
        if isinstance(mod, torch.nn.BatchNorm2d):
            mod.eval()
    return m


def _worker(rank, world, port, out):
    for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT)):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from src.rtdetr_moe.engine import wrap_ddp

    model = _model()
    ddp = wrap_ddp(model, None)
    images, targets, ctx = _batch()
    nb = float(sum(len(t["boxes"]) for t in targets))
    sl = slice(rank, rank + 1)
    # each rank: its image; loss normalised by the global box count, times world (DDP averages)
    loss = _loss(ddp, images[sl], targets[sl], ctx[sl], max(nb, 1.0)) * world
    loss.backward()
    grads = {n: p.grad.detach().clone() for n, p in model.named_parameters() if p.grad is not None}
    torch.save(grads, out / f"g{rank}.pt")
    dist.destroy_process_group()


@pytest.mark.slow
def test_ddp_gloo_world2_matches_single_process(tmp_path):
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_worker, args=(2, port, tmp_path), nprocs=2, join=True)
    g0 = torch.load(tmp_path / "g0.pt", weights_only=True)
    g1 = torch.load(tmp_path / "g1.pt", weights_only=True)
    model = _model()
    images, targets, ctx = _batch()
    nb = float(sum(len(t["boxes"]) for t in targets))
    # per-image losses summed == the DP objective (per-sample matching is independent)
    for i in range(2):
        _loss(model, images[i:i + 1], targets[i:i + 1], ctx[i:i + 1], max(nb, 1.0)).backward()
    ref = {n: p.grad for n, p in model.named_parameters() if p.grad is not None}
    assert set(g0) == set(g1)
    for n in g0:
        assert torch.equal(g0[n], g1[n]), f"ranks disagree on {n}"
        torch.testing.assert_close(g0[n], ref[n], rtol=2e-4, atol=2e-5, msg=lambda m: f"{n}: {m}")


def test_sharded_optimizer_layout():
    """optim.ShardedDPAdamW.layout (host side of the ZeRO-1 data-parallel
    optimizer): every element of every tensor lands in exactly one piece,
    pieces never cross a rank slice, every piece and slice starts at a
    multiple of 8 elements (16-B bf16 / 32-B fp32 vectors), and the slices
    cover each parameter space with at most 8 W - 1 padding elements."""
    from src.rtdetr_moe.optim import ShardedDPAdamW

    rng = __import__("random").Random(3)
    for W in (1, 2, 3, 8):
        tensors = {i: (rng.randint(0, 1), rng.choice([1, 7, 8, 255, 256, 4096, 65537, 262144])) for i in range(40)}
        space_of, poff, S, pieces = ShardedDPAdamW.layout(tensors, W)
        assert all(s % 8 == 0 and s >= 8 for s in S)
        for sp in (0, 1):
            need = sum((n + 7) // 8 * 8 for (s, n) in tensors.values() if s == sp)
            assert need <= S[sp] * W < need + 8 * W + 8
        cover = {i: [] for i in tensors}
        for (i, i0, n, r, s) in pieces:
            a = poff[i] + i0
            assert s == space_of[i] and n > 0 and a % 8 == 0 and i0 % 8 == 0
            assert r * S[s] <= a and a + n <= (r + 1) * S[s] and 0 <= r < W
            cover[i].append((i0, n))
        for i, (s, n) in tensors.items():
            segs = sorted(cover[i])
            assert segs[0][0] == 0 and sum(m for _, m in segs) == n
            assert all(segs[k][0] + segs[k][1] == segs[k + 1][0] for k in range(len(segs) - 1))
