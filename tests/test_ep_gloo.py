"""Expert parallelism on CPU (gloo, world size 2, 4 experts -> 2 per rank):
the fixed-capacity EP layer (src/moe/ep.py: static all-to-all splits, counts
and row maps on the device) reproduces the single-process layer with all
experts -- outputs, input gradients, router gradients (after the DP mean) and
each rank's expert gradients (after the 1/W scaling) -- on skewed,
context-binned inputs, with bf16-path and fp8 (MXFP8-emulating,
src/moe/eager.py) experts.  With slots below the worst case
(ep_capacity_factor 1.0) the overflowing assignments are dropped exactly as a
capacity_factor 1.0 layer drops them, and counted in last_ep_overflow."""
from __future__ import annotations

import os
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
E, K, D, F, TPI = 4, 2, 32, 64, 12  # D, F multiples of the 32-element MX block


def _cfg(ep, dtype="bf16", epcf=2.0, cf=0.0):
    from src.moe.config import MoEConfig

    # ep_lossless_mb=0: slots at the factor at every size (these tiny layers
    # would otherwise fit the default lossless budget and never overflow)
    return MoEConfig(num_experts=E, top_k=K, hidden=F, ep_size=ep, capacity_factor=cf, expert_dtype=dtype,
                     ep_capacity_factor=epcf, ep_lossless_mb=0.0, expert_parallel=ep > 1)


def _inputs(rank):
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randn(3, TPI, D, generator=g)
    ctx = torch.full((3,), rank % 6, dtype=torch.int32)  # one context bin per rank (C4)
    dy = torch.randn(3, TPI, D, generator=g)
    return x, ctx, dy


def _worker(rank, world, port, out, dtype, epcf):
    for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT)):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.set_num_threads(1)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from src.moe.layer import MoEFFN

    torch.manual_seed(0)
    layer = MoEFFN(D, _cfg(world, dtype, epcf))
    x, ctx, dy = _inputs(rank)
    x.requires_grad_(True)
    y = layer(x, ctx)
    lb, z = layer.last_aux
    ((y * dy).sum() + 0.1 * lb + 0.05 * z).backward()
    res = {"y": y.detach(), "dx": x.grad, "hist": layer.last_hist, "overflow": layer.last_ep_overflow}
    for n in ("wg", "ctx_bias"):  # replicated: DP mean over ranks
        g = getattr(layer, n).grad.clone()
        dist.all_reduce(g)
        res["d" + n] = g / world
    for n in ("w1", "b1", "w2", "b2"):
        res["d" + n] = getattr(layer, n).grad.clone()
    torch.save(res, out / f"r{rank}.pt")
    dist.destroy_process_group()


@pytest.mark.slow
@pytest.mark.parametrize("dtype,epcf", [("bf16", 2.0), ("fp8", 2.0), ("bf16", 1.0)],
                         ids=["bf16", "fp8", "bf16_overflow"])
def test_ep_gloo_world2_matches_single_process(tmp_path, dtype, epcf):
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    W = 2
    mp.spawn(_worker, args=(W, port, tmp_path, dtype, epcf), nprocs=W, join=True)
    from src.moe.layer import MoEFFN

    torch.manual_seed(0)
    # slots >= T (epcf k >= E): nothing can drop; else the reference layer has
    # capacity factor epcf on each rank's tokens
    ref = MoEFFN(D, _cfg(1, dtype, cf=0.0 if epcf * K >= E else epcf))
    El = E // W
    overflows = []
    for r in range(W):
        got = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        x, ctx, dy = _inputs(r)
        x.requires_grad_(True)
        ref.zero_grad(set_to_none=True)
        y = ref(x, ctx)
        lb, z = ref.last_aux
        ((y * dy).sum() + 0.1 * lb + 0.05 * z).backward()
        torch.testing.assert_close(got["y"], y.detach(), rtol=1e-5, atol=1e-5)
        torch.testing.assert_close(got["dx"], x.grad, rtol=1e-5, atol=1e-5)
        assert torch.equal(got["hist"], ref.last_hist)
        S = ref.cfg.ep_slot_rows(x.shape[0] * x.shape[1])
        assert int(got["overflow"]) == int((ref.last_hist.long() - S).clamp(min=0).sum())
        overflows.append(int(got["overflow"]))
        if r == 0:
            ref_grads = {n: getattr(ref, n).grad.clone() for n in ("wg", "ctx_bias", "w1", "b1", "w2", "b2")}
        else:
            for n in ref_grads:
                ref_grads[n] += getattr(ref, n).grad
    assert (sum(overflows) > 0) == (epcf * K < E), overflows
    for r in range(W):
        got = torch.load(tmp_path / f"r{r}.pt", weights_only=True)
        for n in ("wg", "ctx_bias"):
            torch.testing.assert_close(got["d" + n], ref_grads[n] / W, rtol=1e-4, atol=1e-5)
        for n in ("w1", "b1", "w2", "b2"):
            torch.testing.assert_close(got["d" + n], ref_grads[n][r * El:(r + 1) * El] / W, rtol=1e-4, atol=1e-5)


def test_compaction_map_is_a_bijection_on_valid_rows():
    """ep.compaction_map: compact expert-major order over (expert, source, j),
    gather and inv mutually inverse on the received rows that hold data."""
    from src.moe.ep import compaction_map

    g = torch.Generator().manual_seed(0)
    for W, El, S in ((1, 4, 5), (2, 2, 7), (4, 3, 3), (8, 2, 1)):
        cnt = torch.randint(0, S + 1, (W, El), generator=g)
        cnt[0, 0] = 0  # an empty (source, expert) block
        gather, inv, offs = compaction_map(cnt, S)
        n = int(cnt.sum())
        assert offs.tolist() == [0] + torch.cumsum(cnt.sum(0), 0).tolist()
        expect = [(s * El + e) * S + j for e in range(El) for s in range(W) for j in range(int(cnt[s, e]))]
        assert gather[:n].tolist() == expect
        valid = torch.zeros(W * El * S, dtype=torch.bool)
        valid[torch.tensor(expect, dtype=torch.long)] = True
        assert torch.equal(gather[:n].long()[inv[valid]], torch.nonzero(valid).view(-1))
        assert torch.equal(inv[gather[:n].long()], torch.arange(n))


def test_ep_slot_rows():
    from src.moe.config import MoEConfig, parse_moe_spec

    # default, per layer: the C4 encoder (lossless buffer 16 x 7,360 x 512 B = 60 MB > 32 MB) at 2x the
    # mean rows, every C4 decoder layer (19.7 MB) lossless
    assert MoEConfig(num_experts=16, top_k=2).ep_slot_rows(7360) == 1840
    assert MoEConfig(num_experts=16, top_k=2).ep_slot_rows(2400) == 2400
    assert MoEConfig(num_experts=16, top_k=2, ep_capacity_factor=0.0).ep_slot_rows(7360) == 7360  # lossless
    assert parse_moe_spec("rtdetr-r50-moe16-top2-ep1-epcf0").moe.ep_slot_rows(7360) == 7360
    assert parse_moe_spec("rtdetr-r50-moe16-top2-ep1").moe.ep_slot_rows(2400) == 2400
    assert parse_moe_spec("rtdetr-r50-moe16-top2-ep1-epmb0").moe.ep_slot_rows(2400) == 600  # no lossless budget
    assert parse_moe_spec("rtdetr-r50-moe16-top2-ep1-epmb100").moe.ep_slot_rows(7360) == 7360
    assert MoEConfig(num_experts=16, top_k=2).ep_slot_rows(2400, d_model=512) == 600  # 39 MB > 32 MB
    c = MoEConfig(num_experts=16, top_k=2, ep_capacity_factor=2.0, ep_lossless_mb=0.0)
    assert c.ep_slot_rows(7360) == 1840        # 2 x mean 920
    c.ep_capacity_factor = 8.0                 # f k >= E: worst case, T
    assert c.ep_slot_rows(7360) == 7360
    c5 = MoEConfig(num_experts=32, top_k=4, capacity_factor=1.25)
    assert c5.ep_slot_rows(14720) == c5.capacity(14720) == 2300
    s = parse_moe_spec("rtdetr-r50-moe16-top2-ep1-epcf3")
    assert s.moe.expert_parallel and s.moe.ep_size == 1 and s.moe.ep_capacity_factor == 3.0
