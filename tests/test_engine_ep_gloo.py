"""Expert parallelism through the boundary on CPU (gloo, world size 2):
``train_rtdetr_detector`` with an ``-ep2`` spec trains, validates in lockstep
on both ranks (the EP forward holds all-to-alls), writes checkpoints whose
expert weights are the stacked [E, ...] tensors of both ranks' shards
(SURVEY.md 5), and ``eval_rtdetr_detector`` evaluates the checkpoint in a
single process with all experts local.  The replicated weights stay
bit-identical across ranks although the gradient clip (clip_norm 0.1, active
at random init) sees a different expert shard on each rank: the clip norm sums
the shards' squared norms over the EP group (step.clip_grad_norm_sharded).
Anchors: /root/reference/src/models/vision/rtdetr.py:83-94 (train with a
``device`` string), rtdetr_thirdparty.py:235-236 (best/last checkpoints)."""
from __future__ import annotations

import os
import sys
from pathlib import Path

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

ROOT = Path(__file__).resolve().parents[1]
SPEC = "rtdetr-r18-moe4-top2-ep2-dec1"
EXPERT_KEYS = ("w1", "b1", "w2", "b2")


def _worker(rank, world, port, out):
    for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT)):
        sys.path.insert(0, p)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(2)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import src.rtdetr_moe.engine as E
    from src.models.vision.rtdetr import RtdetrTrainConfig, train_rtdetr_detector

    built = {}
    orig = E.load_model

    def spy(*a, **k):  # keep this rank's trained module
        built["m"] = orig(*a, **k)
        return built["m"]

    E.load_model = spy
    cfg = RtdetrTrainConfig(data_yaml="synthetic:2", model=SPEC, imgsz=128, epochs=2, batch=2, device="cpu",
                            project=str(out), name="ep2", workers=0)
    res = train_rtdetr_detector(cfg)
    assert (res is not None) == (rank == 0)
    m = built["m"]
    # parameters only: BatchNorm running statistics are per-rank batch statistics (no SyncBN)
    torch.save({k: v.detach().clone() for k, v in m.named_parameters()}, out / f"sd{rank}.pt")
    dist.destroy_process_group()


@pytest.mark.slow
def test_ep2_train_checkpoint_eval_through_boundary(tmp_path):
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    mp.spawn(_worker, args=(2, port, tmp_path), nprocs=2, join=True)
    sd0 = torch.load(tmp_path / "sd0.pt", weights_only=True)
    sd1 = torch.load(tmp_path / "sd1.pt", weights_only=True)
    expert = [k for k in sd0 if k.rsplit(".", 1)[-1] in EXPERT_KEYS and "ffn" in k]
    assert expert, "no expert weights found"
    for k in sd0:
        if k in expert:
            assert sd0[k].shape[0] == 2 and not torch.equal(sd0[k], sd1[k]), k  # E/W = 2 local experts
        else:
            assert torch.equal(sd0[k], sd1[k]), f"replicated weight {k} diverged across EP ranks"
    wdir = tmp_path / "ep2" / "weights"
    ck = torch.load(wdir / "last.pt", weights_only=True)
    assert ck["spec"] == SPEC
    for k in expert:  # stacked [E, ...]: rank 0's experts then rank 1's
        assert torch.equal(ck["state_dict"][k], torch.cat([sd0[k], sd1[k]], 0).float()), k
    for k in sd0:
        if k not in expert:
            assert torch.equal(ck["state_dict"][k], sd0[k].float()), k
    assert (wdir / "best.pt").exists()

    from src.models.vision.rtdetr import eval_rtdetr_detector
    from src.rtdetr_moe.engine import load_model

    m = load_model(wdir / "last.pt", "cpu")  # single process: all 4 experts local
    layers = m.moe_layers()
    assert layers and all(l.ep_size == 1 and l.w1.shape[0] == 4 for l in layers)
    met = eval_rtdetr_detector("synthetic:1", str(wdir / "last.pt"), imgsz=128, batch=2, device="cpu")
    assert "metrics/mAP50(B)" in met.results_dict
