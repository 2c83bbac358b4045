"""Training / validation engine behind src/models/vision/rtdetr.py.

Replaces what the reference delegates to Ultralytics (``RTDETR(cfg.model)
.train(...)`` / ``.val(...)``, src/models/vision/rtdetr.py:82-94, :112-127):
  * ``train(...)``    -> TrainResults  (.results_dict, .model, .save_dir, .best, .last)
  * ``validate(...)`` -> DetMetrics    (.results_dict, .box, .speed, .model)
Devices follow the reference's ``device`` string ("cpu", "0", "0,1,2,3"):
one process per GPU; a multi-GPU string launches that many local workers
(torch.multiprocessing) unless the caller is already under torchrun.  Every
training batch is one ``step.TrainStep`` -- the same step bench.py times: on
the GPU a whole-step hipGraph with bf16 weights + fp32 masters and the flat
RCCL gradient all-reduce; fp32 eager on CPU (config C1).
"""
from __future__ import annotations

import csv
import json
import math
import os
import random
import time
from dataclasses import asdict, dataclass, field
from datetime import timedelta
from pathlib import Path

import numpy as np
import torch
import torch.distributed as dist
from torch.nn.parallel import DistributedDataParallel as DDP

from ..moe.config import parse_moe_spec
from .criterion import SetCriterion
from .data import CocoDataset, SyntheticZOD, YoloDataset, collate
from .metrics import BoxMetrics, DetectionEvaluator
from .model import RTDETRMoE


# ---------------------------------------------------------------------------
# distributed helpers
# ---------------------------------------------------------------------------
def wrap_ddp(model: torch.nn.Module, local_rank: int | None, bucket_cap_mb: int = 64) -> DDP:
    """Data-parallel wrapper over RCCL.  Expert weights
    that are sharded over an expert-parallel group (C4) are excluded from the
    gradient all-reduce."""
    ignore = [n for n, p in model.named_parameters() if getattr(p, "expert_parallel", False)]
    if ignore:
        DDP._set_params_and_buffers_to_ignore_for_model(model, ignore)
    kw = dict(device_ids=[local_rank], output_device=local_rank) if local_rank is not None else {}
    return DDP(model, broadcast_buffers=False, gradient_as_bucket_view=True, bucket_cap_mb=bucket_cap_mb, **kw)


def parse_device(device: str | int | None) -> list:
    """"cpu" -> ["cpu"]; "0" -> [0]; "0,1" -> [0, 1]; "" / None -> [0] if a GPU else ["cpu"]."""
    s = "" if device is None else str(device).strip().lower()
    if s in ("", "auto"):
        return [0] if torch.cuda.is_available() else ["cpu"]
    if s == "cpu":
        return ["cpu"]
    s = s.replace("cuda:", "")
    return [int(v) for v in s.split(",") if v.strip() != ""]


def _dist_ctx():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


# ---------------------------------------------------------------------------
# model handle / results objects (the attributes the reference reads)
# ---------------------------------------------------------------------------
class ModelHandle:
    """``.model`` is the nn.Module (yolo.py:108-114 reads .model.parameters()
    and .model.flops/.GFLOPs)."""

    def __init__(self, module: RTDETRMoE):
        self.model = module

    def __repr__(self):
        return f"ModelHandle({self.model.spec.raw})"


@dataclass
class TrainResults:
    results_dict: dict
    model: ModelHandle | None
    save_dir: Path
    best: Path | None
    last: Path | None
    epochs_run: int = 0
    moe: dict = field(default_factory=dict)


@dataclass
class DetMetrics:
    results_dict: dict
    box: BoxMetrics
    speed: dict
    model: ModelHandle | None
    save_dir: Path | None = None
    moe: dict = field(default_factory=dict)


def _results_dict(box: BoxMetrics) -> dict:
    return {"metrics/precision(B)": box.mp, "metrics/recall(B)": box.mr, "metrics/mAP50(B)": box.map50,
            "metrics/mAP50-95(B)": box.map, "fitness": 0.1 * box.map50 + 0.9 * box.map}


# ---------------------------------------------------------------------------
# checkpoints: plain dicts of tensors / primitives (torch.load weights_only=True)
# ---------------------------------------------------------------------------
def _expert_shard_names(model: RTDETRMoE) -> dict:
    """{state-dict key: (MoEFFN, attribute)} of the expert weights that an
    expert-parallel model holds as [E/W, ...] shards."""
    from ..moe.layer import MoEFFN

    out = {}
    for name, mod in model.named_modules():
        if isinstance(mod, MoEFFN) and mod.ep_size > 1:
            for a in ("w1", "b1", "w2", "b2"):
                out[f"{name}.{a}" if name else a] = (mod, a)
    return out


def gather_expert_shards(model: RTDETRMoE, sd: dict) -> dict:
    """Collective over the expert-parallel group (every rank must call it):
    replace each [E/W, ...] expert shard in ``sd`` by the stacked [E, ...]
    tensor of all ranks (expert weights are saved stacked so EP
    shards re-assemble).  Identity for a model without EP layers."""
    names = _expert_shard_names(model)
    if not names:
        return sd
    out = dict(sd)
    for key, (mod, _) in names.items():
        t = sd[key].detach().contiguous()
        W = mod.ep_size
        parts = [torch.empty_like(t) for _ in range(W)]
        dist.all_gather(parts, t, group=mod.ep_group)
        out[key] = torch.cat(parts, 0)
    return out


def shard_expert_state(model: RTDETRMoE, sd: dict) -> dict:
    """Inverse of gather_expert_shards for loading: stacked [E, ...] expert
    tensors are cut to this rank's [r E/W, (r+1) E/W) slice when the model is
    expert-parallel."""
    names = _expert_shard_names(model)
    if not names:
        return sd
    out = dict(sd)
    for key, (mod, attr) in names.items():
        full = sd.get(key)
        local = getattr(mod, attr)
        if full is None or full.shape[0] == local.shape[0]:
            continue
        El = local.shape[0]
        r = dist.get_rank(mod.ep_group)
        out[key] = full[r * El:(r + 1) * El]
    return out


def resolve_spec(raw: str):
    """Parse a model spec for THIS process: an expert-parallel spec (-ep<W>)
    outside a process group of W ranks builds the same model with all experts
    local (e.g. single-process evaluation of an EP-trained checkpoint)."""
    spec = parse_moe_spec(raw)
    m = spec.moe
    if m is not None and m.ep_size > 1:
        world = dist.get_world_size() if (dist.is_available() and dist.is_initialized()) else 1
        if world != m.ep_size:
            m.ep_size = 1
            m.expert_parallel = False
    return spec


def save_checkpoint(path: Path, model: RTDETRMoE, epoch: int, fitness: float, optimizer=None, state_dict=None):
    path.parent.mkdir(parents=True, exist_ok=True)
    sd = model.state_dict() if state_dict is None else state_dict
    ck = {"spec": model.spec.raw, "num_classes": model.num_classes, "epoch": int(epoch),
          "fitness": float(fitness), "state_dict": {k: v.detach().float().cpu() if v.is_floating_point() else
                                                    v.detach().cpu() for k, v in sd.items()}}
    if model.spec.moe is not None:
        ck["moe_cfg"] = {k: v for k, v in asdict(model.spec.moe).items()}
    if optimizer is not None:
        ck["optimizer"] = optimizer.state_dict()
    torch.save(ck, path)


def load_model(weights: str | Path, device="cpu", num_classes: int = 1) -> RTDETRMoE:
    """A checkpoint written by save_checkpoint, or a bare architecture spec
    (``num_classes`` applies to the spec only; a checkpoint carries its own)."""
    p = Path(str(weights))
    if p.exists():
        ck = torch.load(p, map_location="cpu", weights_only=True)
        model = RTDETRMoE(resolve_spec(ck["spec"]), num_classes=int(ck.get("num_classes", 1)))
        model.load_state_dict(shard_expert_state(model, ck["state_dict"]))
        return model.to(device)
    if str(weights).endswith((".pt", ".pth")):
        raise FileNotFoundError(f"weights file not found: {weights}")
    return RTDETRMoE(resolve_spec(str(weights)), num_classes=num_classes).to(device)


# ---------------------------------------------------------------------------
# data
# ---------------------------------------------------------------------------
def _is_synthetic(data) -> bool:
    return str(data).startswith("synthetic")


def _synthetic_steps(data, default=4) -> int:
    s = str(data)
    return int(s.split(":", 1)[1]) if ":" in s else default


def _hw(imgsz):
    return (imgsz, imgsz) if isinstance(imgsz, int) else (int(imgsz[0]), int(imgsz[1]))


def _batches(data, split, imgsz, batch, workers, seed, rank, world, epoch, drop_last=False):
    h, w = _hw(imgsz)
    if _is_synthetic(data):
        gen = SyntheticZOD(batch=batch, img_h=h, img_w=w, seed=seed * 1000 + rank + (0 if split == "train" else 777)
                           + epoch * 7919)
        for _ in range(_synthetic_steps(data)):
            yield gen.sample()
        return
    if isinstance(data, dict):  # COCO export: {"train"/"val": {"img_folder", "ann_file"}}
        ds = CocoDataset(data[split]["img_folder"], data[split]["ann_file"], imgsz=(h, w))
    else:
        ds = YoloDataset(data, split=split, imgsz=(h, w))
    sampler = torch.utils.data.distributed.DistributedSampler(ds, world, rank, shuffle=split == "train",
                                                              seed=seed) if world > 1 else None
    if sampler is not None:
        sampler.set_epoch(epoch)
    g = torch.Generator().manual_seed(seed + epoch)
    dl = torch.utils.data.DataLoader(ds, batch_size=batch, shuffle=(split == "train" and sampler is None),
                                     sampler=sampler, num_workers=workers, collate_fn=collate,
                                     generator=g, drop_last=drop_last and len(ds) >= batch * world,
                                     persistent_workers=False)
    yield from dl


# ---------------------------------------------------------------------------
# training
# ---------------------------------------------------------------------------
@dataclass
class TrainArgs:
    model: str
    data: str
    imgsz: object = (704, 1248)
    epochs: int = 50
    patience: int = 100
    batch: int = 16
    device: str = "0"
    project: str = "outputs/runs/rtdetr"
    name: str = "baseline"
    seed: int = 0
    workers: int = 8
    lr: float = 1e-4
    lr_backbone: float = 1e-5
    weight_decay: float = 1e-4
    clip_norm: float = 0.1
    num_classes: int = 1


def _seed_all(seed: int):
    random.seed(seed)
    np.random.seed(seed % (2 ** 32))
    torch.manual_seed(seed)


def _master_state_dict(core: RTDETRMoE, step) -> dict:
    """The model's state dict with every bf16 GEMM/conv weight replaced by its
    fp32 master from the optimizer (TrainStep precision "bf16"), so a
    checkpoint carries the exact training state."""
    sd = core.state_dict()
    opt = getattr(step, "opt", None)
    if opt is None or not hasattr(opt, "master_of"):
        return sd
    names = {id(p): n for n, p in core.named_parameters()}
    for p in opt.params:
        if p.dtype == torch.bfloat16 and id(p) in names:
            sd[names[id(p)]] = opt.master_of(p).as_strided(p.shape, p.stride()).detach()
    return sd


def _train_worker(a: TrainArgs, rank: int, world: int, local: int | str) -> TrainResults | None:
    """One rank's training loop.  Each batch is one ``TrainStep`` -- the step
    bench.py measures: on the GPU bf16 GEMM/conv weights with fp32 masters, the
    whole differentiable step (forward, set criterion with the GPU Hungarian
    matcher, backward) replayed as ONE hipGraph, the flat gradient all-reduce
    over RCCL when world > 1, and the fused clip + AdamW (FlatAdamW); on the
    CPU (config C1) fp32 eager with torch.optim.AdamW + clip_grad_norm_ (DDP
    over gloo when world > 1).  The graph has static shapes, so on the GPU the
    train loader drops a last partial batch (every step sees ``batch`` images);
    the loss is accumulated on the device and read once per epoch."""
    from .step import TrainStep

    on_gpu = local != "cpu"
    device = torch.device("cuda", local) if on_gpu else torch.device("cpu")
    if on_gpu:
        torch.cuda.set_device(local)
        from ..moe import _lib

        _lib.lib()  # the GPU path has no fallback: fail now if libmoe_hip.so is missing
        # MIOpen picks convolution kernels by a (fast-mode) search per shape
        # instead of its immediate-mode heuristic: ~17% shorter C2 steps
        os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
        torch.backends.cudnn.benchmark = True
    _seed_all(a.seed)
    model = load_model(a.model, device, a.num_classes)
    if on_gpu:
        model = model.to(memory_format=torch.channels_last)
    core = model
    ep = bool(_expert_shard_names(core))
    crit = SetCriterion(num_classes=core.num_classes)
    save_dir = Path(a.project) / a.name
    wdir = save_dir / "weights"
    if rank == 0:
        wdir.mkdir(parents=True, exist_ok=True)
    best_fit, best_epoch = -1.0, -1
    last_metrics = BoxMetrics()
    csv_rows = []
    epoch = 0
    step = None
    shape = None
    for epoch in range(a.epochs):
        core.train()
        t_ep = time.perf_counter()
        tot = torch.zeros((), dtype=torch.float64, device=device)
        n = 0
        for images, targets, ctx in _batches(a.data, "train", a.imgsz, a.batch, a.workers, a.seed, rank, world,
                                             epoch, drop_last=on_gpu):
            images = images.to(device, non_blocking=True)
            if on_gpu:
                images = images.contiguous(memory_format=torch.channels_last)
            ctx = ctx.to(device)
            tg = [{"boxes": t["boxes"].to(device), "labels": t["labels"].to(device)} for t in targets]
            nb = torch.tensor([float(sum(len(t["boxes"]) for t in targets))], device=device)
            if world > 1:
                dist.all_reduce(nb)
            num_boxes = (nb / world).clamp_(min=1.0).reshape(())
            if step is None:
                step = TrainStep(core, crit, images, ctx, lr=a.lr, lr_backbone=a.lr_backbone,
                                 weight_decay=a.weight_decay, clip_norm=a.clip_norm, graphs=on_gpu, world=world,
                                 precision="bf16" if on_gpu else "fp32",
                                 ddp_local=None, targets=tg if on_gpu else None,
                                 num_boxes=float(num_boxes))
                shape = tuple(images.shape)
            if on_gpu and tuple(images.shape) != shape:
                raise RuntimeError(f"batch shape {tuple(images.shape)} differs from the captured {shape}")
            loss = step(images, ctx, tg, num_boxes if on_gpu else float(num_boxes))
            tot += loss.detach().double()
            n += 1
        # validation: rank 0 evaluates the unwrapped model; an expert-parallel
        # model's forward holds all-to-alls, so every rank runs the same
        # validation batches in lockstep (rank 0 keeps the metrics)
        metrics = None
        if rank == 0 or ep:
            metrics = _evaluate(core, a.data, "val", a.imgsz, a.batch, device, a.workers, a.seed)
        # checkpoint state: fp32 masters; expert shards gathered to [E, ...] (collective)
        # (a sharded data-parallel optimizer gathers masters collectively: every rank joins)
        collective = ep or getattr(getattr(step, "opt", None), "W", 1) > 1
        sd = gather_expert_shards(core, _master_state_dict(core, step)) if (rank == 0 or collective) else None
        if rank == 0:
            last_metrics = metrics
            fit = _results_dict(metrics)["fitness"]
            save_checkpoint(wdir / "last.pt", core, epoch, fit, state_dict=sd)
            if fit > best_fit:
                best_fit, best_epoch = fit, epoch
                save_checkpoint(wdir / "best.pt", core, epoch, fit, state_dict=sd)
            row = {"epoch": epoch + 1, "train/loss": float(tot) / max(n, 1), "time_s": time.perf_counter() - t_ep,
                   **_results_dict(metrics)}
            row.update(_moe_stats(core))
            csv_rows.append(row)
        stop = torch.tensor([0.0], device=device)
        if rank == 0 and epoch - best_epoch >= a.patience:
            stop[0] = 1.0
        if world > 1:
            dist.broadcast(stop, 0)
        if float(stop.item()) > 0:
            break
    if rank != 0:
        return None
    with open(save_dir / "results.csv", "w", newline="") as f:
        if csv_rows:
            wr = csv.DictWriter(f, fieldnames=list(csv_rows[0].keys()))
            wr.writeheader()
            wr.writerows(csv_rows)
    return TrainResults(results_dict=_results_dict(last_metrics), model=ModelHandle(core), save_dir=save_dir,
                        best=wdir / "best.pt", last=wdir / "last.pt", epochs_run=epoch + 1, moe=_moe_stats(core))


def _moe_stats(model: RTDETRMoE) -> dict:
    out = {}
    layers = model.moe_layers()
    for i, m in enumerate(layers):
        if m.last_hist is not None:
            h = m.last_hist.detach().float().cpu()
            out[f"moe/l{i}_load_cv"] = float(h.std() / h.mean().clamp(min=1e-9))
        if getattr(m, "last_ep_overflow", None) is not None:
            out[f"moe/l{i}_ep_overflow"] = int(m.last_ep_overflow)
        if m.last_aux is not None:
            out[f"moe/l{i}_lb"] = float(m.last_aux[0].detach())
            out[f"moe/l{i}_z"] = float(m.last_aux[1].detach())
    return out


def _mp_entry(local_idx, a, devices, port, out_file):
    os.environ.update({"MASTER_ADDR": "127.0.0.1", "MASTER_PORT": str(port), "RANK": str(local_idx),
                       "WORLD_SIZE": str(len(devices)), "LOCAL_RANK": str(local_idx)})
    dev = devices[local_idx]
    torch.cuda.set_device(dev)
    from .step import rccl_env

    rccl_env()
    # collective timeout: a dead rank fails the run instead of hanging it
    dist.init_process_group("nccl", device_id=torch.device("cuda", dev),
                            timeout=timedelta(seconds=float(os.environ.get("MOE_DIST_TIMEOUT_S", "1800"))))
    try:
        res = _train_worker(a, local_idx, len(devices), dev)
        if local_idx == 0 and res is not None:
            Path(out_file).write_text(json.dumps({"results_dict": res.results_dict, "epochs_run": res.epochs_run,
                                                  "moe": res.moe}))
    finally:
        from .step import release_graphs

        release_graphs()  # the rank's step / evaluation graphs, before the communicator goes
        dist.destroy_process_group()


def train(a: TrainArgs) -> TrainResults:
    devices = parse_device(a.device)
    if dist.is_available() and dist.is_initialized():  # already under torchrun
        rank, world = dist.get_rank(), dist.get_world_size()
        local = int(os.environ.get("LOCAL_RANK", rank)) if devices != ["cpu"] else "cpu"
        return _train_worker(a, rank, world, local)
    if devices == ["cpu"] or len(devices) == 1:
        return _train_worker(a, 0, 1, devices[0])
    import socket
    import tempfile

    import torch.multiprocessing as mp

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    out_file = Path(tempfile.mkdtemp()) / "rank0.json"
    mp.spawn(_mp_entry, args=(a, devices, port, str(out_file)), nprocs=len(devices), join=True)
    d = json.loads(out_file.read_text())
    save_dir = Path(a.project) / a.name
    model = load_model(save_dir / "weights" / "last.pt", "cpu")
    return TrainResults(results_dict=d["results_dict"], model=ModelHandle(model), save_dir=save_dir,
                        best=save_dir / "weights" / "best.pt", last=save_dir / "weights" / "last.pt",
                        epochs_run=d["epochs_run"], moe=d.get("moe", {}))


# ---------------------------------------------------------------------------
# validation
# ---------------------------------------------------------------------------
class EvalForward:
    """The inference forward of ``_evaluate`` (no_grad, bf16 autocast on the
    GPU).  On the GPU each input shape is captured once as a hipGraph and
    replayed (static input buffers refreshed by device copies; the outputs are
    the graph's static tensors, valid until the next call) -- the eval forward
    is ~400 kernel launches, which eager PyTorch issues slower than the GPU
    runs them.  MOE_EVAL_GRAPHS=0 keeps it eager; at most ``max_shapes``
    shapes are captured (later ones run eagerly)."""

    def __init__(self, model: RTDETRMoE, max_shapes: int = 2):
        self.model = model
        self.graphs = {}
        self.max_shapes = max_shapes
        self.enabled = os.environ.get("MOE_EVAL_GRAPHS", "1") != "0"

    def _run(self, images, ctx):
        with torch.autocast(images.device.type, dtype=torch.bfloat16, enabled=images.is_cuda, cache_enabled=False):
            return self.model(images, ctx)

    @staticmethod
    def _key(images, ctx):
        return (tuple(images.shape), images.dtype, tuple(images.stride()), tuple(ctx.shape), ctx.dtype)

    @torch.no_grad()
    def prepare(self, images, ctx):
        """Capture the graph for this input shape now (outside any timed span)."""
        if images.is_cuda and self.enabled and self._key(images, ctx) not in self.graphs \
                and len(self.graphs) < self.max_shapes:
            self(images, ctx)

    @torch.no_grad()
    def __call__(self, images, ctx):
        if not (images.is_cuda and self.enabled):
            return self._run(images, ctx)
        key = self._key(images, ctx)
        ent = self.graphs.get(key)
        if ent is None:
            if len(self.graphs) >= self.max_shapes:
                return self._run(images, ctx)
            si, sc = images.clone(), ctx.clone()
            side = torch.cuda.Stream()
            side.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(side):  # warm-up: convolution search, lazy library state, allocator
                for _ in range(2):
                    self._run(si, sc)
            torch.cuda.current_stream().wait_stream(side)
            torch.cuda.synchronize()
            from .step import CAPTURE_MODE, quiesce_collectives

            quiesce_collectives()  # training's eager collectives retired before the capture opens
            g = torch.cuda.CUDAGraph()

            with torch.cuda.graph(g, stream=side, capture_error_mode=CAPTURE_MODE):
                out = self._run(si, sc)
            torch.cuda.synchronize()
            ent = self.graphs[key] = (g, si, sc, out)
        g, si, sc, out = ent
        si.copy_(images)
        sc.copy_(ctx)
        g.replay()
        return out


@torch.no_grad()
def _evaluate(model: RTDETRMoE, data, split, imgsz, batch, device, workers, seed, speed: dict | None = None,
              ev_out: list | None = None):
    model.eval()
    on_gpu = device.type == "cuda"
    fwd = EvalForward(model)
    ev = DetectionEvaluator()
    if ev_out is not None:
        ev_out.append(ev)
    t_pre = t_inf = t_post = 0.0
    n_img = 0
    for images, targets, ctx in _batches(data, split, imgsz, batch, workers, seed, 0, 1, 0):
        t0 = time.perf_counter()
        images = images.to(device, non_blocking=True)
        ctx = ctx.to(device)
        t_cap = 0.0
        if on_gpu:
            images = images.contiguous(memory_format=torch.channels_last)
            tc = time.perf_counter()
            fwd.prepare(images, ctx)  # first batch of a shape: graph capture, untimed
            t_cap = time.perf_counter() - tc
            torch.cuda.synchronize()
        t1 = time.perf_counter()
        out = fwd(images, ctx)
        if on_gpu:
            torch.cuda.synchronize()
        t2 = time.perf_counter()
        H, W = images.shape[-2:]
        dets = model.postprocess(out, [(W, H)] * images.shape[0])
        for det, t in zip(dets, targets):
            gt = t["boxes"].numpy().astype(np.float64)
            gt_xyxy = np.stack([(gt[:, 0] - gt[:, 2] / 2) * W, (gt[:, 1] - gt[:, 3] / 2) * H,
                                (gt[:, 0] + gt[:, 2] / 2) * W, (gt[:, 1] + gt[:, 3] / 2) * H], 1) \
                if len(gt) else np.zeros((0, 4))
            ev.update(det["boxes"].float().cpu().numpy(), det["scores"].float().cpu().numpy(),
                      det["labels"].cpu().numpy(), gt_xyxy, t["labels"].numpy())
        t3 = time.perf_counter()
        t_pre += t1 - t0 - t_cap
        t_inf += t2 - t1
        t_post += t3 - t2
        n_img += images.shape[0]
    model.train()
    if speed is not None and n_img:
        speed.update({"preprocess": 1e3 * t_pre / n_img, "inference": 1e3 * t_inf / n_img,
                      "loss": 0.0, "postprocess": 1e3 * t_post / n_img})
    return ev.compute()


def validate(weights, data, split="val", imgsz=(704, 1248), batch=16, device="0", project=None, name=None,
             workers=4, seed=0) -> DetMetrics:
    devices = parse_device(device)
    dev = torch.device("cpu") if devices == ["cpu"] else torch.device("cuda", devices[0])
    if dev.type == "cuda":
        torch.cuda.set_device(dev)
        from ..moe import _lib

        _lib.lib()
    model = load_model(weights, dev)
    if dev.type == "cuda":
        model = model.to(memory_format=torch.channels_last)
    speed = {}
    box = _evaluate(model, data, split, imgsz, batch, dev, workers, seed, speed)
    save_dir = Path(project) / name if project and name else None
    if save_dir is not None:
        save_dir.mkdir(parents=True, exist_ok=True)
    return DetMetrics(results_dict=_results_dict(box), box=box, speed=speed, model=ModelHandle(model),
                      save_dir=save_dir, moe=_moe_stats(model))
