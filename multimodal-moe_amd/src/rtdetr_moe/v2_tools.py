"""RT-DETRv2 ``tools/train.py`` command line, served by this engine.

The reference's third-party adapter (src/models/vision/rtdetr_thirdparty.py)
writes a JSON override config (:54-119) and runs
``python tools/train.py -c CFG -d DEV [--seed S] [--use-amp] --output-dir D``
to train, or ``... -r WEIGHTS --test-only`` to evaluate (:202-218, :280-293),
in the RT-DETRv2 checkout (third_party/rtdetr/rtdetrv2_pytorch, an empty
submodule in the reference).  It reads back ``best.pth`` / ``last.pth`` from
the output dir (:232-238) and the COCO summary lines from stdout (:132-155).

This module is that program for the build's engine, run as
``python -m src.rtdetr_moe.v2_tools`` with the same flags:

* the config is the adapter's override file (JSON, or YAML read with
  safe_load); ``__include__`` entries that exist are merged underneath it.
  The architecture comes from a ``model`` key when one is present (a build
  spec such as ``rtdetr-r50-moe8-top2``), else from the include's name:
  ``r18`` -> ``rtdetr-r18-moe4-top1`` (config C1), anything else
  (RT-DETRv2's r34/r50/r101 configs) -> the R50 MoE spec of config C2;
* ``train_dataloader`` / ``val_dataloader`` ``dataset.img_folder`` +
  ``ann_file`` (COCO, scripts/export_coco_dataset.py) feed ``CocoDataset``;
  ``eval_spatial_size`` is the image size, ``total_batch_size`` the batch,
  ``epoches`` the epoch count, ``num_classes`` the class count;
* GPU runs use bf16 autocast whatever ``--use-amp`` says (the engine's GPU
  precision); CPU runs are fp32;
* the summary printed is the pycocotools layout for the metrics this engine
  computes (AP@[.50:.95], AP@.50, AP@.75, AR@100, all areas) -- the lines the
  adapter's regexes read.  Values come from the in-house evaluator
  (metrics.py: 101-point interpolated AP per IoU threshold, Ultralytics-style
  matching; AR@100 from the 100 best detections per image), not pycocotools,
  which is absent: parity with pycocotools is unpinned.
"""
from __future__ import annotations

import argparse
import json
import re
import shutil
import sys
from pathlib import Path

import numpy as np

C1_SPEC = "rtdetr-r18-moe4-top1"
C2_SPEC = "rtdetr-r50-moe8-top2"


def _read(path: Path) -> dict:
    text = path.read_text()
    try:
        return json.loads(text)
    except json.JSONDecodeError:
        import yaml

        return yaml.safe_load(text) or {}


def _merge(base: dict, over: dict) -> dict:
    out = dict(base)
    for k, v in over.items():
        out[k] = _merge(out[k], v) if isinstance(v, dict) and isinstance(out.get(k), dict) else v
    return out


def load_config(path: str | Path) -> dict:
    """The override config with its existing ``__include__`` files merged
    underneath (later keys win, as RT-DETRv2's YAMLConfig)."""
    cfg = _read(Path(path))
    merged: dict = {}
    for inc in cfg.get("__include__", []):
        p = Path(inc)
        if p.is_file():
            merged = _merge(merged, load_config(p))
    merged = _merge(merged, {k: v for k, v in cfg.items() if k != "__include__"})
    merged["__include__"] = list(cfg.get("__include__", []))
    return merged


def arch_from_config(cfg: dict) -> str:
    m = cfg.get("model")
    if isinstance(m, str) and m.lower().startswith("rtdetr-"):
        return m
    names = " ".join(Path(p).stem for p in cfg.get("__include__", []))
    return C1_SPEC if re.search(r"r18", names) else C2_SPEC


def _device(dev: str | None) -> str:
    d = (dev or "cpu").strip().lower()
    if d.startswith("cuda"):
        return d.split(":", 1)[1] if ":" in d else "0"
    return d


def _data(cfg: dict) -> dict:
    ds = {}
    for split, key in (("train", "train_dataloader"), ("val", "val_dataloader")):
        d = cfg.get(key, {}).get("dataset", {})
        if "img_folder" not in d or "ann_file" not in d:
            raise KeyError(f"config: {key}.dataset needs img_folder and ann_file")
        ds[split] = {"img_folder": str(d["img_folder"]), "ann_file": str(d["ann_file"])}
    return ds


def coco_summary(box, ap75: float, ar100: float) -> str:
    """pycocotools COCOeval.summarize() layout, the lines this engine computes."""
    row = " {:<18} {} @[ IoU={:<9} | area={:>6s} | maxDets={:>3d} ] = {:0.3f}"
    lines = [row.format("Average Precision", "(AP)", "0.50:0.95", "all", 100, box.map),
             row.format("Average Precision", "(AP)", "0.50", "all", 100, box.map50),
             row.format("Average Precision", "(AP)", "0.75", "all", 100, ap75),
             row.format("Average Recall", "(AR)", "0.50:0.95", "all", 100, ar100)]
    return "\n".join(lines)


def _evaluate(model, data, imgsz, batch, device, workers, seed):
    from . import engine

    evs: list = []
    box = engine._evaluate(model, data, "val", imgsz, batch, device, workers, seed, ev_out=evs)
    ev = evs[0]
    ap75 = 0.0
    if ev.tp and sum(len(t) for t in ev.target_cls):
        from .metrics import ap_per_class

        tp = np.concatenate(ev.tp, 0)
        if len(tp):
            r = ap_per_class(tp.astype(np.float64), np.concatenate(ev.conf), np.concatenate(ev.pred_cls),
                             np.concatenate(ev.target_cls))
            ap75 = float(r["ap"][:, 5].mean())
    ar100 = ev.average_recall(100)
    return box, ap75, max(ar100, 0.0)


def main(argv=None) -> int:
    p = argparse.ArgumentParser(description="RT-DETRv2 tools/train.py command line on the RT-DETR-MoE engine")
    p.add_argument("-c", "--config", required=True)
    p.add_argument("-r", "--resume", default=None, help="checkpoint to resume from / evaluate")
    p.add_argument("-t", "--tuning", default=None, help="checkpoint to fine-tune from")
    p.add_argument("-d", "--device", default="cpu")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--use-amp", action="store_true")
    p.add_argument("--output-dir", default=None)
    p.add_argument("--summary-dir", default=None)
    p.add_argument("--test-only", action="store_true")
    a = p.parse_args(argv)

    import torch

    from . import engine

    cfg = load_config(a.config)
    out_dir = Path(a.output_dir or cfg.get("output_dir", "output")).resolve()
    out_dir.mkdir(parents=True, exist_ok=True)
    data = _data(cfg)
    h, w = (int(v) for v in cfg.get("eval_spatial_size", [704, 1248]))
    batch = int(cfg.get("train_dataloader", {}).get("total_batch_size", 16))
    workers = int(cfg.get("train_dataloader", {}).get("num_workers", 0))
    ncls = int(cfg.get("num_classes", 1))
    device = _device(a.device)
    print(f"engine device: {'cpu' if device == 'cpu' else 'cuda:' + device}", flush=True)
    if a.test_only:
        if not a.resume:
            raise SystemExit("--test-only needs -r WEIGHTS")
        dev = torch.device("cpu") if device == "cpu" else torch.device("cuda", int(device.split(",")[0]))
        if dev.type == "cuda":
            from ..moe import _lib

            torch.cuda.set_device(dev)
            _lib.lib()
        model = engine.load_model(a.resume, dev)
        if dev.type == "cuda":
            model = model.to(memory_format=torch.channels_last)
        box, ap75, ar100 = _evaluate(model, data, (h, w), batch, dev, workers, a.seed)
        print("IoU metric: bbox")
        print(coco_summary(box, ap75, ar100), flush=True)
        (out_dir / "eval.json").write_text(json.dumps(
            {"map50_95": box.map, "map50": box.map50, "map75": ap75, "ar100": ar100, "precision": box.mp,
             "recall": box.mr}, indent=2))
        return 0
    model = a.tuning or a.resume or arch_from_config(cfg)
    res = engine.train(engine.TrainArgs(model=str(model), data=data, imgsz=(h, w),
                                        epochs=int(cfg.get("epoches", cfg.get("epochs", 1))), batch=batch,
                                        device=device, project=str(out_dir), name="engine", seed=a.seed,
                                        workers=workers, num_classes=ncls))
    for src, dst in ((res.best, out_dir / "best.pth"), (res.last, out_dir / "last.pth")):
        if Path(src).exists():
            shutil.copyfile(src, dst)
    rd = res.results_dict
    print(json.dumps({"epochs_run": res.epochs_run, **{k: float(v) for k, v in rd.items()}}), flush=True)
    return 0


if __name__ == "__main__":
    sys.exit(main())
