"""Shared run-artifact writers (the output contract of the detector API).

The reference's RT-DETR adapter reuses these from its YOLO module
(src/models/vision/rtdetr.py:27-33; definitions src/models/vision/yolo.py:
185-376) so every model family writes the same files:
  metrics.json        {map50, map50_95, precision, recall, speed_*_ms_per_img,
                       params_total, params_trainable, flops_g, curves_results?}
  metrics_table.csv   two columns "metric,value", rows sorted by key
  run_metadata.{json,csv}, train_summary.{json,csv}
scripts/report_detector_benchmarks.py reads them back, so key names, key
order and fallbacks match the reference (pinned by tests/golden/
reference_known_answers.json).  The YOLO train/eval half of the reference's
module (yolo.py:19-182, 379-388) is a different model family and out of scope;
its names are exported with the reference's lazy-import behaviour (an
ImportError naming Ultralytics when called), so the reference's unchanged
callers -- scripts/eval_detector.py:28-35 imports eval_yolo_detector and
get_yolo_model_size_stats_from_weights at module load -- import this module.
"""
from __future__ import annotations

import csv
import json
from dataclasses import dataclass
from pathlib import Path
from typing import Union

import numpy as np


@dataclass
class YoloTrainConfig:
    """Field-for-field the reference's YoloTrainConfig (yolo.py:19-37)."""
    data_yaml: str
    model: str = "yolo26s.pt"
    imgsz: Union[int, tuple[int, int]] = (704, 1248)
    rect: bool = True
    epochs: int = 50
    patience: int = 100
    batch: int = 16
    device: str = "0"
    project: str = "outputs/runs/yolo"
    name: str = "baseline"
    seed: int = 0
    workers: int = 8
    scale: float = 0.0
    translate: float = 0.0
    mosaic: float = 0.0
    close_mosaic: int = 0


def _import_ultralytics_yolo():
    """The reference's lazy import (yolo.py:40-60): YOLO runs need Ultralytics,
    which this MI355X build does not ship (YOLO is out of its scope)."""
    try:
        from ultralytics import YOLO  # type: ignore
    except Exception as e:
        raise ImportError(
            "Ultralytics is required for YOLO adapter. Install with `pip install ultralytics`. "
            "(The MI355X build implements the RT-DETR-MoE backend only: use --backend rtdetr.)") from e
    return YOLO


def _format_ultralytics_imgsz(imgsz: Union[int, tuple[int, int]]):
    """(h, w) -> [h, w]; int -> int (reference yolo.py:175-182)."""
    if isinstance(imgsz, tuple):
        return [int(imgsz[0]), int(imgsz[1])]
    return int(imgsz)


def train_yolo_detector(cfg: YoloTrainConfig):
    """Reference yolo.py:63-95 (Ultralytics YOLO.train)."""
    YOLO = _import_ultralytics_yolo()
    model = YOLO(cfg.model)
    return model.train(data=cfg.data_yaml, imgsz=_format_ultralytics_imgsz(cfg.imgsz), rect=cfg.rect,
                       epochs=cfg.epochs, patience=cfg.patience, batch=cfg.batch, device=cfg.device,
                       project=cfg.project, name=cfg.name, seed=cfg.seed, workers=cfg.workers, scale=cfg.scale,
                       translate=cfg.translate, mosaic=cfg.mosaic, close_mosaic=cfg.close_mosaic)


def eval_yolo_detector(data_yaml: str, weights_path: str, split: str = "val",
                       imgsz: Union[int, tuple[int, int]] = (704, 1248), rect: bool = True, batch: int = 16,
                       device: str = "0", project: str | None = None, name: str | None = None):
    """Reference yolo.py:128-172 (Ultralytics YOLO.val)."""
    YOLO = _import_ultralytics_yolo()
    model = YOLO(weights_path)
    kw = {k: v for k, v in (("project", project), ("name", name)) if v}
    return model.val(data=data_yaml, split=split, imgsz=_format_ultralytics_imgsz(imgsz), rect=rect, batch=batch,
                     device=device, **kw)


def get_yolo_model_size_stats_from_weights(weights_path: str) -> dict:
    """Reference yolo.py:379-388: params/FLOPs of YOLO weights (needs Ultralytics)."""
    YOLO = _import_ultralytics_yolo()
    return _size_stats(YOLO(weights_path))

_RESULT_KEYS = (  # output key, Ultralytics results_dict key
    ("map50", "metrics/mAP50(B)"),
    ("map50_95", "metrics/mAP50-95(B)"),
    ("precision", "metrics/precision(B)"),
    ("recall", "metrics/recall(B)"),
)
_BOX_KEYS = (("map50", "map50"), ("map50_95", "map"), ("precision", "mp"), ("recall", "mr"))


def _size_stats(handle) -> dict:
    """params_total / params_trainable / flops_g of ``handle.model`` (best effort)."""
    stats = {"params_total": None, "params_trainable": None, "flops_g": None}
    net = getattr(handle, "model", None) if handle is not None else None
    if net is None:
        return stats
    try:
        params = list(net.parameters())
        stats["params_total"] = int(sum(p.numel() for p in params))
        stats["params_trainable"] = int(sum(p.numel() for p in params if p.requires_grad))
    except Exception:
        pass
    for attr in ("flops", "flops_g", "GFLOPs"):
        if hasattr(net, attr):
            try:
                stats["flops_g"] = float(getattr(net, attr))
                break
            except Exception:
                pass
    return stats


def _floats(values) -> list:
    """1-D float list from a curve payload; class-wise [C, N] arrays are
    averaged over classes (a single class is taken as is)."""
    try:
        arr = np.asarray(values, dtype=float)
        if arr.size == 0:
            return []
        if arr.ndim >= 2:
            arr = arr[0] if arr.shape[0] == 1 else arr.mean(axis=0)
        return [float(v) for v in np.asarray(arr, dtype=float).reshape(-1)]
    except Exception:
        try:
            return [float(v) for v in list(values)]
        except Exception:
            return []


def _curves(box) -> list | None:
    results = getattr(box, "curves_results", None)
    if not isinstance(results, (list, tuple)):
        return None
    names = getattr(box, "curves", None)
    names = [str(n) for n in names] if isinstance(names, (list, tuple)) else []
    curves = []
    for i, item in enumerate(results):
        try:
            if not (isinstance(item, (list, tuple)) and len(item) >= 2):
                continue
            x, y = _floats(item[0]), _floats(item[1])
            n = min(len(x), len(y))
            if n == 0:
                continue
            entry = {"x": x[:n], "y": y[:n]}
            if i < len(names):
                entry["name"] = names[i]
            curves.append(entry)
        except Exception:
            continue
    return curves


def save_yolo_metrics_json(metrics, out_path: str | Path) -> Path:
    """Write the shared metrics.json from a metrics object (.results_dict,
    else .box; .speed; .model; .box.curves_results)."""
    out_path = Path(out_path)
    out_path.parent.mkdir(parents=True, exist_ok=True)
    doc = {}
    rd = getattr(metrics, "results_dict", None)
    if rd is not None:
        rd = dict(rd)
        doc.update({k: float(rd[src]) for k, src in _RESULT_KEYS if src in rd})
    box = getattr(metrics, "box", None)
    if not doc and box is not None:
        doc.update({k: float(getattr(box, a)) for k, a in _BOX_KEYS if hasattr(box, a)})
    speed = getattr(metrics, "speed", None)
    if isinstance(speed, dict):
        for k, v in speed.items():
            try:
                doc[f"speed_{k}_ms_per_img"] = float(v)
            except Exception:
                pass
    doc.update(_size_stats(getattr(metrics, "model", None)))
    try:
        if box is not None:
            curves = _curves(box)
            if curves is not None:
                doc["curves_results"] = curves
    except Exception:
        pass
    out_path.write_text(json.dumps(doc, indent=2))
    return out_path


def save_metrics_table_csv(metrics_dict: dict, out_path: str | Path) -> Path:
    out_path = Path(out_path)
    out_path.parent.mkdir(parents=True, exist_ok=True)
    with out_path.open("w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["metric", "value"])
        w.writerows([k, metrics_dict[k]] for k in sorted(metrics_dict))
    return out_path


def infer_model_variant_from_weights(weights_name: str) -> str:
    """'yolo26n.pt' -> 'yolo26n'; 'rtdetr-r50-moe8-top2' -> itself."""
    return Path(weights_name).stem


def save_run_metadata_artifacts(metadata: dict, out_json_path: str | Path,
                                out_csv_path: str | Path) -> tuple[Path, Path]:
    out_json_path = Path(out_json_path)
    out_json_path.parent.mkdir(parents=True, exist_ok=True)
    out_json_path.write_text(json.dumps(metadata, indent=2))
    return out_json_path, save_metrics_table_csv(metadata, out_csv_path)


def save_yolo_training_summary(*, train_wall_time_s: float, model_name: str, data_yaml: str, run_name: str,
                               out_json_path: str | Path, out_csv_path: str | Path,
                               results=None) -> tuple[Path, Path]:
    summary = {"model_name": model_name, "data_yaml": data_yaml, "run_name": run_name,
               "train_wall_time_s": float(train_wall_time_s)}
    summary.update(_size_stats(getattr(results, "model", None)))
    out_json_path = Path(out_json_path)
    out_json_path.parent.mkdir(parents=True, exist_ok=True)
    out_json_path.write_text(json.dumps(summary, indent=2))
    return out_json_path, save_metrics_table_csv(summary, out_csv_path)
