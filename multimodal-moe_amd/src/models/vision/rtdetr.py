"""RT-DETR operator API -- drop-in for the reference's adapter module.

Same public names, signatures and artifact behaviour as the reference's
src/models/vision/rtdetr.py (RtdetrTrainConfig :36-48, train_rtdetr_detector
:77-95, eval_rtdetr_detector :98-128, save_rtdetr_metrics_json :131-138,
save_rtdetr_training_summary :141-162, get_rtdetr_model_size_stats_from_weights
:165-192, re-exports :27-33), so scripts/train_rtdetr.py and
scripts/eval_detector.py run unchanged against it.  What changes is the
engine: instead of Ultralytics ``RTDETR`` (absent and unpinned) the calls go
to this package's RT-DETR-MoE engine (src/rtdetr_moe), whose transformer FFNs
are the context-aware MoE running on MI355X HIP kernels (libmoe_hip.so).

``cfg.model`` is a local architecture spec ("rtdetr-r50-moe8-top2", see
src/moe/config.py) or a checkpoint written by this engine; a hub weight name
such as the reference default "rtdetr-l.pt" needs a network fetch and raises.
``data_yaml`` is an Ultralytics dataset.yaml (what the reference exports) or
"synthetic[:N]" for ZOD-shaped synthetic batches.
"""
from __future__ import annotations

from dataclasses import dataclass
from pathlib import Path
from typing import Union

from src.models.vision.yolo import (  # shared artifact schema (reference rtdetr.py:27-33)
    infer_model_variant_from_weights,
    save_metrics_table_csv,
    save_run_metadata_artifacts,
    save_yolo_metrics_json,
    save_yolo_training_summary,
)

__all__ = [
    "RtdetrTrainConfig", "train_rtdetr_detector", "eval_rtdetr_detector", "save_rtdetr_metrics_json",
    "save_rtdetr_training_summary", "get_rtdetr_model_size_stats_from_weights",
    "infer_model_variant_from_weights", "save_metrics_table_csv", "save_run_metadata_artifacts",
]

DEFAULT_MODEL = "rtdetr-r50-moe8-top2"
_HUB_NAMES = {"rtdetr-l.pt", "rtdetr-x.pt", "rtdetr-resnet50.pt", "rtdetr-resnet101.pt"}


@dataclass
class RtdetrTrainConfig:
    data_yaml: str
    model: str = DEFAULT_MODEL
    imgsz: Union[int, tuple[int, int]] = (704, 1248)
    epochs: int = 50
    patience: int = 100
    batch: int = 16
    device: str = "0"
    project: str = "outputs/runs/rtdetr"
    name: str = "baseline"
    seed: int = 0
    workers: int = 8


def _engine():
    """Import the engine lazily (as the reference imports Ultralytics lazily),
    with an actionable error when it cannot be loaded."""
    try:
        from src.rtdetr_moe import engine  # noqa: WPS433
    except Exception as e:  # pragma: no cover - import-time failure only
        raise ImportError(f"the RT-DETR-MoE engine failed to import: {e}") from e
    return engine


def _check_model_name(model: str) -> str:
    if Path(model).name in _HUB_NAMES and not Path(model).exists():
        raise ValueError(
            f"{model!r} is an Ultralytics hub weight name (needs a network fetch). Use a local "
            f"architecture spec such as {DEFAULT_MODEL!r} or a checkpoint written by this engine.")
    return model


def _imgsz(imgsz: Union[int, tuple[int, int]]):
    if isinstance(imgsz, (tuple, list)):
        return int(imgsz[0]), int(imgsz[1])
    return int(imgsz)


def train_rtdetr_detector(cfg: RtdetrTrainConfig):
    """Train RT-DETR-MoE; blocks until done and returns a results object with
    ``.results_dict``, ``.model`` (``.model.parameters()``), ``.save_dir``,
    ``.best`` and ``.last`` (checkpoints under ``project/name/weights``)."""
    eng = _engine()
    args = eng.TrainArgs(model=_check_model_name(cfg.model), data=cfg.data_yaml, imgsz=_imgsz(cfg.imgsz),
                         epochs=cfg.epochs, patience=cfg.patience, batch=cfg.batch, device=cfg.device,
                         project=cfg.project, name=cfg.name, seed=cfg.seed, workers=cfg.workers)
    return eng.train(args)


def eval_rtdetr_detector(
    data_yaml: str,
    weights_path: str,
    split: str = "val",
    imgsz: Union[int, tuple[int, int]] = (704, 1248),
    batch: int = 16,
    device: str = "0",
    project: str | None = None,
    name: str | None = None,
):
    """Evaluate a checkpoint on ``split``; returns a metrics object with
    ``.results_dict`` ("metrics/mAP50(B)", ...), ``.box`` (map50, map, mp, mr,
    curves, curves_results), ``.speed`` (ms per image) and ``.model``."""
    eng = _engine()
    return eng.validate(_check_model_name(weights_path), data_yaml, split=split, imgsz=_imgsz(imgsz),
                        batch=batch, device=device, project=project, name=name)


def save_rtdetr_metrics_json(metrics, out_path: str | Path) -> Path:
    """metrics.json in the schema shared with the YOLO runs."""
    return save_yolo_metrics_json(metrics=metrics, out_path=out_path)


def save_rtdetr_training_summary(
    *,
    train_wall_time_s: float,
    model_name: str,
    data_yaml: str,
    run_name: str,
    out_json_path: str | Path,
    out_csv_path: str | Path,
    results=None,
) -> tuple[Path, Path]:
    """train_summary.{json,csv} in the schema shared with the YOLO runs."""
    return save_yolo_training_summary(train_wall_time_s=train_wall_time_s, model_name=model_name,
                                      data_yaml=data_yaml, run_name=run_name, out_json_path=out_json_path,
                                      out_csv_path=out_csv_path, results=results)


def get_rtdetr_model_size_stats_from_weights(weights_path: str) -> dict:
    """{params_total, params_trainable, flops_g}; None for what cannot be read."""
    stats = {"params_total": None, "params_trainable": None, "flops_g": None}
    try:
        net = _engine().load_model(_check_model_name(weights_path), "cpu")
    except Exception:
        return stats
    try:
        params = list(net.parameters())
        stats["params_total"] = int(sum(p.numel() for p in params))
        stats["params_trainable"] = int(sum(p.numel() for p in params if p.requires_grad))
    except Exception:
        pass
    try:
        stats["flops_g"] = float(net.GFLOPs)
    except Exception:
        pass
    return stats
