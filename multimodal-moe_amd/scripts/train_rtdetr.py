"""Train RT-DETR(-MoE) and write the shared run artifacts.

Same command line and outputs as the reference's scripts/train_rtdetr.py
(flags :30-61; artifacts train_summary.{json,csv}, train_metrics.json,
run_metadata.{json,csv} under EVAL_DIR/rtdetr/<run-name>, :91-138), running
on this package's engine.  Example (config C1, CPU plumbing):

  python scripts/train_rtdetr.py --data-yaml synthetic:4 --model rtdetr-r18-moe4-top1 \\
      --img-h 640 --img-w 640 --batch 2 --epochs 1 --device cpu --workers 0
"""
from __future__ import annotations

import argparse
import json
import sys
import time
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(PKG_ROOT)) if str(PKG_ROOT) not in sys.path else None

from src.models.vision.rtdetr import (  # noqa: E402
    RtdetrTrainConfig,
    infer_model_variant_from_weights,
    save_rtdetr_training_summary,
    save_run_metadata_artifacts,
    train_rtdetr_detector,
)
from src.paths import EVAL_DIR, EXPORTS_DIR, RUNS_DIR  # noqa: E402

# (flag, type, default, help) -- the reference's flag set
FLAGS = [
    ("--data-yaml", str, str(EXPORTS_DIR / "yolo" / "pedestrian_v1_exclude_unclear" / "dataset.yaml"),
     "Ultralytics dataset.yaml, or 'synthetic[:N]' for N synthetic ZOD-shaped batches per epoch"),
    ("--model", str, "rtdetr-r50-moe8-top2", "architecture spec or checkpoint path"),
    ("--img-h", int, 704, None),
    ("--img-w", int, 1248, None),
    ("--epochs", int, 50, None),
    ("--patience", int, 100, "Early stopping patience (epochs with no val improvement)."),
    ("--batch", int, 16, None),
    ("--device", str, "0", "'cpu', '0' or '0,1,...' (one process per GPU)"),
    ("--seed", int, 0, None),
    ("--workers", int, 8, None),
    ("--run-name", str, "rtdetr_l_pedestrian_v1", None),
    ("--unclear-policy", str, "exclude_unclear", "Data filtering policy used when exporting dataset labels."),
]


def parse_args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(description="Train RT-DETR(-MoE) detector.")
    for flag, typ, default, hlp in FLAGS:
        ap.add_argument(flag, type=typ, default=default, help=hlp)
    return ap.parse_args(argv)


def _export_name(data_yaml: str) -> str:
    p = Path(data_yaml)
    return p.parent.name if p.name == "dataset.yaml" else p.stem


def main(argv=None) -> None:
    a = parse_args(argv)
    cfg = RtdetrTrainConfig(data_yaml=a.data_yaml, model=a.model, imgsz=(a.img_h, a.img_w), epochs=a.epochs,
                            patience=a.patience, batch=a.batch, device=a.device, seed=a.seed, workers=a.workers,
                            project=str(RUNS_DIR / "rtdetr"), name=a.run_name)
    print("Starting RT-DETR training with config:")
    print(cfg)
    start = time.perf_counter()
    results = train_rtdetr_detector(cfg)
    wall = time.perf_counter() - start

    report = Path(EVAL_DIR) / "rtdetr" / a.run_name
    report.mkdir(parents=True, exist_ok=True)
    js, cs = save_rtdetr_training_summary(train_wall_time_s=wall, model_name=a.model, data_yaml=a.data_yaml,
                                          run_name=a.run_name, out_json_path=report / "train_summary.json",
                                          out_csv_path=report / "train_summary.csv", results=results)
    print(f"Saved training summary -> {js}")
    print(f"Saved training table   -> {cs}")
    if hasattr(results, "results_dict"):
        try:
            (report / "train_metrics.json").write_text(json.dumps(dict(results.results_dict), indent=2))
            print(f"Saved train metrics   -> {report / 'train_metrics.json'}")
        except Exception:
            pass
    meta = {
        "model_family": "rtdetr",
        "model_variant": infer_model_variant_from_weights(a.model),
        "model_weights": a.model,
        "run_name": a.run_name,
        "seed": int(a.seed),
        "split": "train+val",
        "img_h": int(a.img_h),
        "img_w": int(a.img_w),
        "unclear_policy": a.unclear_policy,
        "dataset_export_name": _export_name(a.data_yaml),
        "data_yaml": str(Path(a.data_yaml)),
    }
    mj, mc = save_run_metadata_artifacts(metadata=meta, out_json_path=report / "run_metadata.json",
                                         out_csv_path=report / "run_metadata.csv")
    print(f"Saved run metadata   -> {mj}")
    print(f"Saved metadata table -> {mc}")


if __name__ == "__main__":
    main()
