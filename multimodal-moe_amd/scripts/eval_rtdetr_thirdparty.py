"""Evaluate through the RT-DETRv2 adapter (src/models/vision/rtdetr_thirdparty.py).

Same flags and artifacts as the reference's scripts/eval_rtdetr_thirdparty.py
(flags :35-53; metrics.json, metrics_table.csv, run_metadata.{json,csv},
metrics_key.json under EVAL_DIR/rtdetr_thirdparty/<run-name>, :64-124).
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(PKG_ROOT)) if str(PKG_ROOT) not in sys.path else None

from src.models.vision.rtdetr_thirdparty import (  # noqa: E402
    collect_runtime_info,
    eval_rtdetr_thirdparty,
    save_rtdetr_thirdparty_metrics_json,
    save_rtdetr_thirdparty_run_metadata,
)
from src.models.vision.yolo import infer_model_variant_from_weights, save_metrics_table_csv  # noqa: E402
from src.paths import EVAL_DIR  # noqa: E402

DEFAULT_BASE_CONFIG_L = PKG_ROOT / "configs" / "rtdetrv2" / "rtdetrv2_r50vd_6x_coco.yml"
DEFAULT_BASE_CONFIG_M = PKG_ROOT / "configs" / "rtdetrv2" / "rtdetrv2_r50vd_m_7x_coco.yml"


def parse_args(argv=None) -> argparse.Namespace:
    p = argparse.ArgumentParser(description="Evaluate RT-DETRv2 (third-party adapter) run.")
    p.add_argument("--model-tier", choices=["l", "m"], default="l")
    p.add_argument("--base-config", type=str, default=None, help="Optional explicit RT-DETRv2 config path.")
    p.add_argument("--weights", type=str, required=True, help="Path to checkpoint (.pth), usually best.pth.")
    p.add_argument("--val-img-dir", type=str, required=True)
    p.add_argument("--val-ann-json", type=str, required=True)
    p.add_argument("--split", choices=["val"], default="val")
    p.add_argument("--img-h", type=int, default=704)
    p.add_argument("--img-w", type=int, default=1248)
    p.add_argument("--batch", type=int, default=16)
    p.add_argument("--device", type=str, default="cuda:0")
    p.add_argument("--workers", type=int, default=8)
    p.add_argument("--num-classes", type=int, default=1)
    p.add_argument("--run-name", type=str, default="rtdetrv2_l_thirdparty_eval")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--unclear-policy", type=str, default="exclude_unclear")
    return p.parse_args(argv)


def _resolve_base_config(a: argparse.Namespace) -> Path:
    if a.base_config:
        return Path(a.base_config).resolve()
    return DEFAULT_BASE_CONFIG_L if a.model_tier == "l" else DEFAULT_BASE_CONFIG_M


def main(argv=None) -> None:
    a = parse_args(argv)
    base_config = _resolve_base_config(a)
    out_dir = Path(EVAL_DIR) / "rtdetr_thirdparty" / a.run_name
    out_dir.mkdir(parents=True, exist_ok=True)
    metrics = eval_rtdetr_thirdparty(
        base_config=str(base_config), weights_path=a.weights, val_img_dir=a.val_img_dir,
        val_ann_json=a.val_ann_json, output_dir=str(out_dir), split=a.split, imgsz=(a.img_h, a.img_w),
        batch=a.batch, device=a.device, workers=a.workers, num_classes=a.num_classes)
    out_json = save_rtdetr_thirdparty_metrics_json(metrics=metrics, out_path=out_dir / "metrics.json")
    out_csv = save_metrics_table_csv(metrics, out_dir / "metrics_table.csv")
    print(f"Saved metrics -> {out_json}")
    print(f"Saved table   -> {out_csv}")
    w = Path(a.weights)
    metadata = {
        "model_family": "rtdetr_thirdparty",
        "model_variant": infer_model_variant_from_weights(base_config.stem),
        "model_weights": str(w), "run_name": a.run_name, "seed": int(a.seed), "split": a.split,
        "img_h": int(a.img_h), "img_w": int(a.img_w), "unclear_policy": a.unclear_policy,
        "base_config": str(base_config),
        "val_img_dir": str(Path(a.val_img_dir).resolve()),
        "val_ann_json": str(Path(a.val_ann_json).resolve()),
        "weights_file_size_mb": round(w.stat().st_size / (1024 ** 2), 3) if w.exists() else None,
    }
    metadata.update(collect_runtime_info())
    mj, mc = save_rtdetr_thirdparty_run_metadata(metadata=metadata, out_dir=out_dir)
    print(f"Saved run metadata -> {mj}")
    print(f"Saved metadata table -> {mc}")
    key = out_dir / "metrics_key.json"
    key.write_text(json.dumps({"map50_95": metrics.get("map50_95"), "map50": metrics.get("map50"),
                               "recall": metrics.get("recall")}, indent=2))
    print(f"Saved key metrics -> {key}")


if __name__ == "__main__":
    main()
