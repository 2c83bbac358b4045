"""Train through the RT-DETRv2 adapter (src/models/vision/rtdetr_thirdparty.py).

Same flags and artifacts as the reference's scripts/train_rtdetr_thirdparty.py
(flags :33-58; train_summary.{json,csv}, run_metadata.{json,csv} and
train_adapter_result.json under EVAL_DIR/rtdetr_thirdparty/<run-name>,
:78-140).  The adapter's subprocess is this package's engine
(src/rtdetr_moe/v2_tools.py); the default base configs are the stand-ins in
configs/rtdetrv2/ (tier l: R50 MoE, tier m: R50 MoE with 3 decoder layers).
"""
from __future__ import annotations

import argparse
import json
import sys
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(PKG_ROOT)) if str(PKG_ROOT) not in sys.path else None

from src.models.vision.rtdetr_thirdparty import (  # noqa: E402
    RtdetrThirdPartyTrainConfig,
    collect_runtime_info,
    save_rtdetr_thirdparty_run_metadata,
    save_rtdetr_thirdparty_training_summary,
    train_rtdetr_thirdparty,
)
from src.models.vision.yolo import infer_model_variant_from_weights  # noqa: E402
from src.paths import EVAL_DIR, RUNS_DIR  # noqa: E402

DEFAULT_BASE_CONFIG_L = PKG_ROOT / "configs" / "rtdetrv2" / "rtdetrv2_r50vd_6x_coco.yml"
DEFAULT_BASE_CONFIG_M = PKG_ROOT / "configs" / "rtdetrv2" / "rtdetrv2_r50vd_m_7x_coco.yml"


def parse_args(argv=None) -> argparse.Namespace:
    p = argparse.ArgumentParser(description="Train RT-DETRv2 (third-party adapter) baseline detector.")
    p.add_argument("--model-tier", choices=["l", "m"], default="l")
    p.add_argument("--base-config", type=str, default=None, help="Optional explicit RT-DETRv2 config path.")
    p.add_argument("--train-img-dir", type=str, required=True)
    p.add_argument("--train-ann-json", type=str, required=True)
    p.add_argument("--val-img-dir", type=str, required=True)
    p.add_argument("--val-ann-json", type=str, required=True)
    p.add_argument("--img-h", type=int, default=704)
    p.add_argument("--img-w", type=int, default=1248)
    p.add_argument("--epochs", type=int, default=50)
    p.add_argument("--batch", type=int, default=16)
    p.add_argument("--device", type=str, default="cuda:0")
    p.add_argument("--seed", type=int, default=0)
    p.add_argument("--workers", type=int, default=8)
    p.add_argument("--num-classes", type=int, default=1)
    p.add_argument("--run-name", type=str, default="rtdetrv2_l_thirdparty")
    p.add_argument("--unclear-policy", type=str, default="exclude_unclear")
    p.add_argument("--use-amp", action=argparse.BooleanOptionalAction, default=True,
                   help="Enable/disable automatic mixed precision.")
    return p.parse_args(argv)


def _resolve_base_config(a: argparse.Namespace) -> Path:
    if a.base_config:
        return Path(a.base_config).resolve()
    return DEFAULT_BASE_CONFIG_L if a.model_tier == "l" else DEFAULT_BASE_CONFIG_M


def main(argv=None) -> None:
    a = parse_args(argv)
    base_config = _resolve_base_config(a)
    run_dir = Path(RUNS_DIR) / "rtdetr_thirdparty" / a.run_name
    eval_dir = Path(EVAL_DIR) / "rtdetr_thirdparty" / a.run_name
    run_dir.mkdir(parents=True, exist_ok=True)
    eval_dir.mkdir(parents=True, exist_ok=True)
    cfg = RtdetrThirdPartyTrainConfig(
        base_config=str(base_config), train_img_dir=a.train_img_dir, train_ann_json=a.train_ann_json,
        val_img_dir=a.val_img_dir, val_ann_json=a.val_ann_json, output_dir=str(run_dir), run_name=a.run_name,
        imgsz=(a.img_h, a.img_w), epochs=a.epochs, batch=a.batch, device=a.device, seed=a.seed,
        workers=a.workers, num_classes=a.num_classes, use_amp=bool(a.use_amp))
    print("Starting third-party RT-DETRv2 training with config:")
    print(cfg)
    result = train_rtdetr_thirdparty(cfg)
    sj, sc = save_rtdetr_thirdparty_training_summary(
        run_name=a.run_name, model_name=base_config.stem, base_config=str(base_config),
        train_wall_time_s=float(result["train_wall_time_s"]), out_json_path=eval_dir / "train_summary.json",
        out_csv_path=eval_dir / "train_summary.csv")
    print(f"Saved training summary -> {sj}")
    print(f"Saved training table   -> {sc}")
    metadata = {
        "model_family": "rtdetr_thirdparty",
        "model_variant": infer_model_variant_from_weights(base_config.stem),
        "model_weights": str(result["best_weights_path"]),
        "run_name": a.run_name, "seed": int(a.seed), "split": "train+val",
        "img_h": int(a.img_h), "img_w": int(a.img_w), "unclear_policy": a.unclear_policy,
        "base_config": str(base_config),
        "train_img_dir": str(Path(a.train_img_dir).resolve()),
        "train_ann_json": str(Path(a.train_ann_json).resolve()),
        "val_img_dir": str(Path(a.val_img_dir).resolve()),
        "val_ann_json": str(Path(a.val_ann_json).resolve()),
        "run_dir": str(run_dir), "resolved_config_path": str(result["resolved_config_path"]),
        "best_weights_path": str(result["best_weights_path"]),
        "last_weights_path": str(result["last_weights_path"]),
    }
    metadata.update(collect_runtime_info())
    mj, mc = save_rtdetr_thirdparty_run_metadata(metadata=metadata, out_dir=eval_dir)
    print(f"Saved run metadata   -> {mj}")
    print(f"Saved metadata table -> {mc}")
    raw = eval_dir / "train_adapter_result.json"
    raw.write_text(json.dumps(result, indent=2))
    print(f"Saved adapter output -> {raw}")


if __name__ == "__main__":
    main()
