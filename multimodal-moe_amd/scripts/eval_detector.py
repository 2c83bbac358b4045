"""Evaluate a detector run and write metrics.json / metrics_table.csv /
run_metadata.{json,csv} under EVAL_DIR/<backend>/<run-name>.

Same flags and artifacts as the reference's scripts/eval_detector.py
(flags :57-89, derived speed metrics :99-116, runtime info :119-141, rtdetr
branch :214-263).  The rtdetr backend runs this package's RT-DETR-MoE engine;
the yolo backend (Ultralytics YOLO) is out of scope here and raises.
"""
from __future__ import annotations

import argparse
import json
import platform
import socket
import sys
from pathlib import Path

PKG_ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(PKG_ROOT)) if str(PKG_ROOT) not in sys.path else None

from src.models.vision.rtdetr import (  # noqa: E402
    eval_rtdetr_detector,
    get_rtdetr_model_size_stats_from_weights,
    infer_model_variant_from_weights,
    save_metrics_table_csv,
    save_rtdetr_metrics_json,
    save_run_metadata_artifacts,
)
from src.paths import EVAL_DIR, EXPORTS_DIR, RUNS_DIR  # noqa: E402


def parse_args(argv=None) -> argparse.Namespace:
    ap = argparse.ArgumentParser(description="Evaluate detector run.")
    ap.add_argument("--backend", choices=["yolo", "rtdetr"], default="yolo")
    ap.add_argument("--data-yaml", type=str,
                    default=str(EXPORTS_DIR / "yolo" / "pedestrian_v1_exclude_unclear" / "dataset.yaml"))
    ap.add_argument("--weights", type=str, required=True, help="checkpoint (best.pt / last.pt) or architecture spec")
    ap.add_argument("--split", choices=["train", "val", "test"], default="val")
    ap.add_argument("--img-h", type=int, default=704)
    ap.add_argument("--img-w", type=int, default=1248)
    ap.add_argument("--rect", action=argparse.BooleanOptionalAction, default=True,
                    help="Rectangular validation batches (inputs here are always H x W, padded to 32).")
    ap.add_argument("--batch", type=int, default=16)
    ap.add_argument("--device", type=str, default="0")
    ap.add_argument("--run-name", type=str, default="yolo_eval")
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--unclear-policy", type=str, default="exclude_unclear",
                    help="Data filtering policy used when exporting dataset labels.")
    return ap.parse_args(argv)


def _num(v):
    try:
        return float(v)
    except Exception:
        return None


def _add_derived_speed_metrics(m: dict) -> dict:
    """fps_inference_only = 1000 / inference ms; speed_total / fps_end_to_end
    when all three stage timings exist."""
    pre, inf, post = (_num(m.get(f"speed_{k}_ms_per_img")) for k in ("preprocess", "inference", "postprocess"))
    if inf is not None and inf > 0:
        m["fps_inference_only"] = 1000.0 / inf
    if None not in (pre, inf, post):
        total = pre + inf + post
        m["speed_total_ms_per_img"] = total
        if total > 0:
            m["fps_end_to_end"] = 1000.0 / total
    return m


def _collect_runtime_info() -> dict:
    info = {"hostname": socket.gethostname(), "platform": platform.platform(),
            "python_version": platform.python_version()}
    try:
        import torch

        info["torch_version"] = str(torch.__version__)
        info["cuda_available"] = bool(torch.cuda.is_available())
        info["cuda_version"] = str(torch.version.cuda)
        info["hip_version"] = str(getattr(torch.version, "hip", None))
        info["cudnn_version"] = int(torch.backends.cudnn.version()) if torch.backends.cudnn.is_available() else None
        if torch.cuda.is_available():
            info["gpu_name"] = str(torch.cuda.get_device_name(0))
            info["gpu_total_mem_gb"] = round(float(torch.cuda.get_device_properties(0).total_memory) / 1024 ** 3, 3)
    except Exception:
        pass
    return info


def main(argv=None) -> None:
    a = parse_args(argv)
    out_dir = Path(EVAL_DIR) / a.backend / a.run_name
    out_dir.mkdir(parents=True, exist_ok=True)
    if a.backend != "rtdetr":
        raise SystemExit("backend 'yolo' (Ultralytics YOLO) is not part of this build; use --backend rtdetr")

    metrics = eval_rtdetr_detector(data_yaml=a.data_yaml, weights_path=a.weights, split=a.split,
                                   imgsz=(a.img_h, a.img_w), batch=a.batch, device=a.device,
                                   project=str(RUNS_DIR / "rtdetr"), name=f"{a.run_name}_val")
    out_json = save_rtdetr_metrics_json(metrics=metrics, out_path=out_dir / "metrics.json")
    doc = _add_derived_speed_metrics(json.loads(out_json.read_text()))
    if doc.get("params_total") is None and doc.get("flops_g") is None:
        try:
            doc.update(get_rtdetr_model_size_stats_from_weights(a.weights))
        except Exception:
            pass
    out_json.write_text(json.dumps(doc, indent=2))
    out_csv = save_metrics_table_csv(doc, out_dir / "metrics_table.csv")

    yaml_path = Path(a.data_yaml)
    w = Path(a.weights)
    meta = {
        "model_family": "rtdetr",
        "model_variant": infer_model_variant_from_weights(a.weights),
        "model_weights": a.weights,
        "run_name": a.run_name,
        "seed": int(a.seed),
        "split": a.split,
        "img_h": int(a.img_h),
        "img_w": int(a.img_w),
        "unclear_policy": a.unclear_policy,
        "dataset_export_name": yaml_path.parent.name if yaml_path.name == "dataset.yaml" else yaml_path.stem,
        "data_yaml": str(yaml_path),
        "weights_file_size_mb": round(w.stat().st_size / 1024 ** 2, 3) if w.exists() else None,
    }
    meta.update(_collect_runtime_info())
    mj, mc = save_run_metadata_artifacts(metadata=meta, out_json_path=out_dir / "run_metadata.json",
                                         out_csv_path=out_dir / "run_metadata.csv")
    print(f"Saved metrics -> {out_json}")
    print(f"Saved table   -> {out_csv}")
    print(f"Saved run metadata -> {mj}")
    print(f"Saved metadata table -> {mc}")


if __name__ == "__main__":
    main()
