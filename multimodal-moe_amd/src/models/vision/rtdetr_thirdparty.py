"""RT-DETRv2 third-party adapter, pointed at this package's engine.

Same API, config schema and artifacts as the reference's
src/models/vision/rtdetr_thirdparty.py:

* ``RtdetrThirdPartyTrainConfig`` (:23-38), ``train_rtdetr_thirdparty``
  (:182-238), ``eval_rtdetr_thirdparty`` (:241-319),
  ``save_rtdetr_thirdparty_metrics_json`` (:322-326),
  ``save_rtdetr_thirdparty_training_summary`` (:329-347),
  ``save_rtdetr_thirdparty_run_metadata`` (:350-360), ``collect_runtime_info``;
* the override config written next to the run (``resolved_config.yml``,
  JSON text, keys as :74-114, including the upstream spelling ``epoches``);
* a subprocess with the RT-DETRv2 ``tools/train.py`` flags, its stdout/stderr
  saved as ``stdout.log``/``stderr.log`` (``stdout_eval.log``/
  ``stderr_eval.log`` for eval), ``RuntimeError`` naming the logs on a
  non-zero exit, and the COCO summary parsed from stdout with the
  reference's patterns (:132-155).

The difference: the subprocess is ``python -m src.rtdetr_moe.v2_tools``
(the RT-DETR-MoE engine with its HIP kernels) run from this package's root,
instead of the RT-DETRv2 checkout, which is an empty submodule in the
reference.  ``base_config`` may name an RT-DETRv2 config (its file name picks
the architecture, see v2_tools.arch_from_config) or a YAML/JSON file with a
``model`` key holding a build spec.
"""
from __future__ import annotations

import json
import platform
import re
import socket
import subprocess
import sys
import time
from dataclasses import dataclass
from pathlib import Path
from typing import Any

from src.models.vision.yolo import save_metrics_table_csv, save_run_metadata_artifacts


@dataclass
class RtdetrThirdPartyTrainConfig:
    base_config: str
    train_img_dir: str
    train_ann_json: str
    val_img_dir: str
    val_ann_json: str
    output_dir: str
    run_name: str
    imgsz: tuple[int, int] = (704, 1248)
    epochs: int = 50
    batch: int = 16
    device: str = "cuda:0"
    seed: int = 0
    workers: int = 8
    num_classes: int = 1
    use_amp: bool = True


def _engine_root() -> Path:
    # src/models/vision/rtdetr_thirdparty.py -> package root is parents[3]
    return Path(__file__).resolve().parents[3]


def _write_runtime_config(*, base_config: str, out_path: Path, train_img_dir: str, train_ann_json: str,
                          val_img_dir: str, val_ann_json: str, output_dir: str, img_h: int, img_w: int, epochs: int,
                          batch: int, workers: int, num_classes: int) -> Path:
    """The override config (the reference's schema, :74-114)."""
    def ds(img_dir, ann, ops):
        return {"img_folder": str(Path(img_dir).resolve()), "ann_file": str(Path(ann).resolve()),
                "transforms": {"ops": ops}}

    size = [int(img_h), int(img_w)]
    train_ops = [{"type": "RandomPhotometricDistort", "p": 0.5}, {"type": "RandomHorizontalFlip"},
                 {"type": "Resize", "size": size}, {"type": "SanitizeBoundingBoxes", "min_size": 1},
                 {"type": "ConvertPILImage", "dtype": "float32", "scale": True},
                 {"type": "ConvertBoxes", "fmt": "cxcywh", "normalize": True}]
    val_ops = [{"type": "Resize", "size": size}, {"type": "ConvertPILImage", "dtype": "float32", "scale": True}]
    cfg: dict[str, Any] = {
        "__include__": [str(Path(base_config).resolve())],
        "output_dir": str(Path(output_dir).resolve()),
        "epoches": int(epochs),  # upstream spelling
        "num_classes": int(num_classes),
        "remap_mscoco_category": False,
        "eval_spatial_size": size,
        "train_dataloader": {"dataset": ds(train_img_dir, train_ann_json, train_ops),
                             "collate_fn": {"type": "BatchImageCollateFunction"},
                             "total_batch_size": int(batch), "num_workers": int(workers)},
        "val_dataloader": {"dataset": ds(val_img_dir, val_ann_json, val_ops),
                           "total_batch_size": int(batch), "num_workers": int(workers)},
    }
    out_path.parent.mkdir(parents=True, exist_ok=True)
    out_path.write_text(json.dumps(cfg, indent=2))
    return out_path


def _run_subprocess(command: list[str], cwd: Path) -> subprocess.CompletedProcess:
    return subprocess.run(command, cwd=str(cwd), text=True, capture_output=True, check=False)


_COCO_PATTERNS = {
    "map50_95": r"Average Precision\s+\(AP\)\s+@\[ IoU=0\.50:0\.95 .* =\s+([0-9.]+)",
    "map50": r"Average Precision\s+\(AP\)\s+@\[ IoU=0\.50\s+\|.* =\s+([0-9.]+)",
    "recall": r"Average Recall\s+\(AR\)\s+@\[ IoU=0\.50:0\.95 .* maxDets=\s*100 \]\s*=\s*([0-9.]+)",
}


def _parse_coco_summary_from_stdout(stdout: str) -> dict[str, float | None]:
    """AP/AR from COCO summary lines (the reference's patterns, :132-155);
    precision is not in the summary and stays None."""
    metrics: dict[str, float | None] = {"map50_95": None, "map50": None, "precision": None, "recall": None}
    for key, pat in _COCO_PATTERNS.items():
        m = re.search(pat, stdout)
        if m:
            try:
                metrics[key] = float(m.group(1))
            except ValueError:
                metrics[key] = None
    return metrics


def _collect_runtime_info() -> dict:
    info = {"hostname": socket.gethostname(), "platform": platform.platform(),
            "python_version": platform.python_version()}
    try:
        import torch

        info["torch_version"] = str(torch.__version__)
        info["cuda_available"] = bool(torch.cuda.is_available())
        info["cuda_version"] = str(torch.version.cuda)
        info["hip_version"] = str(torch.version.hip)
        info["cudnn_version"] = int(torch.backends.cudnn.version()) if torch.backends.cudnn.is_available() else None
        if torch.cuda.is_available():
            info["gpu_name"] = str(torch.cuda.get_device_name(0))
            props = torch.cuda.get_device_properties(0)
            info["gpu_total_mem_gb"] = round(float(props.total_memory) / (1024 ** 3), 3)
    except Exception:
        pass
    return info


def _tool(args: list[str]) -> list[str]:
    return [sys.executable, "-m", "src.rtdetr_moe.v2_tools", *args]


def _failed(what: str, command: list[str], rc: int, out: Path, err: Path) -> RuntimeError:
    return RuntimeError(f"RT-DETR third-party {what} failed.\nCommand: {' '.join(command)}\n"
                        f"Return code: {rc}\nSee logs: {out} and {err}")


def train_rtdetr_thirdparty(cfg: RtdetrThirdPartyTrainConfig) -> dict[str, Any]:
    run_dir = Path(cfg.output_dir).resolve()
    run_dir.mkdir(parents=True, exist_ok=True)
    resolved = run_dir / "resolved_config.yml"
    _write_runtime_config(base_config=cfg.base_config, out_path=resolved, train_img_dir=cfg.train_img_dir,
                          train_ann_json=cfg.train_ann_json, val_img_dir=cfg.val_img_dir,
                          val_ann_json=cfg.val_ann_json, output_dir=str(run_dir), img_h=int(cfg.imgsz[0]),
                          img_w=int(cfg.imgsz[1]), epochs=int(cfg.epochs), batch=int(cfg.batch),
                          workers=int(cfg.workers), num_classes=int(cfg.num_classes))
    command = _tool(["-c", str(resolved), "-d", cfg.device, "--seed", str(cfg.seed), "--output-dir", str(run_dir)])
    if cfg.use_amp:
        command.append("--use-amp")
    t0 = time.perf_counter()
    proc = _run_subprocess(command, _engine_root())
    elapsed = time.perf_counter() - t0
    out, err = run_dir / "stdout.log", run_dir / "stderr.log"
    out.write_text(proc.stdout or "")
    err.write_text(proc.stderr or "")
    if proc.returncode != 0:
        raise _failed("training", command, proc.returncode, out, err)
    return {"run_dir": str(run_dir), "resolved_config_path": str(resolved),
            "best_weights_path": str(run_dir / "best.pth"), "last_weights_path": str(run_dir / "last.pth"),
            "train_wall_time_s": float(elapsed)}


def eval_rtdetr_thirdparty(*, base_config: str, weights_path: str, val_img_dir: str, val_ann_json: str,
                           output_dir: str, split: str = "val", imgsz: tuple[int, int] = (704, 1248), batch: int = 16,
                           device: str = "cuda:0", workers: int = 8, num_classes: int = 1) -> dict[str, Any]:
    """Test-only run on ``val``; AP/AR parsed from the printed COCO summary."""
    if split != "val":
        raise ValueError("Third-party v1 adapter currently supports split='val' only.")
    eval_dir = Path(output_dir).resolve()
    eval_dir.mkdir(parents=True, exist_ok=True)
    resolved = eval_dir / "resolved_eval_config.yml"
    _write_runtime_config(base_config=base_config, out_path=resolved, train_img_dir=val_img_dir,
                          train_ann_json=val_ann_json, val_img_dir=val_img_dir, val_ann_json=val_ann_json,
                          output_dir=str(eval_dir), img_h=int(imgsz[0]), img_w=int(imgsz[1]), epochs=1,
                          batch=int(batch), workers=int(workers), num_classes=int(num_classes))
    command = _tool(["-c", str(resolved), "-r", str(Path(weights_path).resolve()), "-d", device, "--test-only",
                     "--output-dir", str(eval_dir)])
    t0 = time.perf_counter()
    proc = _run_subprocess(command, _engine_root())
    elapsed = time.perf_counter() - t0
    out, err = eval_dir / "stdout_eval.log", eval_dir / "stderr_eval.log"
    out.write_text(proc.stdout or "")
    err.write_text(proc.stderr or "")
    if proc.returncode != 0:
        raise _failed("eval", command, proc.returncode, out, err)
    metrics = _parse_coco_summary_from_stdout(proc.stdout or "")
    metrics.update({"split": split, "speed_total_s_eval_run": float(elapsed), "speed_total_ms_per_img": None,
                    "fps_end_to_end": None, "params_total": None, "params_trainable": None, "flops_g": None})
    return metrics


def save_rtdetr_thirdparty_metrics_json(metrics: dict[str, Any], out_path: str | Path) -> Path:
    out_path = Path(out_path)
    out_path.parent.mkdir(parents=True, exist_ok=True)
    out_path.write_text(json.dumps(metrics, indent=2))
    return out_path


def save_rtdetr_thirdparty_training_summary(*, run_name: str, model_name: str, base_config: str,
                                            train_wall_time_s: float, out_json_path: str | Path,
                                            out_csv_path: str | Path) -> tuple[Path, Path]:
    summary = {"run_name": run_name, "model_name": model_name, "base_config": str(base_config),
               "train_wall_time_s": float(train_wall_time_s)}
    out_json_path = Path(out_json_path)
    out_json_path.parent.mkdir(parents=True, exist_ok=True)
    out_json_path.write_text(json.dumps(summary, indent=2))
    return out_json_path, save_metrics_table_csv(summary, out_csv_path)


def save_rtdetr_thirdparty_run_metadata(*, metadata: dict[str, Any], out_dir: str | Path) -> tuple[Path, Path]:
    out_dir = Path(out_dir)
    return save_run_metadata_artifacts(metadata=metadata, out_json_path=out_dir / "run_metadata.json",
                                       out_csv_path=out_dir / "run_metadata.csv")


def collect_runtime_info() -> dict:
    return _collect_runtime_info()
