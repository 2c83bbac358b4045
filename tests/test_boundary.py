"""The drop-in boundary: the reference's operator API names/signatures, the
CLI flags, and config C1 (R18, 4 experts, top-1, 2 images, CPU) end to end."""
from __future__ import annotations

import inspect
import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "multimodal-moe_amd"


def test_operator_api_matches_reference_signatures():
    from src.models.vision import rtdetr as R

    # reference src/models/vision/rtdetr.py:36-48, 77, 98-107, 131, 141-150, 165
    assert [f for f in R.RtdetrTrainConfig.__dataclass_fields__] == [
        "data_yaml", "model", "imgsz", "epochs", "patience", "batch", "device", "project", "name", "seed", "workers"]
    cfg = R.RtdetrTrainConfig(data_yaml="x")
    assert (cfg.imgsz, cfg.epochs, cfg.patience, cfg.batch, cfg.device, cfg.project, cfg.name, cfg.seed,
            cfg.workers) == ((704, 1248), 50, 100, 16, "0", "outputs/runs/rtdetr", "baseline", 0, 8)
    assert list(inspect.signature(R.train_rtdetr_detector).parameters) == ["cfg"]
    ev = inspect.signature(R.eval_rtdetr_detector).parameters
    assert list(ev) == ["data_yaml", "weights_path", "split", "imgsz", "batch", "device", "project", "name"]
    assert [ev[k].default for k in ("split", "imgsz", "batch", "device", "project", "name")] == \
        ["val", (704, 1248), 16, "0", None, None]
    assert list(inspect.signature(R.save_rtdetr_metrics_json).parameters) == ["metrics", "out_path"]
    assert list(inspect.signature(R.save_rtdetr_training_summary).parameters) == [
        "train_wall_time_s", "model_name", "data_yaml", "run_name", "out_json_path", "out_csv_path", "results"]
    assert list(inspect.signature(R.get_rtdetr_model_size_stats_from_weights).parameters) == ["weights_path"]
    for name in ("infer_model_variant_from_weights", "save_metrics_table_csv", "save_run_metadata_artifacts"):
        assert callable(getattr(R, name))


def test_hub_weight_name_is_rejected():
    from src.models.vision import rtdetr as R

    with pytest.raises(ValueError, match="network"):
        R.train_rtdetr_detector(R.RtdetrTrainConfig(data_yaml="synthetic:1", model="rtdetr-l.pt", device="cpu"))


def test_cli_flags_match_reference():
    sys.path.insert(0, str(PKG))
    from scripts import eval_detector, train_rtdetr

    t = vars(train_rtdetr.parse_args([]))
    assert set(t) == {"data_yaml", "model", "img_h", "img_w", "epochs", "patience", "batch", "device", "seed",
                      "workers", "run_name", "unclear_policy"}
    assert (t["img_h"], t["img_w"], t["epochs"], t["batch"], t["device"]) == (704, 1248, 50, 16, "0")
    e = vars(eval_detector.parse_args(["--weights", "w.pt"]))
    assert set(e) == {"backend", "data_yaml", "weights", "split", "img_h", "img_w", "rect", "batch", "device",
                      "run_name", "seed", "unclear_policy"}


def test_config_c1_train_then_eval_on_cpu(tmp_path):
    """BASELINE.json configs[0]: train_rtdetr.py R18 + 4-expert top-1 MoE, 2 frames, CPU only."""
    env = dict(os.environ, OUTPUTS_DIR=str(tmp_path), OMP_NUM_THREADS="4")
    common = ["--img-h", "640", "--img-w", "640", "--device", "cpu", "--data-yaml", "synthetic:1"]
    r = subprocess.run([sys.executable, str(PKG / "scripts/train_rtdetr.py"), "--model", "rtdetr-r18-moe4-top1",
                        "--batch", "2", "--epochs", "1", "--workers", "0", "--run-name", "c1", *common],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    ev = tmp_path / "eval" / "rtdetr" / "c1"
    summ = json.loads((ev / "train_summary.json").read_text())
    assert summ["params_total"] > 1e6 and summ["flops_g"] > 0
    assert json.loads((ev / "run_metadata.json").read_text())["model_family"] == "rtdetr"
    ck = tmp_path / "runs" / "rtdetr" / "c1" / "weights" / "best.pt"
    assert ck.exists()
    r = subprocess.run([sys.executable, str(PKG / "scripts/eval_detector.py"), "--backend", "rtdetr", "--weights",
                        str(ck), "--batch", "2", "--run-name", "c1e", *common],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-2000:]
    m = json.loads((tmp_path / "eval" / "rtdetr" / "c1e" / "metrics.json").read_text())
    for k in ("map50", "map50_95", "precision", "recall", "fps_inference_only", "params_total"):
        assert k in m
