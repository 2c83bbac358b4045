"""The reference's own, unchanged callers run against this build's operator API.

``/root/reference/scripts/train_rtdetr.py`` and ``eval_detector.py`` put their
project root on ``sys.path`` only when it is not there yet
(train_rtdetr.py:16-18, eval_detector.py:24-26).  With
``PYTHONPATH=<build pkg>:<reference root>`` both roots are on the path, the
build's first, so ``from src.models.vision.rtdetr import ...`` (and
``src.models.vision.yolo``, ``src.paths``) resolve to this package while the
scripts themselves are the reference's files, executed where they lie (no copy,
no bytecode written: PYTHONDONTWRITEBYTECODE).  This is INTEGRATION.md 1's
recipe.  Build-container only: skipped where /root/reference is absent (the GPU
box), never imported by product code.  Config C1 (BASELINE.json configs[0]):
RT-DETR-R18 + 4-expert top-1 MoE, 2 frames at 640x640, CPU.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "multimodal-moe_amd"
REF = Path("/root/reference")

pytestmark = pytest.mark.skipif(not (REF / "scripts" / "train_rtdetr.py").exists(),
                                reason="reference checkout not present (build container only)")


def _env(tmp_path):
    return dict(os.environ, PYTHONPATH=f"{PKG}{os.pathsep}{REF}", PYTHONDONTWRITEBYTECODE="1",
                OUTPUTS_DIR=str(tmp_path), EVAL_DIR=str(tmp_path / "eval"), RUNS_DIR=str(tmp_path / "runs"),
                OMP_NUM_THREADS="8")


def test_reference_eval_detector_imports_resolve_to_build(tmp_path):
    """eval_detector.py:28-41 imports eval_yolo_detector and
    get_yolo_model_size_stats_from_weights at module load; with the build first
    on the path every imported name comes from this package."""
    code = ("import runpy, sys; sys.argv=['eval_detector.py', '--help']\n"
            "import src.models.vision.yolo as y, src.models.vision.rtdetr as r\n"
            f"assert y.__file__.startswith({str(PKG)!r}), y.__file__\n"
            f"assert r.__file__.startswith({str(PKG)!r}), r.__file__\n"
            "try:\n"
            f"    runpy.run_path({str(REF / 'scripts' / 'eval_detector.py')!r}, run_name='__main__')\n"
            "except SystemExit as e:\n"
            "    assert e.code == 0, e.code\n")
    r = subprocess.run([sys.executable, "-c", code], capture_output=True, text=True, env=_env(tmp_path),
                       timeout=300, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    assert "--backend" in r.stdout


def test_reference_scripts_train_then_eval_c1(tmp_path):
    """The reference's train_rtdetr.py then eval_detector.py --backend rtdetr,
    unchanged, on config C1 (R18 + moe4 top-1, 2x 640x640 frames, CPU)."""
    env = _env(tmp_path)
    common = ["--img-h", "640", "--img-w", "640", "--device", "cpu", "--data-yaml", "synthetic:1"]
    r = subprocess.run([sys.executable, str(REF / "scripts" / "train_rtdetr.py"), "--model", "rtdetr-r18-moe4-top1",
                        "--batch", "2", "--epochs", "1", "--workers", "0", "--run-name", "ref_c1", *common],
                       capture_output=True, text=True, env=env, timeout=900, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    ev = tmp_path / "eval" / "rtdetr" / "ref_c1"
    summ = json.loads((ev / "train_summary.json").read_text())
    assert summ["model_name"] == "rtdetr-r18-moe4-top1" and summ["params_total"] > 1e6 and summ["flops_g"] > 0
    meta = json.loads((ev / "run_metadata.json").read_text())
    assert meta["model_family"] == "rtdetr" and meta["img_h"] == 640
    assert (ev / "train_metrics.json").exists()
    ck = tmp_path / "runs" / "rtdetr" / "ref_c1" / "weights" / "best.pt"
    assert ck.exists()
    r = subprocess.run([sys.executable, str(REF / "scripts" / "eval_detector.py"), "--backend", "rtdetr",
                        "--weights", str(ck), "--batch", "2", "--run-name", "ref_c1e", *common],
                       capture_output=True, text=True, env=env, timeout=900, cwd=str(tmp_path))
    assert r.returncode == 0, r.stderr[-3000:]
    m = json.loads((tmp_path / "eval" / "rtdetr" / "ref_c1e" / "metrics.json").read_text())
    for k in ("map50", "map50_95", "precision", "recall", "speed_inference_ms_per_img", "fps_inference_only",
              "params_total", "flops_g"):
        assert k in m, k
    assert (tmp_path / "eval" / "rtdetr" / "ref_c1e" / "metrics_table.csv").exists()
    assert json.loads((tmp_path / "eval" / "rtdetr" / "ref_c1e" / "run_metadata.json").read_text())["split"] == "val"


def test_reference_yolo_backend_fails_with_import_error(tmp_path):
    """The YOLO branch is out of scope: it fails the way the reference does
    without Ultralytics (ImportError from the lazy import), not at import time."""
    r = subprocess.run([sys.executable, str(REF / "scripts" / "eval_detector.py"), "--backend", "yolo",
                        "--weights", "yolo26n.pt", "--device", "cpu"],
                       capture_output=True, text=True, env=_env(tmp_path), timeout=300, cwd=str(tmp_path))
    assert r.returncode != 0
    assert "ImportError" in r.stderr and "Ultralytics is required" in r.stderr
