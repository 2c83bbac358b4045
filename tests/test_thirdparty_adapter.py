"""The RT-DETRv2 adapter: the reference's API names,
its override-config schema, its COCO-summary parsing, the COCO input path,
and a CPU train -> test-only eval round trip through the adapter's subprocess
(src/rtdetr_moe/v2_tools.py).  Reference: src/models/vision/rtdetr_thirdparty.py,
scripts/{train,eval}_rtdetr_thirdparty.py."""
from __future__ import annotations

import inspect
import json
import os
import subprocess
import sys
from pathlib import Path

import numpy as np
import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "multimodal-moe_amd"

# pycocotools COCOeval.summarize() output (its fixed layout; values arbitrary)
PYCOCO_SUMMARY = """IoU metric: bbox
 Average Precision  (AP) @[ IoU=0.50:0.95 | area=   all | maxDets=100 ] = 0.412
 Average Precision  (AP) @[ IoU=0.50      | area=   all | maxDets=100 ] = 0.705
 Average Precision  (AP) @[ IoU=0.75      | area=   all | maxDets=100 ] = 0.431
 Average Precision  (AP) @[ IoU=0.50:0.95 | area= small | maxDets=100 ] = 0.210
 Average Recall     (AR) @[ IoU=0.50:0.95 | area=   all | maxDets=  1 ] = 0.301
 Average Recall     (AR) @[ IoU=0.50:0.95 | area=   all | maxDets= 10 ] = 0.489
 Average Recall     (AR) @[ IoU=0.50:0.95 | area=   all | maxDets=100 ] = 0.553
"""


def test_api_names_and_config_defaults():
    from src.models.vision import rtdetr_thirdparty as T

    for name in ("RtdetrThirdPartyTrainConfig", "train_rtdetr_thirdparty", "eval_rtdetr_thirdparty",
                 "save_rtdetr_thirdparty_metrics_json", "save_rtdetr_thirdparty_training_summary",
                 "save_rtdetr_thirdparty_run_metadata", "collect_runtime_info"):
        assert hasattr(T, name), name
    f = T.RtdetrThirdPartyTrainConfig.__dataclass_fields__
    assert list(f) == ["base_config", "train_img_dir", "train_ann_json", "val_img_dir", "val_ann_json",
                       "output_dir", "run_name", "imgsz", "epochs", "batch", "device", "seed", "workers",
                       "num_classes", "use_amp"]
    c = T.RtdetrThirdPartyTrainConfig("b", "ti", "ta", "vi", "va", "o", "r")
    assert (c.imgsz, c.epochs, c.batch, c.device, c.seed, c.workers, c.num_classes, c.use_amp) == \
        ((704, 1248), 50, 16, "cuda:0", 0, 8, 1, True)
    ev = inspect.signature(T.eval_rtdetr_thirdparty).parameters
    assert list(ev) == ["base_config", "weights_path", "val_img_dir", "val_ann_json", "output_dir", "split",
                        "imgsz", "batch", "device", "workers", "num_classes"]


def test_runtime_config_schema(tmp_path):
    from src.models.vision.rtdetr_thirdparty import _write_runtime_config

    p = _write_runtime_config(base_config="base.yml", out_path=tmp_path / "r.yml", train_img_dir="ti",
                              train_ann_json="ta.json", val_img_dir="vi", val_ann_json="va.json",
                              output_dir=str(tmp_path), img_h=704, img_w=1248, epochs=3, batch=4, workers=2,
                              num_classes=1)
    d = json.loads(p.read_text())
    assert set(d) == {"__include__", "output_dir", "epoches", "num_classes", "remap_mscoco_category",
                      "eval_spatial_size", "train_dataloader", "val_dataloader"}
    assert d["epoches"] == 3 and d["eval_spatial_size"] == [704, 1248] and d["remap_mscoco_category"] is False
    tr = d["train_dataloader"]
    assert [o["type"] for o in tr["dataset"]["transforms"]["ops"]] == [
        "RandomPhotometricDistort", "RandomHorizontalFlip", "Resize", "SanitizeBoundingBoxes", "ConvertPILImage",
        "ConvertBoxes"]
    assert tr["collate_fn"] == {"type": "BatchImageCollateFunction"}
    assert (tr["total_batch_size"], tr["num_workers"]) == (4, 2)
    assert [o["type"] for o in d["val_dataloader"]["dataset"]["transforms"]["ops"]] == ["Resize", "ConvertPILImage"]


def test_parse_coco_summary():
    from src.models.vision.rtdetr_thirdparty import _parse_coco_summary_from_stdout as parse
    from src.rtdetr_moe.metrics import BoxMetrics
    from src.rtdetr_moe.v2_tools import coco_summary

    assert parse(PYCOCO_SUMMARY) == {"map50_95": 0.412, "map50": 0.705, "precision": None, "recall": 0.553}
    assert parse("") == {"map50_95": None, "map50": None, "precision": None, "recall": None}
    # the engine's printed summary parses back to its values
    out = coco_summary(BoxMetrics(map=0.25, map50=0.5), 0.125, 0.375)
    assert parse(out) == {"map50_95": 0.25, "map50": 0.5, "precision": None, "recall": 0.375}


def test_arch_from_config(tmp_path):
    from src.rtdetr_moe.v2_tools import arch_from_config, load_config

    base = PKG / "configs" / "rtdetrv2" / "rtdetrv2_r50vd_m_7x_coco.yml"
    over = tmp_path / "o.yml"
    over.write_text(json.dumps({"__include__": [str(base)], "num_classes": 1}))
    assert arch_from_config(load_config(over)) == "rtdetr-r50-moe8-top2-dec3"
    over.write_text(json.dumps({"__include__": ["/absent/rtdetrv2_r18vd_120e_coco.yml"]}))
    assert arch_from_config(load_config(over)) == "rtdetr-r18-moe4-top1"
    over.write_text(json.dumps({"__include__": ["/absent/rtdetrv2_r101vd_6x_coco.yml"]}))
    assert arch_from_config(load_config(over)) == "rtdetr-r50-moe8-top2"


def _coco(tmp_path, n_img=4, w=96, h=64):
    from PIL import Image

    rng = np.random.default_rng(0)
    img_dir = tmp_path / "images"
    img_dir.mkdir()
    images, anns = [], []
    bins = ["night", "twilight", None, "high_sun"]
    for i in range(n_img):
        Image.fromarray(rng.integers(0, 255, (h, w, 3), dtype=np.uint8)).save(img_dir / f"f{i}.jpg")
        im = {"id": i + 1, "file_name": f"f{i}.jpg", "width": w, "height": h}
        im["solar_context_bin"] = bins[i % 4]
        images.append(im)
        for j in range(i % 3):
            anns.append({"id": len(anns) + 1, "image_id": i + 1, "category_id": 1,
                         "bbox": [10.0 + 20 * j, 8.0, 16.0, 30.0], "area": 480.0, "iscrowd": 0})
    anns.append({"id": len(anns) + 1, "image_id": 1, "category_id": 1, "bbox": [90.0, 60.0, 40.0, 40.0],
                 "area": 1600.0, "iscrowd": 0})  # clipped to 6 x 4 px
    anns.append({"id": len(anns) + 1, "image_id": 1, "category_id": 1, "bbox": [1.0, 1.0, 5.0, 5.0],
                 "area": 25.0, "iscrowd": 1})  # crowd: skipped
    ann = tmp_path / "ann.json"
    ann.write_text(json.dumps({"images": images, "annotations": anns,
                               "categories": [{"id": 1, "name": "pedestrian", "supercategory": "person"}]}))
    return img_dir, ann


def test_coco_dataset_boxes_and_contexts(tmp_path):
    import torch

    from src.moe.context import MISSING_ID, context_id_from_label
    from src.rtdetr_moe.data import CocoDataset

    img_dir, ann = _coco(tmp_path)
    ds = CocoDataset(img_dir, ann, imgsz=(64, 96), pad_to=32)
    assert len(ds) == 4 and ds.num_classes == 1
    img, t, ctx = ds[0]
    assert img.shape == (3, 64, 96) and ctx == context_id_from_label("night")
    # only the clipped box (90..96 x 60..64) survives in image 1; label 0 (category id 1)
    torch.testing.assert_close(t["boxes"], torch.tensor([[93 / 96, 62 / 64, 6 / 96, 4 / 64]]))
    assert t["labels"].tolist() == [0]
    _, t2, ctx2 = ds[2]
    assert ctx2 == MISSING_ID and len(t2["boxes"]) == 2
    torch.testing.assert_close(t2["boxes"][1], torch.tensor([38 / 96, 23 / 64, 16 / 96, 30 / 64]))


@pytest.mark.slow
def test_train_then_eval_through_adapter_on_cpu(tmp_path):
    """train_rtdetr_thirdparty.py -> eval_rtdetr_thirdparty.py on a 4-image COCO
    export, R18 stand-in config, CPU: every artifact the reference writes.
    (256 x 160 frames: enough encoder tokens for the 300 queries.)"""
    img_dir, ann = _coco(tmp_path, w=256, h=160)
    env = dict(os.environ, OUTPUTS_DIR=str(tmp_path / "out"), OMP_NUM_THREADS="4")
    base = str(PKG / "configs" / "rtdetrv2" / "rtdetrv2_r18vd_120e_coco.yml")
    common = ["--base-config", base, "--val-img-dir", str(img_dir), "--val-ann-json", str(ann), "--img-h", "160",
              "--img-w", "256", "--batch", "2", "--device", "cpu", "--workers", "0"]
    r = subprocess.run([sys.executable, str(PKG / "scripts/train_rtdetr_thirdparty.py"), "--train-img-dir",
                        str(img_dir), "--train-ann-json", str(ann), "--epochs", "1", "--run-name", "v2",
                        "--no-use-amp", *common], capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:] + r.stdout[-2000:]
    run = tmp_path / "out" / "runs" / "rtdetr_thirdparty" / "v2"
    ev = tmp_path / "out" / "eval" / "rtdetr_thirdparty" / "v2"
    for f in ("resolved_config.yml", "stdout.log", "stderr.log", "best.pth", "last.pth"):
        assert (run / f).exists(), f
    for f in ("train_summary.json", "train_summary.csv", "run_metadata.json", "run_metadata.csv",
              "train_adapter_result.json"):
        assert (ev / f).exists(), f
    assert json.loads((ev / "run_metadata.json").read_text())["model_family"] == "rtdetr_thirdparty"
    r = subprocess.run([sys.executable, str(PKG / "scripts/eval_rtdetr_thirdparty.py"), "--weights",
                        str(run / "best.pth"), "--run-name", "v2e", *common],
                       capture_output=True, text=True, env=env, timeout=600)
    assert r.returncode == 0, r.stderr[-3000:] + r.stdout[-2000:]
    ee = tmp_path / "out" / "eval" / "rtdetr_thirdparty" / "v2e"
    m = json.loads((ee / "metrics.json").read_text())
    assert m["split"] == "val" and m["speed_total_s_eval_run"] > 0
    for k in ("map50_95", "map50", "recall"):
        assert isinstance(m[k], float) and 0.0 <= m[k] <= 1.0, (k, m[k])
    assert set(json.loads((ee / "metrics_key.json").read_text())) == {"map50_95", "map50", "recall"}
    assert "Average Precision  (AP) @[ IoU=0.50:0.95" in (ee / "stdout_eval.log").read_text()
