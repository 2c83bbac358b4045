"""The real ZOD input path: ``YoloDataset`` / ``CocoDataset`` read exports in the
reference's on-disk format.

* Hand-written export (always runs): the layout and label syntax of
  /root/reference/src/data/exports.py:178-336 (``images/<split>/<frame_id>.jpg``,
  ``labels/<split>/<frame_id>.txt`` with ``class xc yc w h`` at 6 decimals, an
  empty file for a frame with no kept boxes, ``dataset.yaml`` written the way
  write_yolo_dataset_yaml does) plus the COCO json of
  /root/reference/scripts/export_coco_dataset.py:139-195
  (``annotations/instances_<split>.json``, ``images[].solar_context_bin`` as a
  bin label or null).
* Reference-written export (skips where /root/reference is absent): the
  reference's own ``export_yolo_split`` / ``write_yolo_dataset_yaml`` /
  ``export_coco_split`` run in a child process on a small frames table; both
  readers must return the same boxes and context ids from it.
"""
from __future__ import annotations

import json
import os
import subprocess
import sys
import textwrap
from pathlib import Path

import numpy as np
import pytest
import torch

REF = Path("/root/reference")

# content size of the exported (resized) frames and the padded network input
W, H = 96, 60
PAD_W, PAD_H = 96, 64

FRAMES = [  # frame_id, xyxy boxes (pixels), unclear flags, solar bin label
    ("000011", [[10.0, 5.0, 30.0, 45.0], [50.5, 10.25, 70.0, 40.0]], [False, False], "night(<-6)"),
    ("000023", [[0.0, 0.0, 12.0, 20.0], [40.0, 30.0, 60.0, 59.0]], [False, True], "high_sun(>45)"),
    ("000037", [], [], None),
    ("000042", [[80.0, 2.0, 95.0, 58.0]], [True], "low_sun(0..15)"),
]


def _write_jpg(path: Path, value: int):
    from PIL import Image

    path.parent.mkdir(parents=True, exist_ok=True)
    Image.fromarray(np.full((H, W, 3), value, np.uint8)).save(path, quality=95)


def _yolo_line(b):
    x1, y1, x2, y2 = b
    w, h = x2 - x1, y2 - y1
    return f"0 {(x1 + w / 2) / W:.6f} {(y1 + h / 2) / H:.6f} {w / W:.6f} {h / H:.6f}"


def _expected_boxes(boxes, unclear):
    """Kept boxes (exclude_unclear), cxcywh normalised to the padded tensor."""
    out = []
    for b, u in zip(boxes, unclear):
        if u:
            continue
        x1, y1, x2, y2 = b
        out.append([(x1 + x2) / 2 / PAD_W, (y1 + y2) / 2 / PAD_H, (x2 - x1) / PAD_W, (y2 - y1) / PAD_H])
    return np.asarray(out, np.float64).reshape(-1, 4)


def _hand_export(root: Path):
    split = "train"
    images, anns = [], []
    for i, (fid, boxes, unclear, ctx) in enumerate(FRAMES, start=1):
        _write_jpg(root / "images" / split / f"{fid}.jpg", 40 * i)
        lines = [_yolo_line(b) for b, u in zip(boxes, unclear) if not u]
        lp = root / "labels" / split / f"{fid}.txt"
        lp.parent.mkdir(parents=True, exist_ok=True)
        lp.write_text("\n".join(lines) + ("\n" if lines else ""))
        images.append({"id": i, "file_name": f"{fid}.jpg", "width": W, "height": H, "solar_context_bin": ctx})
        for b, u in zip(boxes, unclear):
            if not u:
                anns.append({"id": len(anns) + 1, "image_id": i, "category_id": 1,
                             "bbox": [b[0], b[1], b[2] - b[0], b[3] - b[1]], "area": 1.0, "iscrowd": 0})
    (root / "annotations").mkdir(parents=True, exist_ok=True)
    (root / "annotations" / f"instances_{split}.json").write_text(json.dumps(
        {"images": images, "annotations": anns,
         "categories": [{"id": 1, "name": "pedestrian", "supercategory": "person"}]}))
    (root / "dataset.yaml").write_text(
        f"path: {root.resolve()}\ntrain: images/train\nval: images/val\ntest: images/test\nnc: 1\nnames:\n  0: pedestrian\n")


def _check_yolo(root: Path):
    from src.moe.context import MISSING_ID, context_id_from_label
    from src.rtdetr_moe.data import YoloDataset, collate

    ds = YoloDataset(root / "dataset.yaml", split="train", imgsz=(H, W), pad_to=32)
    assert len(ds) == len(FRAMES) and ds.num_classes == 1
    assert (ds.pad_h, ds.pad_w) == (PAD_H, PAD_W)
    for i, (fid, boxes, unclear, ctx) in enumerate(FRAMES):
        img, t, cid = ds[i]
        assert ds.images[i].stem == fid
        assert img.shape == (3, PAD_H, PAD_W)
        assert torch.all(img[:, H:, :] == 0)  # bottom zero pad
        np.testing.assert_allclose(img[:, :H].mean().item(), 40 * (i + 1) / 255.0, atol=2 / 255)
        np.testing.assert_allclose(t["boxes"].numpy(), _expected_boxes(boxes, unclear), atol=2e-6)
        assert t["labels"].tolist() == [0] * len(t["boxes"])
        assert cid == (MISSING_ID if ctx is None else context_id_from_label(ctx))
        assert cid != MISSING_ID or ctx is None
    imgs, targets, ctx_ids = collate([ds[i] for i in range(len(ds))])
    assert imgs.shape == (4, 3, PAD_H, PAD_W) and ctx_ids.dtype == torch.int32
    assert [len(t["boxes"]) for t in targets] == [2, 1, 0, 0]
    return ds


def _check_coco_matches_yolo(root: Path, ds):
    from src.rtdetr_moe.data import CocoDataset

    cd = CocoDataset(root / "images" / "train", root / "annotations" / "instances_train.json", imgsz=(H, W))
    assert len(cd) == len(ds) and cd.num_classes == 1
    for i in range(len(ds)):
        a, ta, ca = ds[i]
        b, tb, cb = cd[i]
        torch.testing.assert_close(a, b)
        np.testing.assert_allclose(ta["boxes"].numpy(), tb["boxes"].numpy(), atol=2e-6)
        assert ta["labels"].tolist() == tb["labels"].tolist()  # category id 1 -> label 0
        assert ca == cb


def test_yolo_export_hand_written(tmp_path):
    _hand_export(tmp_path)
    ds = _check_yolo(tmp_path)
    _check_coco_matches_yolo(tmp_path, ds)


def test_yolo_export_missing_label_file_and_contexts_json(tmp_path):
    """A frame whose label file is absent has no boxes; ``contexts.json`` next to
    dataset.yaml supplies the bins when no COCO export is present."""
    from src.moe.context import MISSING_ID, context_id_from_label
    from src.rtdetr_moe.data import YoloDataset

    _hand_export(tmp_path)
    (tmp_path / "annotations" / "instances_train.json").unlink()
    (tmp_path / "labels" / "train" / "000011.txt").unlink()
    (tmp_path / "contexts.json").write_text(json.dumps({"000011": "twilight(-6..0)", "000042": None}))
    ds = YoloDataset(tmp_path / "dataset.yaml", split="train", imgsz=(H, W))
    _, t, c = ds[0]
    assert len(t["boxes"]) == 0 and c == context_id_from_label("twilight(-6..0)")
    assert ds[1][2] == MISSING_ID and ds[3][2] == MISSING_ID
    with pytest.raises(KeyError):
        YoloDataset(tmp_path / "dataset.yaml", split="calib")


_CHILD = textwrap.dedent("""
    import json, sys
    from pathlib import Path
    import numpy as np, pandas as pd
    out, frames = Path(sys.argv[1]), json.loads(sys.argv[2])
    from src.data.exports import export_yolo_split, write_yolo_dataset_yaml
    from scripts.export_coco_dataset import export_coco_split
    rows = [dict(frame_id=int(f), resized_image_path=str(out / "src" / f"{f}.jpg"),
                 xyxy_bboxes=np.asarray(b, np.float32).reshape(-1, 4), ped_unclear_list=u, new_w=W, new_h=H,
                 solar_context_bin=c) for f, b, u, c, W, H in frames]
    df = pd.DataFrame(rows)
    s1 = export_yolo_split("train", df, out)
    write_yolo_dataset_yaml(out, {0: "pedestrian"})
    s2 = export_coco_split(split_name="train", frames_df=df, out_dataset_dir=out)
    print(json.dumps([s1.n_boxes_written, s1.n_empty_label_files, s2.n_annotations_written]))
""")


@pytest.mark.skipif(not REF.exists(), reason="reference tree absent (GPU box)")
def test_reference_written_export(tmp_path):
    """The reference's own exporters write the dataset (child process with the
    reference root first on sys.path, nothing imported into this process); the
    build's readers return the same boxes and contexts from both formats."""
    for i, (fid, *_rest) in enumerate(FRAMES, start=1):
        _write_jpg(tmp_path / "src" / f"{fid}.jpg", 40 * i)
    frames = [[fid, b, u, c, W, H] for fid, b, u, c in FRAMES]
    env = dict(os.environ, PYTHONPATH=str(REF), PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-c", _CHILD, str(tmp_path), json.dumps(frames)], cwd=str(REF), env=env,
                       capture_output=True, text=True, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    n_boxes, n_empty, n_ann = json.loads(r.stdout.strip().splitlines()[-1])
    assert (n_boxes, n_empty, n_ann) == (3, 2, 3)
    ds = _check_yolo(tmp_path)
    _check_coco_matches_yolo(tmp_path, ds)
