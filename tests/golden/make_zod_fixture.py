"""Write tests/golden/zod_mini/: a six-frame ZOD-format dataset at the
reference's native 1248x704 size, exported by the REFERENCE's own exporters
(run in the build container only; the output is data and travels to the GPU
box, the reference does not).

  frames/<id>.jpg            synthetic 1248x704 frames (this script, PIL)
  images/{train,val}/<id>.jpg  relative symlinks written by
                             /root/reference/src/data/exports.py:178
                             export_yolo_split (and the COCO exporter)
  labels/{train,val}/<id>.txt  YOLO labels, same exporter (unclear boxes
                             excluded, an empty file for a frame without kept
                             boxes)
  dataset.yaml               /root/reference/src/data/exports.py:295
                             write_yolo_dataset_yaml
  annotations/instances_{train,val}.json
                             /root/reference/scripts/export_coco_dataset.py:93
                             export_coco_split, images[].solar_context_bin
                             (the router context, :146-148)
  expected.json              frame ids, splits, context labels and the
                             exporters' summary counts (for the tests)

Geometry (notes/experiment_protocol_camera.md:25): 1248x704 -- the S5 grid is
22x39 = 858 tokens, the deformable-attention levels 88x156 / 44x78 / 22x39.
The exporter is handed relative image paths, so its symlinks are relative and
the fixture is relocatable.  dataset.yaml keeps the absolute ``path:`` the
reference writes (/root/repo/tests/golden/zod_mini, valid on the GPU box too);
the build's YoloDataset falls back to the yaml's directory when it is absent.

Usage:  python tests/golden/make_zod_fixture.py
"""
from __future__ import annotations

import json
import os
import shutil
import subprocess
import sys
import textwrap
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
OUT = Path(__file__).resolve().parent / "zod_mini"
W, H = 1248, 704

# frame_id, split, xyxy boxes (pixels of the 1248x704 frame), unclear flags, solar bin label
FRAMES = [
    ("000101", "train", [[100.0, 300.0, 130.0, 390.0], [600.5, 280.25, 640.0, 400.0], [900.0, 310.0, 915.0, 352.0]],
     [False, False, True], "night(<-6)"),
    ("000102", "train", [[0.0, 250.0, 40.0, 420.0], [1200.0, 300.0, 1260.0, 460.0]], [False, False],
     "mid_sun(15..45)"),
    ("000103", "train", [[500.0, 330.0, 520.0, 380.0]], [False], "high_sun(>45)"),
    ("000104", "train", [[300.0, 320.0, 330.0, 400.0], [700.0, 100.0, 760.0, 300.0]], [True, False], None),
    ("000201", "val", [[410.0, 300.0, 450.0, 410.0], [800.0, 290.0, 830.0, 370.0]], [False, False],
     "low_sun(0..15)"),
    ("000202", "val", [], [], "twilight(-6..0)"),
]

CHILD = textwrap.dedent("""
    import json, os, sys
    from pathlib import Path
    import numpy as np, pandas as pd
    out, frames = Path(sys.argv[1]), json.loads(sys.argv[2])
    from src.data.exports import export_yolo_split, write_yolo_dataset_yaml
    from scripts.export_coco_dataset import export_coco_split
    summary = {}
    for split in ("train", "val"):
        rows = [dict(frame_id=int(f), resized_image_path=f"../../frames/{f}.jpg",
                     xyxy_bboxes=np.asarray(b, np.float32).reshape(-1, 4), ped_unclear_list=u, new_w=W, new_h=H,
                     solar_context_bin=c) for f, s, b, u, c, W, H in frames if s == split]
        df = pd.DataFrame(rows)
        (out / "images" / split).mkdir(parents=True, exist_ok=True)
        os.chdir(out / "images" / split)  # the relative image paths resolve from here (and so do the symlinks)
        y = export_yolo_split(split, df, out)
        c = export_coco_split(split_name=split, frames_df=df, out_dataset_dir=out)
        summary[split] = dict(yolo_boxes=y.n_boxes_written, yolo_empty=y.n_empty_label_files,
                              yolo_dropped_unclear=y.n_boxes_dropped_unclear, coco_annotations=c.n_annotations_written,
                              images=y.n_images_written)
    write_yolo_dataset_yaml(out, {0: "pedestrian"})
    print(json.dumps(summary))
""")


def _frame(seed: int) -> np.ndarray:
    """A smooth road-scene-like frame (gradient sky / road, a few blocks):
    compresses to a few tens of KB."""
    rng = np.random.default_rng(seed)
    y = np.linspace(0.0, 1.0, H)[:, None, None]
    x = np.linspace(0.0, 1.0, W)[None, :, None]
    base = np.concatenate([0.5 + 0.4 * (1 - y) + 0 * x, 0.45 + 0.3 * (1 - y) + 0.05 * x, 0.4 + 0.2 * y + 0 * x], 2)
    img = np.broadcast_to(base, (H, W, 3)).copy()
    for _ in range(6):
        x0, y0 = int(rng.integers(0, W - 120)), int(rng.integers(H // 3, H - 80))
        img[y0:y0 + int(rng.integers(20, 80)), x0:x0 + int(rng.integers(20, 120))] = rng.uniform(0.1, 0.9, 3)
    return (np.clip(img, 0, 1) * 255).astype(np.uint8)


def main():
    from PIL import Image

    if not REF.exists():
        raise SystemExit("the reference tree /root/reference is needed to write this fixture")
    if OUT.exists():
        shutil.rmtree(OUT)
    (OUT / "frames").mkdir(parents=True)
    for i, (fid, *_rest) in enumerate(FRAMES):
        Image.fromarray(_frame(i)).save(OUT / "frames" / f"{fid}.jpg", quality=80)
    frames = [[fid, s, b, u, c, W, H] for fid, s, b, u, c in FRAMES]
    env = dict(os.environ, PYTHONPATH=str(REF), PYTHONDONTWRITEBYTECODE="1")
    r = subprocess.run([sys.executable, "-c", CHILD, str(OUT), json.dumps(frames)], cwd=str(REF), env=env,
                       capture_output=True, text=True, timeout=300)
    if r.returncode != 0:
        raise SystemExit(r.stderr[-3000:])
    summary = json.loads(r.stdout.strip().splitlines()[-1])
    expected = {"img_w": W, "img_h": H, "summary": summary,
                "frames": [{"frame_id": fid, "split": s, "solar_context_bin": c} for fid, s, _b, _u, c in FRAMES]}
    (OUT / "expected.json").write_text(json.dumps(expected, indent=1) + "\n")
    print(json.dumps(summary))


if __name__ == "__main__":
    main()
