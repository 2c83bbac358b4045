"""Detection inputs for the RT-DETR-MoE engine.

* ``SyntheticZOD``: ZOD-shaped synthetic batches -- images
  uniform in [0,1] (the reference feeds /255 tensors, src/data/zodmoe_frames.py:
  156-160), 1280x720 content bottom-padded to 736; 0 pedestrians with p=0.4242
  else 1+Poisson(4.533) (mean 3.186 per frame, notebooks/zod_frames_index_sanity
  cells 6-7); box sizes resampled from 4096 real ZOD pedestrian boxes
  (zod_ped_box_wh.npy, made by tests/golden/make_golden.py from
  notebooks/outputs/analysis/ped_box_wh.parquet); per-image solar context drawn
  with the ZOD bin frequencies (context_field_frequencies_final.csv:22-26).
* ``YoloDataset``: the Ultralytics export the reference writes
  (src/data/exports.py: dataset.yaml + images/ + labels/*.txt with
  ``class xc yc w h``), plus an optional per-image ``solar_context_bin`` taken
  from a COCO export (scripts/export_coco_dataset.py:146-148) or a
  ``contexts.json`` {image stem: bin label} next to dataset.yaml.
* ``CocoDataset``: the COCO export (scripts/export_coco_dataset.py:120-195:
  ``images[]`` with ``file_name`` and ``solar_context_bin``, ``annotations[]``
  with pixel ``bbox`` [x, y, w, h] and ``category_id``), the input of the
  RT-DETRv2 adapter (src/models/vision/rtdetr_thirdparty.py:81-108
  img_folder + ann_file).  Category ids map to contiguous labels in id order
  (the export's single pedestrian id 1 -> label 0).
Box helpers restate src/data/bboxes.py (clamp to [0,W-1]x[0,H-1], min 2 px).
"""
from __future__ import annotations

import json
import math
from pathlib import Path

import numpy as np
import torch

from ..moe.context import MISSING_ID, SOLAR_FREQUENCIES, context_id_from_label

_WH_FILE = Path(__file__).resolve().parent / "zod_ped_box_wh.npy"
ZOD_ORIG_W, ZOD_ORIG_H = 3848, 2168


# ---------------------------------------------------------------------------
# box helpers (semantics of the reference's src/data/bboxes.py)
# ---------------------------------------------------------------------------
def clamp_xyxy(box, img_w=1248, img_h=704):
    x1, y1, x2, y2 = box
    cx = lambda v: max(0.0, min(v, img_w - 1))  # noqa: E731
    cy = lambda v: max(0.0, min(v, img_h - 1))  # noqa: E731
    return [cx(x1), cy(y1), cx(x2), cy(y2)]


def xyxy_to_yolo(box, img_w=1248, img_h=704):
    x1, y1, x2, y2 = box
    w, h = x2 - x1, y2 - y1
    return [(x1 + w / 2.0) / img_w, (y1 + h / 2.0) / img_h, w / img_w, h / img_h]


def is_valid_box(box, min_size=2.0):
    return (box[2] - box[0]) >= min_size and (box[3] - box[1]) >= min_size


# ---------------------------------------------------------------------------
# synthetic ZOD-shaped batches
# ---------------------------------------------------------------------------
class SyntheticZOD:
    P_EMPTY = 0.4242
    POISSON_MEAN = 4.533
    MAX_BOXES = 127

    def __init__(self, batch=8, img_h=720, img_w=1280, pad_to=32, seed=0, single_context=None,
                 num_classes=1):
        self.batch = batch
        self.img_h, self.img_w = img_h, img_w
        self.pad_h = int(math.ceil(img_h / pad_to) * pad_to)
        self.pad_w = int(math.ceil(img_w / pad_to) * pad_to)
        self.rng = np.random.default_rng(seed)
        self.gen = torch.Generator().manual_seed(seed)
        self.single_context = single_context
        self.num_classes = num_classes
        self.wh = np.load(_WH_FILE) if _WH_FILE.exists() else np.array([[31.0, 84.0]], np.float32)

    def _targets(self):
        targets = []
        sx, sy = self.img_w / ZOD_ORIG_W, self.img_h / ZOD_ORIG_H
        for _ in range(self.batch):
            n = 0 if self.rng.random() < self.P_EMPTY else min(1 + self.rng.poisson(self.POISSON_MEAN), self.MAX_BOXES)
            boxes = []
            for _ in range(n):
                w, h = self.wh[self.rng.integers(len(self.wh))]
                w, h = float(w) * sx, float(h) * sy
                cx = self.rng.uniform(0, self.img_w)
                cy = self.rng.uniform(0, self.img_h)
                b = clamp_xyxy([cx - w / 2, cy - h / 2, cx + w / 2, cy + h / 2], self.img_w, self.img_h)
                if not is_valid_box(b, 1.0):
                    continue
                # normalised to the padded input tensor (content occupies the top img_h rows)
                boxes.append(xyxy_to_yolo(b, self.pad_w, self.pad_h))
            bt = torch.tensor(boxes, dtype=torch.float32).reshape(-1, 4)
            targets.append({"boxes": bt, "labels": torch.zeros(len(bt), dtype=torch.int64)})
        return targets

    def _contexts(self):
        if self.single_context is not None:
            return torch.full((self.batch,), int(self.single_context), dtype=torch.int32)
        p = np.asarray(SOLAR_FREQUENCIES, np.float64)
        return torch.as_tensor(self.rng.choice(len(p), size=self.batch, p=p / p.sum()), dtype=torch.int32)

    def sample(self, device="cpu", dtype=torch.float32):
        """One batch: images [B,3,pad_h,pad_w] (bottom/right zero pad), targets, ctx ids."""
        img = torch.zeros((self.batch, 3, self.pad_h, self.pad_w), dtype=dtype)
        img[:, :, : self.img_h, : self.img_w] = torch.rand((self.batch, 3, self.img_h, self.img_w),
                                                          generator=self.gen).to(dtype)
        return img.to(device), self._targets(), self._contexts().to(device)

    def __iter__(self):
        while True:
            yield self.sample()


# ---------------------------------------------------------------------------
# Ultralytics-format dataset (what the reference exports)
# ---------------------------------------------------------------------------
_IMG_EXT = {".jpg", ".jpeg", ".png", ".bmp"}


def _read_yaml(path: Path) -> dict:
    import yaml

    with open(path) as f:
        return yaml.safe_load(f) or {}


class YoloDataset(torch.utils.data.Dataset):
    def __init__(self, data_yaml: str | Path, split="train", imgsz=(704, 1248), pad_to=32):
        self.yaml_path = Path(data_yaml)
        cfg = _read_yaml(self.yaml_path)
        root = Path(cfg.get("path", self.yaml_path.parent))
        if not root.is_absolute():
            root = (self.yaml_path.parent / root).resolve()
        if not root.exists():  # an export moved since write_yolo_dataset_yaml wrote its absolute path
            root = self.yaml_path.parent.resolve()
        rel = cfg.get(split)
        if rel is None:
            raise KeyError(f"split {split!r} missing in {data_yaml}")
        img_dir = Path(rel) if Path(rel).is_absolute() else root / rel
        self.names = cfg.get("names", {0: "pedestrian"})
        self.num_classes = len(self.names)
        self.images = sorted(p for p in img_dir.rglob("*") if p.suffix.lower() in _IMG_EXT)
        self.h, self.w = (imgsz, imgsz) if isinstance(imgsz, int) else imgsz
        self.pad_h = int(math.ceil(self.h / pad_to) * pad_to)
        self.pad_w = int(math.ceil(self.w / pad_to) * pad_to)
        self.contexts = self._load_contexts(root)

    def _load_contexts(self, root: Path) -> dict:
        ctx = {}
        side = self.yaml_path.parent / "contexts.json"
        if side.exists():
            ctx.update({str(k): context_id_from_label(v) for k, v in json.loads(side.read_text()).items()})
        for coco in list(root.glob("*.json")) + list((root / "annotations").glob("*.json")):
            try:
                d = json.loads(coco.read_text())
                for im in d.get("images", []):
                    if "solar_context_bin" in im:
                        ctx[Path(im.get("file_name", "")).stem] = context_id_from_label(im["solar_context_bin"])
            except Exception:
                continue
        return ctx

    def __len__(self):
        return len(self.images)

    def _label_path(self, img: Path) -> Path:
        parts = list(img.parts)
        if "images" in parts:
            i = len(parts) - 1 - parts[::-1].index("images")
            parts[i] = "labels"
        return Path(*parts).with_suffix(".txt")

    def __getitem__(self, i):
        from PIL import Image

        p = self.images[i]
        im = Image.open(p).convert("RGB").resize((self.w, self.h), Image.BILINEAR)
        arr = torch.from_numpy(np.asarray(im, dtype=np.uint8).copy()).permute(2, 0, 1).float() / 255.0
        img = torch.zeros((3, self.pad_h, self.pad_w))
        img[:, : self.h, : self.w] = arr
        boxes, labels = [], []
        lp = self._label_path(p)
        if lp.exists():
            for line in lp.read_text().splitlines():
                v = line.split()
                if len(v) != 5:
                    continue
                c, xc, yc, w, h = int(v[0]), *map(float, v[1:])
                # rescale normalised coords from the content area to the padded tensor
                boxes.append([xc * self.w / self.pad_w, yc * self.h / self.pad_h, w * self.w / self.pad_w,
                              h * self.h / self.pad_h])
                labels.append(c)
        t = {"boxes": torch.tensor(boxes, dtype=torch.float32).reshape(-1, 4),
             "labels": torch.tensor(labels, dtype=torch.int64), "orig_size": (self.pad_w, self.pad_h)}
        return img, t, self.contexts.get(p.stem, MISSING_ID)


class CocoDataset(torch.utils.data.Dataset):
    def __init__(self, img_folder: str | Path, ann_file: str | Path, imgsz=(704, 1248), pad_to=32):
        self.img_folder = Path(img_folder)
        d = json.loads(Path(ann_file).read_text())
        cats = sorted(int(c["id"]) for c in d.get("categories", []))
        if not cats:
            cats = sorted({int(a["category_id"]) for a in d.get("annotations", [])}) or [1]
        self.cat_to_label = {c: i for i, c in enumerate(cats)}
        self.num_classes = len(cats)
        self.images = sorted(d.get("images", []), key=lambda im: im["id"])
        self.anns = {im["id"]: [] for im in self.images}
        for a in d.get("annotations", []):
            if a.get("iscrowd", 0) or a["image_id"] not in self.anns:
                continue
            self.anns[a["image_id"]].append(a)
        self.h, self.w = (imgsz, imgsz) if isinstance(imgsz, int) else imgsz
        self.pad_h = int(math.ceil(self.h / pad_to) * pad_to)
        self.pad_w = int(math.ceil(self.w / pad_to) * pad_to)

    def __len__(self):
        return len(self.images)

    def __getitem__(self, i):
        from PIL import Image

        im = self.images[i]
        pil = Image.open(self.img_folder / im["file_name"]).convert("RGB")
        ow, oh = int(im.get("width", pil.width)), int(im.get("height", pil.height))
        pil = pil.resize((self.w, self.h), Image.BILINEAR)
        arr = torch.from_numpy(np.asarray(pil, dtype=np.uint8).copy()).permute(2, 0, 1).float() / 255.0
        img = torch.zeros((3, self.pad_h, self.pad_w))
        img[:, : self.h, : self.w] = arr
        boxes, labels = [], []
        for a in self.anns[im["id"]]:
            x, y, w, h = map(float, a["bbox"])
            x0, y0 = max(x, 0.0), max(y, 0.0)  # SanitizeBoundingBoxes: clip, drop < 1 px
            x1, y1 = min(x + w, ow), min(y + h, oh)
            if x1 - x0 < 1 or y1 - y0 < 1:
                continue
            # normalised to the content area, then rescaled to the padded tensor
            boxes.append([(x0 + x1) / 2 / ow * self.w / self.pad_w, (y0 + y1) / 2 / oh * self.h / self.pad_h,
                          (x1 - x0) / ow * self.w / self.pad_w, (y1 - y0) / oh * self.h / self.pad_h])
            labels.append(self.cat_to_label[int(a["category_id"])])
        t = {"boxes": torch.tensor(boxes, dtype=torch.float32).reshape(-1, 4),
             "labels": torch.tensor(labels, dtype=torch.int64), "orig_size": (self.pad_w, self.pad_h)}
        ctx = im.get("solar_context_bin")
        return img, t, MISSING_ID if ctx is None else context_id_from_label(ctx)


def collate(batch):
    imgs = torch.stack([b[0] for b in batch])
    targets = [b[1] for b in batch]
    ctx = torch.tensor([b[2] for b in batch], dtype=torch.int32)
    return imgs, targets, ctx
