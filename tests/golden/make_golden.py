"""Generate the reference-pinned golden vectors (run in the build container only).

Runs the REFERENCE's own code from /root/reference (read-only, in a child
process with the reference on sys.path, so nothing of it is copied here) and
stores its outputs as data:

  tests/golden/reference_known_answers.json
    solar_bins    : per-row labels written by scripts/add_solar_context_bins.py
                    (its main(), on a temp parquet of probe angles)
    frequency     : scripts/analyze_context_frequencies.py::_build_frequency_table
                    solar rows for the same probe angles
    bboxes        : src/data/bboxes.py points_to_xyxy / xyxy_to_yolo /
                    clamp_xyxy / is_valid_box on probe boxes
    metrics_json  : src/models/vision/yolo.py::save_yolo_metrics_json of a stub
                    metrics object + scripts/eval_detector.py::
                    _add_derived_speed_metrics
    train_summary : src/models/vision/yolo.py::save_yolo_training_summary of a
                    stub results object; save_metrics_table_csv text
  multimodal-moe_amd/src/rtdetr_moe/zod_ped_box_wh.npy
    4096 (w, h) pedestrian box sizes (original 3848x2168 px) sampled with seed 0
    from notebooks/outputs/analysis/ped_box_wh.parquet (43,790 boxes), for the
    synthetic ZOD-shaped targets of SURVEY.md 8(d).

Usage:  python tests/golden/make_golden.py
"""
from __future__ import annotations

import json
import math
import subprocess
import sys
import tempfile
from pathlib import Path

import numpy as np

REF = Path("/root/reference")
HERE = Path(__file__).resolve().parent
ROOT = HERE.parents[1]

PROBE_ANGLES = [-90.0, -6.000001, -6.0, -5.999, -3.0, 0.0, 0.001, 7.5, 15.0, 15.0001, 30.0, 45.0,
                45.0001, 60.0, 89.9, float("nan"), -1e9, 1e9]

CHILD = r'''
import json, sys, math, tempfile, subprocess, types
from pathlib import Path
import numpy as np
import pandas as pd
sys.path.insert(0, "/root/reference")
from src.data import bboxes as B
from src.models.vision import yolo as Y
from scripts.analyze_context_frequencies import _build_frequency_table
from scripts.eval_detector import _add_derived_speed_metrics

angles = json.loads(sys.argv[1])
out = {}
with tempfile.TemporaryDirectory() as td:
    inp = Path(td) / "in.parquet"; outp = Path(td) / "out.parquet"
    pd.DataFrame({"solar_angle_elevation": [a if a is not None else float("nan") for a in angles]}).to_parquet(inp)
    subprocess.run([sys.executable, "/root/reference/scripts/add_solar_context_bins.py",
                    "--in-parquet", str(inp), "--out-parquet", str(outp)], check=True,
                   capture_output=True, env={"PYTHONDONTWRITEBYTECODE": "1", "PATH": "/usr/bin:/bin",
                                             "OUTPUTS_DIR": td})
    out["solar_bins"] = [str(v) for v in pd.read_parquet(outp)["solar_context_bin"].tolist()]
df = pd.DataFrame({"solar_angle_elevation": angles, "scraped_weather": "x", "time_of_day": "day",
                   "road_type": "city", "road_condition": "normal"})
ft = _build_frequency_table(df)
ft = ft[ft["field"] == "solar_context_bin"]
out["frequency"] = {r.category: int(r["count"]) for _, r in ft.iterrows()}

pts = [[522.21405, 357.98141], [523.92322, 361.11176], [522.4378, 367.88547], [520.35565, 361.11176]]
xyxy = B.points_to_xyxy(pts)
boxes = [[-3, 5, 1300, 800], [10.5, 20.25, 30.0, 44.0], [0, 0, 1.5, 10], [1247.9, 703.2, 1250, 705]]
out["bboxes"] = {
    "points": pts, "points_to_xyxy": xyxy,
    "xyxy_to_yolo_1248x704": B.xyxy_to_yolo(xyxy, 1248, 704),
    "is_valid": B.is_valid_box(xyxy),
    "probe_boxes": boxes,
    "clamp_1248x704": [B.clamp_xyxy(b, 1248, 704) for b in boxes],
    "yolo_1248x704": [B.xyxy_to_yolo(b, 1248, 704) for b in boxes],
    "is_valid_probe": [bool(B.is_valid_box(b)) for b in boxes],
    "degenerate_points_to_xyxy": B.points_to_xyxy([[1.0, 1.0], [1.0, 5.0]]),
}

class _Box: pass
box = _Box(); box.map50 = 0.5; box.map = 0.25; box.mp = 0.6; box.mr = 0.4
box.curves = ["Precision-Recall(B)", "F1-Confidence(B)"]
box.curves_results = [[np.linspace(0, 1, 5), np.array([[1.0, 0.8, 0.6, 0.4, 0.2]])],
                      [np.linspace(0, 1, 3), np.array([[0.1, 0.5, 0.3]])]]
class _Net:
    def parameters(self):
        import torch
        return [torch.nn.Parameter(torch.zeros(10, 3)), torch.nn.Parameter(torch.zeros(5), requires_grad=False)]
    flops = 12.5
class _Wrap: pass
wrap = _Wrap(); wrap.model = _Net()
class _M: pass
m = _M()
m.results_dict = {"metrics/mAP50(B)": 0.5, "metrics/mAP50-95(B)": 0.25, "metrics/precision(B)": 0.6,
                  "metrics/recall(B)": 0.4, "fitness": 0.3}
m.speed = {"preprocess": 1.0, "inference": 4.0, "postprocess": 0.5}
m.box = box
m.model = wrap
with tempfile.TemporaryDirectory() as td:
    p = Y.save_yolo_metrics_json(m, Path(td) / "metrics.json")
    d = json.loads(p.read_text())
    d = _add_derived_speed_metrics(d)
    out["metrics_json"] = d
    out["metrics_json_keys"] = list(d.keys())
    m2 = _M(); m2.box = box  # no results_dict -> box fallback
    out["metrics_json_box_fallback"] = json.loads(Y.save_yolo_metrics_json(m2, Path(td) / "m2.json").read_text())
    res = _M(); res.model = wrap
    js, cs = Y.save_yolo_training_summary(train_wall_time_s=12.5, model_name="rtdetr-r50-moe8-top2",
                                          data_yaml="d.yaml", run_name="r", out_json_path=Path(td) / "s.json",
                                          out_csv_path=Path(td) / "s.csv", results=res)
    out["train_summary"] = json.loads(js.read_text())
    out["train_summary_csv"] = cs.read_text()
    out["infer_model_variant"] = {w: Y.infer_model_variant_from_weights(w)
                                  for w in ["yolo26n.pt", "runs/x/weights/best.pt", "rtdetr-r50-moe8-top2"]}
print(json.dumps(out))
'''


def main() -> None:
    if not REF.exists():
        raise SystemExit("needs /root/reference (build container only)")
    angles = [None if (isinstance(a, float) and math.isnan(a)) else a for a in PROBE_ANGLES]
    res = subprocess.run([sys.executable, "-c", CHILD, json.dumps(angles)], capture_output=True, text=True,
                         cwd=tempfile.gettempdir(), env={"PYTHONDONTWRITEBYTECODE": "1", "PATH": "/usr/bin:/bin",
                                                         "HOME": "/tmp"})
    if res.returncode != 0:
        raise SystemExit(res.stderr)
    out = json.loads(res.stdout.strip().splitlines()[-1])
    out["probe_angles"] = angles
    out["source"] = "scaleoutsystems/multimodal-MoE @2026-02-20 (/root/reference), generated by tests/golden/make_golden.py"
    (HERE / "reference_known_answers.json").write_text(json.dumps(out, indent=1))

    import pandas as pd

    df = pd.read_parquet(REF / "notebooks/outputs/analysis/ped_box_wh.parquet")
    rng = np.random.default_rng(0)
    sel = rng.choice(len(df), size=4096, replace=False)
    wh = df[["bbox_w", "bbox_h"]].to_numpy(np.float32)[sel]
    np.save(ROOT / "multimodal-moe_amd/src/rtdetr_moe/zod_ped_box_wh.npy", wh)
    print("wrote", HERE / "reference_known_answers.json", "and zod_ped_box_wh.npy", wh.shape)


if __name__ == "__main__":
    main()
