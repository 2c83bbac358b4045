"""Product code vs golden vectors produced by the REFERENCE itself
(tests/golden/reference_known_answers.json, written by tests/golden/make_golden.py
from /root/reference).  CPU only."""
from __future__ import annotations

import json
import math
import types
from pathlib import Path

import numpy as np
import pytest

GOLD = json.loads((Path(__file__).parent / "golden" / "reference_known_answers.json").read_text())


def test_solar_context_bins_match_reference():
    from src.moe.context import CONTEXT_LABELS, solar_context_id, solar_context_ids
    from oracle import moe_oracle as O

    angles = [float("nan") if a is None else a for a in GOLD["probe_angles"]]
    ref = GOLD["solar_bins"]
    assert [CONTEXT_LABELS[i] for i in solar_context_ids(angles)] == ref
    assert [CONTEXT_LABELS[solar_context_id(a)] for a in angles] == ref
    assert [O.solar_context_bin(a) for a in angles] == ref  # oracle pinned too


def test_frequency_table_counts_match_reference():
    from src.moe.context import CONTEXT_LABELS, solar_context_ids

    angles = [float("nan") if a is None else a for a in GOLD["probe_angles"]]
    ids = solar_context_ids(angles)
    counts = {CONTEXT_LABELS[i]: int((ids == i).sum()) for i in set(ids.tolist())}
    assert counts == GOLD["frequency"]


def test_box_helpers_match_reference():
    from src.rtdetr_moe.data import clamp_xyxy, is_valid_box, xyxy_to_yolo

    b = GOLD["bboxes"]
    for box, cl, yo, ok in zip(b["probe_boxes"], b["clamp_1248x704"], b["yolo_1248x704"], b["is_valid_probe"]):
        assert clamp_xyxy(box, 1248, 704) == pytest.approx(cl)
        assert xyxy_to_yolo(box, 1248, 704) == pytest.approx(yo)
        assert is_valid_box(box) == ok
    assert xyxy_to_yolo(b["points_to_xyxy"], 1248, 704) == pytest.approx(b["xyxy_to_yolo_1248x704"])


def _stub_metrics():
    box = types.SimpleNamespace(map50=0.5, map=0.25, mp=0.6, mr=0.4,
                                curves=["Precision-Recall(B)", "F1-Confidence(B)"],
                                curves_results=[[np.linspace(0, 1, 5), np.array([[1.0, 0.8, 0.6, 0.4, 0.2]])],
                                                [np.linspace(0, 1, 3), np.array([[0.1, 0.5, 0.3]])]])

    class _Net:
        def parameters(self):
            import torch

            return [torch.nn.Parameter(torch.zeros(10, 3)), torch.nn.Parameter(torch.zeros(5), requires_grad=False)]

        flops = 12.5

    m = types.SimpleNamespace(
        results_dict={"metrics/mAP50(B)": 0.5, "metrics/mAP50-95(B)": 0.25, "metrics/precision(B)": 0.6,
                      "metrics/recall(B)": 0.4, "fitness": 0.3},
        speed={"preprocess": 1.0, "inference": 4.0, "postprocess": 0.5}, box=box,
        model=types.SimpleNamespace(model=_Net()))
    return m, box, _Net


def test_metrics_json_schema_matches_reference(tmp_path):
    import importlib.util
    from src.models.vision.rtdetr import save_rtdetr_metrics_json

    spec = importlib.util.spec_from_file_location(
        "eval_detector_build", Path(__file__).resolve().parents[1] / "multimodal-moe_amd/scripts/eval_detector.py")
    ev = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(ev)
    m, box, _ = _stub_metrics()
    p = save_rtdetr_metrics_json(m, tmp_path / "metrics.json")
    d = ev._add_derived_speed_metrics(json.loads(p.read_text()))
    assert list(d.keys()) == GOLD["metrics_json_keys"]
    assert json.loads(json.dumps(d)) == GOLD["metrics_json"]
    fb = json.loads(save_rtdetr_metrics_json(types.SimpleNamespace(box=box), tmp_path / "m2.json").read_text())
    assert fb == GOLD["metrics_json_box_fallback"]


def test_training_summary_matches_reference(tmp_path):
    from src.models.vision.rtdetr import infer_model_variant_from_weights, save_rtdetr_training_summary

    m, _, _Net = _stub_metrics()
    js, cs = save_rtdetr_training_summary(train_wall_time_s=12.5, model_name="rtdetr-r50-moe8-top2",
                                          data_yaml="d.yaml", run_name="r", out_json_path=tmp_path / "s.json",
                                          out_csv_path=tmp_path / "s.csv",
                                          results=types.SimpleNamespace(model=types.SimpleNamespace(model=_Net())))
    assert json.loads(js.read_text()) == GOLD["train_summary"]
    assert cs.read_text() == GOLD["train_summary_csv"]
    for w, v in GOLD["infer_model_variant"].items():
        assert infer_model_variant_from_weights(w) == v
