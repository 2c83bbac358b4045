"""Per-image router context.

The context id is the reference's solar-elevation bin
(scripts/add_solar_context_bins.py:87-107: pd.cut with bins
[-1e9, -6, 0, 15, 45, 1e9], right-closed, include_lowest, NaN -> "missing"),
carried per image in the COCO export as ``images[].solar_context_bin``
(scripts/export_coco_dataset.py:146-148).  The router sees it as an integer
``ctx_id`` per image that selects a row of the additive logit bias.
"""
from __future__ import annotations

import math

import numpy as np

SOLAR_EDGES = (-1e9, -6.0, 0.0, 15.0, 45.0, 1e9)
SOLAR_LABELS = (
    "night(<-6)",
    "twilight(-6..0)",
    "low_sun(0..15)",
    "mid_sun(15..45)",
    "high_sun(>45)",
)
CONTEXT_LABELS = SOLAR_LABELS + ("missing",)
NUM_CONTEXTS = len(CONTEXT_LABELS)
MISSING_ID = NUM_CONTEXTS - 1
# ZOD frame frequencies of the five solar bins
# (outputs/analysis/camera/detection/context_field_frequencies_final.csv:22-26)
SOLAR_FREQUENCIES = (0.19006, 0.03647, 0.16332, 0.41417, 0.19597)


def solar_context_ids(angles) -> np.ndarray:
    """Vectorised bin ids (0..4, 5 = missing) of solar elevation angles (deg)."""
    a = np.asarray(angles, dtype=np.float64).reshape(-1)
    out = np.full(a.shape, MISSING_ID, dtype=np.int32)
    ok = np.isfinite(a) & (a >= SOLAR_EDGES[0]) & (a <= SOLAR_EDGES[-1])
    # right-closed bins: id = number of interior edges strictly below a
    interior = np.asarray(SOLAR_EDGES[1:-1])
    ids = np.searchsorted(interior, a[ok], side="left").astype(np.int32)
    out[ok] = ids
    return out


def solar_context_id(angle) -> int:
    try:
        a = float(angle)
    except (TypeError, ValueError):
        return MISSING_ID
    if math.isnan(a):
        return MISSING_ID
    return int(solar_context_ids([a])[0])


def context_id_from_label(label) -> int:
    """Map a ``solar_context_bin`` string (parquet / COCO export) to its id."""
    if label is None:
        return MISSING_ID
    s = str(label)
    return CONTEXT_LABELS.index(s) if s in CONTEXT_LABELS else MISSING_ID
