"""Project paths, each overridable by an environment variable of the same
name (the reference's idiom, src/paths.py:5-41).  Defaults are relative to
this package so runs stay inside the checkout."""
from __future__ import annotations

import os
from pathlib import Path

PROJECT_ROOT = Path(__file__).resolve().parents[1]


def env_path(var: str, default) -> Path:
    return Path(os.environ.get(var, str(default))).expanduser().resolve()


ZOD_MOE_DATA = env_path("ZOD_MOE_DATA", "~/zod_moe")
RESIZED_IMAGES_DIR = env_path("RESIZED_IMAGES_DIR", ZOD_MOE_DATA / "resized_images")
SPLITS_DIR = env_path("SPLITS_DIR", ZOD_MOE_DATA / "splits")
OUTPUTS_DIR = env_path("OUTPUTS_DIR", PROJECT_ROOT / "outputs")
INDEX_DIR = env_path("INDEX_DIR", OUTPUTS_DIR / "index")
EXPORTS_DIR = env_path("EXPORTS_DIR", OUTPUTS_DIR / "exports")
RUNS_DIR = env_path("RUNS_DIR", OUTPUTS_DIR / "runs")
EVAL_DIR = env_path("EVAL_DIR", OUTPUTS_DIR / "eval")
