"""Build libmoe_hip.so (gfx950) in-tree: one hipcc -c per .hip, then link.

Used by __graft_entry__.build() and by hand: ``python multimodal-moe_amd/build_ext.py``.
The .so lands in multimodal-moe_amd/lib/ (git-ignored, travels with gpurun).
"""
from __future__ import annotations

import concurrent.futures as cf
import os
import shutil
import subprocess
import sys
from pathlib import Path

PKG = Path(__file__).resolve().parent
CSRC = PKG / "csrc"
LIB_DIR = PKG / "lib"
LIB = LIB_DIR / "libmoe_hip.so"
OBJ_DIR = PKG / "build" / "obj"
ARCH = os.environ.get("MOE_HIP_ARCH", "gfx950")
CXXFLAGS = ["-O3", "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-Wall", "-Wno-unused-function"]


def _hipcc() -> str:
    for cand in (shutil.which("hipcc"), "/opt/rocm/bin/hipcc"):
        if cand and Path(cand).exists():
            return cand
    raise RuntimeError("hipcc not found (ROCm toolchain required to build libmoe_hip.so)")


def sources() -> list[Path]:
    return sorted(CSRC.glob("*.hip"))


def _needs_rebuild(src: Path, obj: Path) -> bool:
    if not obj.exists():
        return True
    deps = [src, *CSRC.glob("*.h"), PKG.parent / "include" / "moe_hip.h"]
    return any(d.stat().st_mtime > obj.stat().st_mtime for d in deps if d.exists())


def build(verbose: bool = False, force: bool = False) -> Path:
    hipcc = _hipcc()
    OBJ_DIR.mkdir(parents=True, exist_ok=True)
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    objs = []
    jobs = []
    for src in sources():
        obj = OBJ_DIR / (src.stem + ".o")
        objs.append(obj)
        if force or _needs_rebuild(src, obj):
            jobs.append([hipcc, *CXXFLAGS, "-c", str(src), "-o", str(obj)])
    workers = min(len(jobs), max(1, min(8, os.cpu_count() or 1))) if jobs else 1
    with cf.ThreadPoolExecutor(max_workers=workers) as ex:
        for cmd, res in zip(jobs, ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), jobs)):
            if verbose:
                print(" ".join(cmd))
            if res.returncode != 0:
                raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    if force or jobs or not LIB.exists():
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", "-o", str(LIB), *map(str, objs)]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    return LIB


if __name__ == "__main__":
    print(build(verbose=True, force="--force" in sys.argv))
