"""Build libmoe_hip.so (gfx950) in-tree: one hipcc -c per .hip, then link.

Used by __graft_entry__.build() and by hand: ``python multimodal-moe_amd/build_ext.py``.
The .so lands in multimodal-moe_amd/lib/ (git-ignored, travels with gpurun).

Variants (sanitizers / debug build):
  --debug  lib/libmoe_hip_debug.so: -O1 -g and -DMOE_DEBUG, which turns on the
           kernels' device-side asserts (MOE_DASSERT: gather indices, expert
           offsets, split-K arrival counters, output row maps); select it with
           MOE_HIP_LIB=<path> (src/moe/_lib.py).  A failing assert traps the
           wave: use it to locate a fault already seen, not as a routine run.
  --asan   lib/libmoe_hip_asan.so + build/capi_asan: the host code of the
           library and of tools/capi_asan.cpp (every C-ABI argument check
           driven with invalid arguments) under AddressSanitizer
           (-Xarch_host -fsanitize=address; the device code is not
           instrumented), run by tests/test_capi_asan.py on the CPU.
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


VARIANTS = {
    "release": dict(lib=LIB, obj=OBJ_DIR, flags=CXXFLAGS, link=[]),
    "debug": dict(lib=LIB_DIR / "libmoe_hip_debug.so", obj=PKG / "build" / "obj_debug",
                  flags=["-O1", "-g", "-DMOE_DEBUG"] + CXXFLAGS[1:], link=[]),
    "asan": dict(lib=LIB_DIR / "libmoe_hip_asan.so", obj=PKG / "build" / "obj_asan",
                 flags=CXXFLAGS[:1] + ["-g", "-Xarch_host", "-fsanitize=address", "-Xarch_host",
                                      "-fno-omit-frame-pointer"] + CXXFLAGS[1:],
                 link=["-Xarch_host", "-fsanitize=address"]),
}


def _needs_rebuild(src: Path, obj: Path) -> bool:
    if not obj.exists():
        return True
    deps = [src, *CSRC.glob("*.h"), PKG.parent / "include" / "moe_hip.h"]
    return any(d.stat().st_mtime > obj.stat().st_mtime for d in deps if d.exists())


def build(verbose: bool = False, force: bool = False, variant: str = "release") -> Path:
    hipcc = _hipcc()
    v = VARIANTS[variant]
    obj_dir, lib_path = v["obj"], v["lib"]
    obj_dir.mkdir(parents=True, exist_ok=True)
    LIB_DIR.mkdir(parents=True, exist_ok=True)
    objs = []
    jobs = []
    for src in sources():
        obj = obj_dir / (src.stem + ".o")
        objs.append(obj)
        if force or _needs_rebuild(src, obj):
            jobs.append([hipcc, *v["flags"], "-c", str(src), "-o", str(obj)])
    workers = min(len(jobs), max(1, min(8, os.cpu_count() or 1))) if jobs else 1
    with cf.ThreadPoolExecutor(max_workers=workers) as ex:
        for cmd, res in zip(jobs, ex.map(lambda c: subprocess.run(c, capture_output=True, text=True), jobs)):
            if verbose:
                print(" ".join(cmd))
            if res.returncode != 0:
                raise RuntimeError(f"hipcc failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    if force or jobs or not lib_path.exists():
        cmd = [hipcc, f"--offload-arch={ARCH}", "-shared", "-fPIC", *v["link"], "-o", str(lib_path),
               *map(str, objs)]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"link failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    return lib_path


ASAN_DRIVER = PKG / "build" / "capi_asan"


def build_asan_driver(verbose: bool = False) -> Path:
    """libmoe_hip_asan.so and the host-side argument-check driver, both under ASan."""
    lib_path = build(verbose=verbose, variant="asan")
    src = PKG.parent / "tools" / "capi_asan.cpp"
    if (not ASAN_DRIVER.exists() or ASAN_DRIVER.stat().st_mtime < max(src.stat().st_mtime,
                                                                      lib_path.stat().st_mtime)):
        cmd = [_hipcc(), "-g", "-fsanitize=address", "-fno-omit-frame-pointer", str(src), "-o", str(ASAN_DRIVER),
               f"-L{LIB_DIR}", "-lmoe_hip_asan", f"-Wl,-rpath,{LIB_DIR}"]
        res = subprocess.run(cmd, capture_output=True, text=True)
        if res.returncode != 0:
            raise RuntimeError(f"asan driver build failed: {' '.join(cmd)}\n{res.stdout}\n{res.stderr}")
    return ASAN_DRIVER


if __name__ == "__main__":
    force = "--force" in sys.argv
    if "--asan" in sys.argv:
        print(build_asan_driver(verbose=True))
    else:
        print(build(verbose=True, force=force, variant="debug" if "--debug" in sys.argv else "release"))
