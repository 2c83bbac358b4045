import os
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]
PKG = ROOT / "multimodal-moe_amd"
for p in (str(ROOT), str(PKG)):
    if p not in sys.path:
        sys.path.insert(0, p)

os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (run with -m gpu)")
    config.addinivalue_line("markers", "slow: longer CPU test")


def gpu_available() -> bool:
    try:
        import torch

        return torch.cuda.is_available()
    except Exception:
        return False


@pytest.fixture(scope="session")
def hip_lib():
    """The built libmoe_hip.so, loaded; GPU tests fail (not skip) without it."""
    from src.moe import _lib

    return _lib.lib()


@pytest.fixture(scope="module", autouse=True)
def _release_gpu_memory_between_modules(request):
    """After each test module: drop unreachable graphs / tensors and return the
    caching allocator's free blocks, so that one process can run the whole GPU
    suite (hundreds of captured hipGraphs and full-size layers).  With
    MOE_TEST_MEMLOG set, one line per module: device free / reserved bytes and
    the number of live CUDAGraph objects after the cleanup."""
    yield
    try:
        import torch
    except Exception:
        return
    if not torch.cuda.is_available():
        return
    import gc

    gc.collect()
    torch.cuda.synchronize()
    torch.cuda.empty_cache()
    log = os.environ.get("MOE_TEST_MEMLOG")
    if log:
        free, total = torch.cuda.mem_get_info()
        graphs = sum(1 for o in gc.get_objects() if isinstance(o, torch.cuda.CUDAGraph))
        with open(log, "a") as f:
            f.write(f"{request.module.__name__} free_GiB={free / 2**30:.1f} total_GiB={total / 2**30:.1f} "
                    f"reserved_GiB={torch.cuda.memory_reserved() / 2**30:.1f} live_graphs={graphs}\n")


_SEGV_FILE = None


@pytest.fixture(autouse=True)
def _native_segv_backtrace():
    """MOE_SEGV_BT=1: print the native backtrace of a host segfault (tools/segv,
    put in front of whatever handler is installed -- Python's faulthandler --
    before every test).  Diagnostic only."""
    if os.environ.get("MOE_SEGV_BT") == "1":
        import ctypes

        so = ROOT / "tools" / "segv" / "libsegv_bt.so"
        if so.exists():
            global _SEGV_FILE
            if _SEGV_FILE is None:  # pytest captures fd 2: write to a file of our own
                _SEGV_FILE = open(os.environ.get("MOE_SEGV_BT_FILE", "segv_bt.txt"), "a")
            ctypes.CDLL(str(so)).segv_bt_install(_SEGV_FILE.fileno())
    yield
