"""Host-side logic added in round 6, on the CPU: the RCCL process-group
settings and capture drain (step.rccl_env / quiesce_collectives), the
deferred convolution weight-gradient scope (conv.deferred_wgrads: nesting,
flush points, disabled scopes), and the per-launch expert-GEMM traffic join
(tools/gemm_traffic.py) on a synthetic record / PMC set."""
from __future__ import annotations

import csv
import json
import subprocess
import sys
from pathlib import Path

import pytest

ROOT = Path(__file__).resolve().parents[1]


def test_rccl_env_sets_default_only(monkeypatch):
    from src.rtdetr_moe import step

    monkeypatch.delenv("TORCH_NCCL_CUDA_EVENT_CACHE", raising=False)
    step.rccl_env()
    import os

    assert os.environ["TORCH_NCCL_CUDA_EVENT_CACHE"] == "0"
    monkeypatch.setenv("TORCH_NCCL_CUDA_EVENT_CACHE", "1")  # an explicit choice is kept
    step.rccl_env()
    assert os.environ["TORCH_NCCL_CUDA_EVENT_CACHE"] == "1"


def test_quiesce_collectives_without_rccl_returns_at_once(monkeypatch):
    import time

    import torch.distributed as dist

    from src.rtdetr_moe import step

    monkeypatch.setattr(step, "_DRAIN_S", 5.0)
    t = time.perf_counter()
    step.quiesce_collectives()  # no process group
    assert time.perf_counter() - t < 1.0
    if dist.is_initialized():
        pytest.skip("a process group is already initialised in this process")
    import socket

    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("gloo", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1)
    try:
        t = time.perf_counter()
        step.quiesce_collectives()  # gloo: nothing to drain (no RCCL watchdog)
        assert time.perf_counter() - t < 1.0
    finally:
        dist.destroy_process_group()


def test_deferred_wgrads_scope_rules(monkeypatch):
    from src.rtdetr_moe import conv as Cv

    assert Cv._WG_PENDING[0] is None
    Cv.flush_wgrads()  # outside a scope: no-op
    with Cv.deferred_wgrads():
        assert Cv._WG_PENDING[0] == []
        with pytest.raises(RuntimeError):
            with Cv.deferred_wgrads():
                pass
        Cv.flush_wgrads()  # nothing pending: no library call
    assert Cv._WG_PENDING[0] is None
    with Cv.deferred_wgrads(enabled=False):
        assert Cv._WG_PENDING[0] is None  # disabled: every wgrad reduces at once
    monkeypatch.setattr(Cv, "_WG_DEFER_ON", False)  # MOE_CONV_WG_DEFER=0
    with Cv.deferred_wgrads():
        assert Cv._WG_PENDING[0] is None
    with pytest.raises(ValueError):  # an exception inside the scope still closes it
        with Cv.deferred_wgrads(enabled=True):
            raise ValueError
    assert Cv._WG_PENDING[0] is None


def _pmc_csv(path, counter, rows):
    path.parent.mkdir(parents=True, exist_ok=True)
    with open(path, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["Dispatch_Id", "Kernel_Name", "Grid_Size", "Counter_Name", "Counter_Value"])
        for i, (name, grid, val) in enumerate(rows):
            w.writerow([i, name, grid, counter, val])


def test_gemm_traffic_join(tmp_path):
    """Records and PMC rows joined by position; a dense (FL 16) launch and the
    warm-up step's launches are skipped; gfx950 corrections (KiB, FETCH x2)."""
    tri = "void moe::gemm_triple_kernel<moe::BodyV2<64, 128, 2, false>>(moe::GemmParams)"
    g1 = "void moe::gemm_v2_kernel<64, 128, 2, true, false, 0, 3, false, 0>(moe::GemmParams)"
    dense = "void moe::gemm_v2_kernel<64, 128, 2, true, true, 0, 2, false, 16>(moe::GemmParams)"
    recs = [["grouped_gemm", 0.01, 1e9, 1.0e6], ["conv", 0.02, 1e9, 5e6], ["grouped_gemm", 0.03, 2e9, 4.0e6]]
    (tmp_path / "records.json").write_text(json.dumps({"steps": 1, "records": recs}))
    # warm-up step (2 launches) + timed step (2 launches); a dense launch in between
    _pmc_csv(tmp_path / "fetch" / "p_counter_collection.csv", "FETCH_SIZE",
             [(g1, 256 * 704, 100.0), (tri, 256 * 864, 100.0), (dense, 256 * 80, 50.0),
              (g1, 256 * 704, 500.0), (tri, 256 * 864, 1000.0)])
    _pmc_csv(tmp_path / "write" / "p_counter_collection.csv", "WRITE_SIZE",
             [(g1, 256 * 704, 10.0), (tri, 256 * 864, 10.0), (dense, 256 * 80, 5.0),
              (g1, 256 * 704, 100.0), (tri, 256 * 864, 200.0)])
    out = tmp_path / "out.json"
    r = subprocess.run([sys.executable, str(ROOT / "tools" / "gemm_traffic.py"), str(tmp_path), str(out)],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr
    d = json.loads(out.read_text())
    assert d["launches"] == 2
    per = {p["kernel"].split(" ")[0]: p for p in d["per_launch"]}
    g = per["gemm_v2<64,"]
    assert g["alg_bytes"] == 1.0e6 and g["pmc_read"] == 2 * 500.0 * 1024 and g["pmc_write"] == 100.0 * 1024
    t = per["gemm_triple"]
    assert t["alg_bytes"] == 4.0e6 and t["pmc_read"] == 2 * 1000.0 * 1024 and t["pmc_write"] == 200.0 * 1024
    assert abs(d["ratio"] - (2 * 1500 * 1024 + 300 * 1024) / 5.0e6) < 1e-12
