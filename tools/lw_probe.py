"""Probe: rtdetr_linear_wgrad (dense dW = gy^T x + db = colsum(gy), G = 1) at
the TokenLinear shapes of the C2/C5 step, device time per call from a replayed
hipGraph, across split-K factors and the two main-loop bodies (v1 register
staged, v2 LDS-DMA ring of 2-4 stages); torch's dy^T x (+ dy.sum(0)) beside.

    python tools/lw_probe.py > gpurun_out/lw/probe.jsonl
"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "multimodal-moe_amd"))


def t(fn, reps=50):
    fn()
    torch.cuda.synchronize()
    st = torch.cuda.Stream()
    with torch.cuda.stream(st):
        fn()
        st.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=st):
            for _ in range(reps):
                fn()
    g.replay()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    g.replay()
    e.record()
    torch.cuda.synchronize()
    return 1e3 * s.elapsed_time(e) / reps


def main():
    from src.moe import _lib as L

    L.lib()
    tiny = torch.zeros(1, device="cuda")
    print(json.dumps({"null_kernel_us": round(t(lambda: tiny.add_(1.0)), 2)}), flush=True)
    gy = torch.randn(2400, 256, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(2400, 256, device="cuda", dtype=torch.bfloat16)
    res = {"K": 2400, "M": 256, "N": 256, "debug": "gemm_debug 1 = no C stores, 2 = no main loop"}
    for ks in (1, 8):
        L.set_tuning("ksplit", ks)
        for dbg in (0, 1, 2, 3):
            L.set_tuning("gemm_debug", dbg)
            res[f"ks{ks}_dbg{dbg}"] = round(t(lambda: L.linear_wgrad(gy, x, torch.bfloat16)), 2)
    L.set_tuning("gemm_debug", 0)
    L.set_tuning("ksplit", 0)
    print(json.dumps(res), flush=True)
    if len(sys.argv) > 1 and sys.argv[1] == "--debug-only":
        return
    shapes = [(2400, 256, 256), (2400, 512, 256), (2400, 192, 256), (2400, 1024, 256), (2400, 256, 1024),
              (4800, 256, 256), (7360, 256, 256), (7360, 768, 256), (14720, 256, 256)]
    for K, m, n in shapes:
        gy = torch.randn(K, m, device="cuda", dtype=torch.bfloat16)
        x = torch.randn(K, n, device="cuda", dtype=torch.bfloat16)
        ref = gy.t().float().mm(x.float())
        res = {"K": K, "M": m, "N": n, "torch_mm_sum": round(t(lambda: (gy.t().mm(x), gy.sum(0))), 2)}
        for var, stages in [(1, 0), (2, 2), (2, 3), (2, 4)]:
            L.set_tuning("gemm_variant", var)
            L.set_tuning("gemm_stages", stages)
            for ks in (0, 1, 2, 4, 8):
                L.set_tuning("ksplit", ks)
                f = lambda: L.linear_wgrad(gy, x, torch.bfloat16)  # noqa: E731
                dw, _ = f()
                err = float((dw.float() - ref).abs().max() / ref.abs().max())
                res[f"v{var}s{stages}_ks{ks}"] = round(t(f), 2)
                if err > 1e-2:
                    res[f"v{var}s{stages}_ks{ks}_err"] = err
        for k in ("gemm_variant", "gemm_stages", "ksplit"):
            L.set_tuning(k, 0)
        print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
