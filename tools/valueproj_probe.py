"""Probe: the decoder's batched value projection (_ValueProjAll) at C2 --
memory [B S = 154,560, 256] against the six layers' stacked weights
[1536, 256] -- on hipBLASLt (what the node issues: F.linear, G.mm(W), the
chunked bmm weight gradient + bias column sum) against libmoe_hip's dense
grouped GEMM (G = 1) and its wgrad kernel (weight + bias gradient in one
launch).  Device time per call from a replayed hipGraph (mm_probe_small.t);
max relative error against an fp32 product.

  python tools/valueproj_probe.py > probe.jsonl
"""
import json
import sys
from pathlib import Path

import torch
import torch.nn.functional as F

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "multimodal-moe_amd"))
sys.path.insert(0, str(ROOT / "tools"))

from mm_probe_small import t  # noqa: E402


def err(got, ref):
    return float((got.float() - ref).abs().max() / ref.abs().max())


def main():
    from src.moe import _lib as L
    from src.rtdetr_moe.linear import bias_grad, chunked_wgrad

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    rows = [int(a) for a in (sys.argv[1:] or ["154560"])]
    for M in rows:
        K, N = 256, 1536
        x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
        w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
        b = torch.randn(N, device=dev, dtype=torch.bfloat16)
        g = torch.randn(M, N, device=dev, dtype=torch.bfloat16) * 0.1
        offs = torch.tensor([0, M], dtype=torch.int32, device=dev)
        rec = {"rows": M, "K": K, "N": N}
        ref = F.linear(x.float(), w.float(), b.float())
        rec["fwd_blas_us"] = round(t(lambda: F.linear(x, w, b), reps=10), 1)
        rec["fwd_blas_err"] = err(F.linear(x, w, b), ref)
        f = lambda: L.grouped_gemm(x, w, offs, 1, M, N, K, 1, L.EPI_BIAS, bias=b, dense=True)  # noqa: E731
        rec["fwd_hip_us"] = round(t(f, reps=10), 1)
        rec["fwd_hip_err"] = err(f(), ref)
        del ref
        ref = g.float().mm(w.float())
        rec["dgrad_blas_us"] = round(t(lambda: g.mm(w), reps=10), 1)
        rec["dgrad_blas_err"] = err(g.mm(w), ref)
        f = lambda: L.grouped_gemm(g, w, offs, 1, M, K, N, 0, L.EPI_NONE, dense=True)  # noqa: E731
        rec["dgrad_hip_us"] = round(t(f, reps=10), 1)
        rec["dgrad_hip_err"] = err(f(), ref)
        del ref
        ref = g.t().float().mm(x.float())
        rb = g.float().sum(0)
        blas = lambda: (chunked_wgrad(g, x).to(torch.bfloat16), bias_grad(g, torch.bfloat16))  # noqa: E731
        rec["wgrad_blas_us"] = round(t(blas, reps=10), 1)
        gw, gb = blas()
        rec["wgrad_blas_err"] = [err(gw, ref), err(gb, rb)]
        for S in (0, 4, 2):
            if S:
                L.set_tuning("ksplit", S)
            f = lambda: L.linear_wgrad(g, x, torch.bfloat16)  # noqa: E731
            rec[f"wgrad_hip{S}_us"] = round(t(f, reps=10), 1)
            gw, gb = f()
            rec[f"wgrad_hip{S}_err"] = [err(gw, ref), err(gb, rb)]
        L.set_tuning("ksplit", 0)
        print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
