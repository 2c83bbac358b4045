"""Probe: the RT-DETR decoder / encoder dense linears (2,400 query rows and
7,360 AIFI tokens at C2) on hipBLASLt (F.linear / mm, what TokenLinear
issues) against libmoe_hip's dense grouped GEMM (G = 1, bias epilogue), per
call, forward (x W^T + b) and data gradient (dY W).  Device time per call from
a replayed hipGraph of 50 calls (tools/mm_probe_small.t).

  python tools/linear_probe.py > probe.jsonl
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


def main():
    from src.moe import _lib as L

    dev = torch.device("cuda", 0)
    torch.manual_seed(0)
    for M in (2400, 7360):
        for K, N in ((256, 256), (256, 512), (512, 256), (256, 1024), (1024, 256), (256, 192), (256, 96), (256, 4),
                     (256, 1), (4, 512)):
            x = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
            w = torch.randn(N, K, device=dev, dtype=torch.bfloat16) * 0.05
            b = torch.randn(N, device=dev, dtype=torch.bfloat16)
            g = torch.randn(M, N, device=dev, dtype=torch.bfloat16)
            offs = torch.tensor([0, M], dtype=torch.int32, device=dev)
            rec = {"M": M, "K": K, "N": N}
            rec["fwd_blas_us"] = round(t(lambda: F.linear(x, w, b)), 2)
            rec["dgrad_blas_us"] = round(t(lambda: g.mm(w)), 2)
            if N % 128 == 0 and K % 64 == 0:
                ref = F.linear(x, w, b).float()
                got = L.grouped_gemm(x, w, offs, 1, M, N, K, 1, L.EPI_BIAS, bias=b, dense=True).float()
                rec["fwd_err"] = float((got - ref).abs().max() / ref.abs().max())
                rec["fwd_hip_us"] = round(t(lambda: L.grouped_gemm(x, w, offs, 1, M, N, K, 1, L.EPI_BIAS, bias=b,
                                                                   dense=True)), 2)
            if K % 128 == 0 and N % 64 == 0:
                ref = g.mm(w).float()
                got = L.grouped_gemm(g, w, offs, 1, M, K, N, 0, L.EPI_NONE, dense=True).float()
                rec["dgrad_err"] = float((got - ref).abs().max() / ref.abs().max())
                rec["dgrad_hip_us"] = round(t(lambda: L.grouped_gemm(g, w, offs, 1, M, K, N, 0, L.EPI_NONE,
                                                                     dense=True)), 2)
            print(json.dumps(rec), flush=True)


if __name__ == "__main__":
    main()
