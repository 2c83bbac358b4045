"""Time the decoder's batched value projection GEMMs (C2: [B*S = 154,560, 256]
x [256, 6 * 256]) on hipBLASLt (F.linear / mm) vs the grouped GEMM with G = 1
(dense): forward with the bias epilogue and the data gradient.  Prints one
JSON line per case (us per call, max abs difference vs the hipBLASLt result).
    python tools/vproj_probe.py
"""
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) * 1e3 / reps


def main():
    from src.moe import _lib as L

    L.lib()
    dev = torch.device("cuda")
    torch.manual_seed(0)
    M, K, N = 154560, 256, 1536
    x = torch.randn(M, K, device=dev).to(torch.bfloat16)
    W = (torch.randn(N, K, device=dev) * 0.05).to(torch.bfloat16)
    b = (torch.randn(N, device=dev) * 0.1).to(torch.bfloat16)
    g = torch.randn(M, N, device=dev).to(torch.bfloat16)
    off = torch.tensor([0, M], dtype=torch.int32, device=dev)
    ref = F.linear(x, W, b)
    out = L.grouped_gemm(x, W, off, 1, M, N, K, 1, L.EPI_BIAS, bias=b, dense=True)
    torch.cuda.synchronize()
    rows = [("fwd hipBLASLt", timeit(lambda: F.linear(x, W, b)), 0.0),
            ("fwd grouped dense", timeit(lambda: L.grouped_gemm(x, W, off, 1, M, N, K, 1, L.EPI_BIAS, bias=b,
                                                                 dense=True)),
             float((out.float() - ref.float()).abs().max()))]
    ref2 = g.mm(W)
    out2 = L.grouped_gemm(g, W, off, 1, M, K, N, 0, L.EPI_NONE, dense=True)
    torch.cuda.synchronize()
    rows += [("dgrad hipBLASLt", timeit(lambda: g.mm(W)), 0.0),
             ("dgrad grouped dense", timeit(lambda: L.grouped_gemm(g, W, off, 1, M, K, N, 0, L.EPI_NONE, dense=True)),
              float((out2.float() - ref2.float()).abs().max()))]
    for name, us, err in rows:
        print(json.dumps({"case": name, "us": round(us, 1), "max_abs_diff": err}), flush=True)


if __name__ == "__main__":
    main()
