"""Probe: the decoder linears' weight gradients, dW = dY^T X over B*Q = 2,400
(C2) / 4,800 (C5) query rows with a 256-512 x 256 output.  torch.mm of the
transposed view (what TokenLinear's backward issued) took ~25 us per call in
the C2 step (45 calls/step, tools/torch_prof.py); this times the alternatives:
the transposed product X^T dY (then .t()), a contiguous dY^T copy, chunked bmm
+ fp32 sum, and libmoe_hip's wgrad kernel (G = 1)."""
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "multimodal-moe_amd"))


def t(fn, reps=50):
    """Device time per call: `reps` calls captured in one hipGraph and replayed
    (host launch overhead excluded -- an eager loop of these short kernels is
    host-bound at ~20 us per call)."""
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
    for K in (2400, 4800):
        for (m, n) in [(256, 256), (192, 256), (96, 256), (512, 4), (256, 512), (768, 256), (4, 256)]:
            dy = torch.randn(K, m, device="cuda", dtype=torch.bfloat16)
            x = torch.randn(K, n, device="cuda", dtype=torch.bfloat16)
            ref = dy.t().float().mm(x.float())
            res = {"mm_tview": t(lambda: dy.t().mm(x)),
                   "contig": t(lambda: dy.t().contiguous().mm(x))}
            for S in (4, 8):
                kc = K // S
                res[f"bmm{S}"] = t(lambda: torch.bmm(dy.view(S, kc, m).transpose(1, 2), x.view(S, kc, n))
                                   .sum(0, dtype=torch.float32))
            if m % 64 == 0 and n % 128 == 0:
                off = torch.tensor([0, K], dtype=torch.int32, device="cuda")
                f = lambda: L.grouped_gemm_wgrad(dy, x, off, 1)  # noqa: E731
                got = f()[0][0]
                res["hip_wgrad"] = t(f)
                res["hip_err"] = float((got.float() - ref).abs().max() / ref.abs().max())
                for ks in (4, 8):
                    L.set_tuning("ksplit", ks)
                    res[f"hip_ks{ks}"] = t(f)
                    got = f()[0][0]
                    res[f"hip_ks{ks}_err"] = float((got.float() - ref).abs().max() / ref.abs().max())
                L.set_tuning("ksplit", 0)
            print({"K": K, "m": m, "n": n, **{k: round(v, 2) if isinstance(v, float) else v for k, v in res.items()}},
                  flush=True)


if __name__ == "__main__":
    main()
