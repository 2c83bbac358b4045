"""Probe: weight-gradient GEMMs with a huge reduction dim (the decoder's
Linear layers over all 154,560 encoder-memory tokens at 1280x736, batch 8).
Times torch.mm (hipBLASLt's pick) against chunked bmm + sum."""
import torch


def t(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return 1e3 * s.elapsed_time(e) / reps


K = 154560
for (m, n) in [(256, 256), (4, 256), (1, 256)]:
    dy = torch.randn(K, m, device="cuda", dtype=torch.bfloat16)
    x = torch.randn(K, n, device="cuda", dtype=torch.bfloat16)
    base = t(lambda: dy.t().mm(x))
    ref = dy.t().float().mm(x.float())
    res = {"mm": round(base, 1)}
    for S in (16, 32, 64, 128, 240):
        if K % S:
            continue
        f = lambda: torch.bmm(dy.view(S, K // S, m).transpose(1, 2), x.view(S, K // S, n)).sum(0, dtype=torch.float32)
        err = (f() - ref).abs().max().item() / ref.abs().max().item()
        res[f"bmm{S}"] = round(t(f), 1)
        res[f"err{S}"] = f"{err:.1e}"
        f2 = lambda: torch.baddbmm(torch.zeros(1, device="cuda"), dy.view(S, K // S, m).transpose(1, 2).float(),
                                   x.view(S, K // S, n).float()).sum(0) if False else None
    print(m, n, res, flush=True)
