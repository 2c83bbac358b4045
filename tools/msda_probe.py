"""Probe: the fused deformable-attention kernels at the C2 decoder shape
(B 8, Q 300, H 8, D 32, L 3, P 4, levels 92x160 / 46x80 / 23x40), forward and
backward time per call (eager loop between events), level-batched kernels vs
the generic ones and the deterministic backward (moe_set_tuning msda_generic), and their agreement.

    python tools/msda_probe.py > gpurun_out/ms/probe.jsonl
"""
import json
import sys
from pathlib import Path

import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "multimodal-moe_amd"))


def timed(fn, reps=20):
    """Mean wall time per call of an eager loop between events (these kernels
    run 50-100 us, far above the launch cost; autograd is not graph-captured)."""
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(reps):
        fn()
    e.record()
    torch.cuda.synchronize()
    return 1e3 * s.elapsed_time(e) / reps


def main():
    from src.moe import _lib as L
    from src.rtdetr_moe.decoder import _level_tensors

    g = torch.Generator().manual_seed(2)
    shapes = [(92, 160), (46, 80), (23, 40)]
    B, Q, H, D, Lv, P = 8, 300, 8, 32, 3, 4
    S = sum(h * w for h, w in shapes)
    dev = "cuda"
    value = torch.randn(B, S, H, D, generator=g).to(torch.bfloat16).to(dev)
    off = (torch.randn(B, Q, H * Lv * P * 2, generator=g) * 2).to(torch.bfloat16).to(dev)
    logits = torch.randn(B, Q, H * Lv * P, generator=g).to(torch.bfloat16).to(dev)
    ref = torch.cat([torch.rand(B, Q, 2, generator=g) * 0.8 + 0.1, torch.rand(B, Q, 2, generator=g) * 0.3 + 0.02],
                    -1).to(dev)
    gout = torch.randn(B, Q, H * D, generator=g).to(torch.bfloat16).to(dev)
    st, so = _level_tensors(shapes, torch.device(dev))
    # the step's layout: six layers' values side by side ([B, S, 6 H D]), this layer's slice at column 2 H D
    C = 6 * H * D
    value_all = torch.randn(B, S, C, generator=g).to(torch.bfloat16).to(dev)
    grad_all = torch.zeros(B, S, C, dtype=torch.bfloat16, device=dev)
    col0 = 2 * H * D
    res, outs = {}, {}
    for generic in (3, 0):
        L.set_tuning("msda_generic", generic)
        fwd = lambda: L.msda_fused_fwd_slice(value_all, col0, H, D, st, so, off, ref, logits, 0.5, Lv, P)  # noqa: E731
        bwd = lambda: L.msda_fused_bwd_slice(value_all, grad_all, col0, H, D, st, so, off, ref, logits, 0.5, Lv, P,  # noqa: E731
                                             gout)
        res[f"generic{generic}_fwd_us"] = round(timed(fwd), 2)
        res[f"generic{generic}_bwd_us"] = round(timed(bwd), 2)
        grad_all.zero_()
        go, gl = bwd()
        outs[generic] = (fwd().float(), grad_all[..., col0:col0 + H * D].float().clone(), go.float(), gl.float())
        grad_all.zero_()
    L.set_tuning("msda_generic", 0)
    hw = [h * w for h, w in shapes]
    det = lambda: L.msda_fused_bwd_slice_det(value_all, grad_all, col0, H, D, st, so, hw, off, ref, logits, 0.5,  # noqa: E731
                                             Lv, P, gout)
    res["det_bwd_us"] = round(timed(det), 2)
    for name, a, b in zip(("out", "dvalue", "doff", "dlogits"), outs[3], outs[0]):
        res[f"{name}_max_abs_diff"] = float((a - b).abs().max())
        res[f"{name}_rel"] = float((a - b).norm() / a.norm().clamp_min(1e-12))
    print(json.dumps(res), flush=True)


if __name__ == "__main__":
    main()
