"""Interleaved A/B of one rtdetr_conv_set_tuning knob on the convolution
forward and data gradient (flipped weight), hipGraph-replayed
(tools/conv_bench.timeit), with each variant's relative difference from the
first variant's outputs (bitwise-equal kernels print 0.0).

    python tools/conv_knob_ab.py conv_8ph=0,1 [B,C,N,H,W,KS[,stride] ...] > gpurun_out/ab.jsonl
"""
from __future__ import annotations

import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT), str(ROOT / "tools")):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from conv_bench import timeit  # noqa: E402

SHAPES = [(8, 256, 256, 92, 160, 3), (8, 256, 256, 46, 80, 3), (8, 512, 512, 23, 40, 3), (8, 256, 256, 92, 160, 1),
          (8, 1024, 256, 46, 80, 1), (8, 256, 256, 92, 160, 3, 2), (8, 512, 512, 46, 80, 3, 2)]


def main():
    from src.moe import _lib as L
    from src.rtdetr_moe import conv as C

    lib = L.lib()
    dev = torch.device("cuda", 0)
    knob, vals = sys.argv[1].split("=")
    variants = [int(v) for v in vals.split(",")]
    args = [a for a in sys.argv[2:] if "," in a]
    shapes = [tuple(int(v) for v in s.split(",")) for s in args] if args else SHAPES
    for shape in shapes:
        B, Ci, Co, H, W, ks = shape[:6]
        st = shape[6] if len(shape) > 6 else 1
        Ho, Wo = (H - 1) // st + 1, (W - 1) // st + 1
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(B, Ci, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = (torch.randn(Co, Ci, ks, ks, device=dev, generator=g) * (ks * ks * Ci) ** -0.5).to(
            torch.bfloat16).contiguous(memory_format=torch.channels_last)
        gy = torch.randn(B, Co, Ho, Wo, device=dev, generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        z = C._zero(dev).data_ptr()
        flop = 2.0 * B * Ho * Wo * Ci * Co * ks * ks
        nb = lib.rtdetr_conv_dgrad_workspace(B, H, W, Ci, Co, ks)
        wk = torch.empty(max(nb // 2, Co * Ci * ks * ks), dtype=torch.bfloat16, device=dev)
        L._check(lib.rtdetr_conv_set_tuning(b"conv_dgrad_flip", 1), "tuning")
        outs, res = {}, {}
        for _ in range(3):
            for v in variants:
                L._check(lib.rtdetr_conv_set_tuning(knob.encode(), v), "tuning")
                y = torch.empty_like(gy)
                gx = torch.empty_like(x)
                tf = timeit(lambda: lib.rtdetr_conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), z, B, H, W, Ci, Co,
                                                        ks, st, None, None, 0, L._stream()))
                td = timeit(lambda: lib.rtdetr_conv_dgrad(gy.data_ptr(), w.data_ptr(), wk.data_ptr(), gx.data_ptr(), z,
                                                          B, H, W, Ci, Co, ks, st, None, None, L._stream()))
                res.setdefault(v, []).append((tf, td))
                outs[v] = (y, gx)
        L._check(lib.rtdetr_conv_set_tuning(b"conv_dgrad_flip", -1), "tuning")
        ref = outs[variants[0]]
        rel = lambda a, b: float((a.float() - b.float()).norm() / b.float().norm())  # noqa: E731
        for v in variants:
            tf = sorted(r[0] for r in res[v])[1]
            td = sorted(r[1] for r in res[v])[1]
            print(json.dumps({"shape": list(shape), knob: v, "fwd_us": round(tf, 1), "dgrad_us": round(td, 1),
                              "fwd_tflops": round(flop / tf / 1e6, 1), "dgrad_tflops": round(flop / td / 1e6, 1),
                              "rel_vs_first": [round(rel(outs[v][0], ref[0]), 7), round(rel(outs[v][1], ref[1]), 7)]}),
                  flush=True)
        # restore the knob's default (automatic where it has one)
        L._check(lib.rtdetr_conv_set_tuning(knob.encode(), -1 if knob in ("conv_8ph", "conv_halo", "conv_k32") else 0),
                 "tuning")


if __name__ == "__main__":
    main()
