"""A/B of the 3x3 stride-1 convolution kernels (csrc/conv.hip): the
implicit-GEMM tile (conv_halo=0) against the halo-staged kernel
(conv_halo=1: 256 x 128, 8 waves; 2: 128 x 128, 4 waves), forward and data
gradient (flipped weight), interleaved per shape, hipGraph-replayed
(tools/conv_bench.timeit); also the relative error of each variant's output
against the conv_halo=0 output.

    python tools/conv_halo_ab.py [B,C,N,H,W ...] > gpurun_out/halo_ab.jsonl
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

SHAPES = [(8, 256, 256, 92, 160), (8, 128, 128, 92, 160), (8, 256, 256, 46, 80), (8, 512, 512, 23, 40),
          (8, 256, 256, 23, 40)]


def main():
    from src.moe import _lib as L
    from src.rtdetr_moe import conv as C

    lib = L.lib()
    dev = torch.device("cuda", 0)
    args = [a for a in sys.argv[1:] if "," in a]
    shapes = [tuple(int(v) for v in s.split(",")) for s in args] if args else SHAPES
    variants = [0, 1, 2]
    for (B, Ci, Co, H, W) in shapes:
        g = torch.Generator(device=dev).manual_seed(0)
        x = torch.randn(B, Ci, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        w = (torch.randn(Co, Ci, 3, 3, device=dev, generator=g) * (9 * Ci) ** -0.5).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        gy = torch.randn(B, Co, H, W, device=dev, generator=g).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        z = C._zero(dev).data_ptr()
        flop = 2.0 * B * H * W * Ci * Co * 9
        nb = lib.rtdetr_conv_dgrad_workspace(B, H, W, Ci, Co, 3)
        wk = torch.empty(max(nb // 2, Co * Ci * 9), dtype=torch.bfloat16, device=dev)
        L._check(lib.rtdetr_conv_set_tuning(b"conv_dgrad_flip", 1), "tuning")
        outs, res = {}, {}
        for rnd in range(3):
            for v in variants:
                L._check(lib.rtdetr_conv_set_tuning(b"conv_halo", v), "tuning")
                y = torch.empty_like(gy)
                gx = torch.empty_like(x)
                tf = timeit(lambda: lib.rtdetr_conv_fwd(x.data_ptr(), w.data_ptr(), y.data_ptr(), z, B, H, W, Ci, Co,
                                                        3, 1, None, None, 0, L._stream()))
                td = timeit(lambda: lib.rtdetr_conv_dgrad(gy.data_ptr(), w.data_ptr(), wk.data_ptr(), gx.data_ptr(), z,
                                                          B, H, W, Ci, Co, 3, 1, None, None, L._stream()))
                res.setdefault(v, []).append((tf, td))
                outs[v] = (y, gx)
        L._check(lib.rtdetr_conv_set_tuning(b"conv_halo", 0), "tuning")
        L._check(lib.rtdetr_conv_set_tuning(b"conv_dgrad_flip", -1), "tuning")
        ref = outs[0]
        rel = lambda a, b: float((a.float() - b.float()).norm() / b.float().norm())  # noqa: E731
        for v in variants:
            tf = sorted(r[0] for r in res[v])[1]
            td = sorted(r[1] for r in res[v])[1]
            print(json.dumps({"shape": [B, Ci, Co, H, W], "conv_halo": v, "fwd_us": round(tf, 1),
                              "dgrad_us": round(td, 1), "fwd_tflops": round(flop / tf / 1e6, 1),
                              "dgrad_tflops": round(flop / td / 1e6, 1),
                              "rel_vs_halo0": [round(rel(outs[v][0], ref[0]), 6), round(rel(outs[v][1], ref[1]), 6)]}),
                  flush=True)


if __name__ == "__main__":
    main()
