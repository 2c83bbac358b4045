"""Per-shape timing of the body's convolutions: MIOpen (F.conv2d, with the
bench's find-db and benchmark mode) against the HIP implicit-GEMM kernels
(csrc/conv.hip), forward, data gradient and weight gradient separately.

    python tools/conv_bench.py > gpurun_out/conv_bench.jsonl
"""
from __future__ import annotations

import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
os.environ.setdefault("MIOPEN_USER_DB_PATH", str(ROOT / "multimodal-moe_amd" / "miopen_db"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

# (B, Cin, Cout, H, W, KS): the C2 step's stride-1 convolutions with 128-multiple channels
SHAPES = [(8, 256, 256, 46, 80, 3), (8, 256, 256, 92, 160, 3), (8, 256, 256, 23, 40, 3), (8, 128, 128, 92, 160, 3),
          (8, 512, 512, 23, 40, 3), (8, 256, 256, 46, 80, 1), (8, 256, 256, 92, 160, 1), (8, 1024, 256, 46, 80, 1),
          (8, 256, 1024, 46, 80, 1), (8, 512, 128, 92, 160, 1), (8, 128, 512, 92, 160, 1), (8, 2048, 512, 23, 40, 1),
          (8, 512, 2048, 23, 40, 1), (8, 512, 256, 92, 160, 1),
          # ResNet stage 1 (64-channel tiles)
          (8, 64, 64, 184, 320, 3), (8, 256, 64, 184, 320, 1), (8, 64, 256, 184, 320, 1), (8, 64, 64, 184, 320, 1),
          # stride 2 (ResNet-D stage entries, encoder downsampling): input sizes
          (8, 128, 128, 184, 320, 3, 2), (8, 256, 256, 92, 160, 3, 2), (8, 512, 512, 46, 80, 3, 2),
          (8, 256, 256, 46, 80, 3, 2)]


def timeit(fn, reps=20):
    """GPU time per call of fn replayed from a hipGraph (as the training step
    runs): no host launch gaps between a library's kernels."""
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(s)
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(reps):
            fn()
    g.replay()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    g.replay()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) * 1e3 / reps  # us


def main():
    from src.moe import _lib as L
    from src.rtdetr_moe import conv as C

    L.lib()
    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    shapes = SHAPES
    args = [a for a in sys.argv[1:] if "=" not in a]
    for kv in [a for a in sys.argv[1:] if "=" in a]:  # e.g. conv_bm=256
        k, v = kv.split("=")
        L._check(L.lib().rtdetr_conv_set_tuning(k.encode(), int(v)), "rtdetr_conv_set_tuning")
    if args:
        shapes = [tuple(int(v) for v in s.split(",")) for s in args]
    for shape in shapes:
        B, Ci, Co, H, W, ks = shape[:6]
        st = shape[6] if len(shape) > 6 else 1  # stride (3x3 only for 2)
        Ho, Wo = (H - 1) // st + 1, (W - 1) // st + 1
        x = torch.randn(B, Ci, H, W, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(Co, Ci, ks, ks, device=dev) * 0.05).to(torch.bfloat16).contiguous(
            memory_format=torch.channels_last)
        gy = torch.randn(B, Co, Ho, Wo, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        pad = (ks - 1) // 2
        flop = 2.0 * B * Ho * Wo * Ci * Co * ks * ks
        t_mf = timeit(lambda: F.conv2d(x, w, None, st, pad))
        t_md = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [st, st], [pad, pad], [1, 1], False,
                                                                  [0, 0], 1, [True, False, False]))
        t_mw = timeit(lambda: torch.ops.aten.convolution_backward(gy, x, w, None, [st, st], [pad, pad], [1, 1], False,
                                                                  [0, 0], 1, [False, True, False]))
        z = C._zero(dev).data_ptr()
        lib = L.lib()
        yh = torch.empty_like(gy)
        t_hf = timeit(lambda: lib.rtdetr_conv_fwd(x.data_ptr(), w.data_ptr(), yh.data_ptr(), z, B, H, W, Ci, Co, ks,
                                                  st, None, None, 0, L._stream()))
        gx = torch.empty_like(x)
        nb = lib.rtdetr_conv_dgrad_workspace(B, H, W, Ci, Co, ks)
        wk = torch.empty(max(nb // 2, 8), dtype=torch.bfloat16, device=dev)
        t_hd = timeit(lambda: lib.rtdetr_conv_dgrad(gy.data_ptr(), w.data_ptr(), wk.data_ptr(), gx.data_ptr(), z, B, H,
                                                    W, Ci, Co, ks, st, None, None, L._stream()))
        ns = lib.rtdetr_conv_wgrad_splits(B, Ho, Wo, Ci, Co, ks)
        part = torch.empty(ns * Co * Ci * ks * ks, dtype=torch.float32, device=dev)
        gw = torch.empty_like(w)
        t_hw = timeit(lambda: lib.rtdetr_conv_wgrad(gy.data_ptr(), x.data_ptr(), part.data_ptr(), ns, gw.data_ptr(), 1,
                                                    z, B, H, W, Ci, Co, ks, st, L._stream()))
        # correctness of the variant under test (HIP vs MIOpen, bf16 outputs)
        yref = F.conv2d(x, w, None, st, pad)
        xref = torch.ops.aten.convolution_backward(gy, x, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
                                                   [True, False, False])[0]
        wref = torch.ops.aten.convolution_backward(gy, x, w, None, [st, st], [pad, pad], [1, 1], False, [0, 0], 1,
                                                   [False, True, False])[1]
        rel = lambda a, b: round(float((a.float() - b.float()).norm() / b.float().norm().clamp(min=1e-12)), 5)  # noqa: E731
        errs = [rel(yh, yref), rel(gx, xref), rel(gw, wref)]
        # the same GEMM (M = output pixels, N = Cout, K = KS^2 Cin) on hipBLASLt
        # (torch.mm, bf16): what a library GEMM reaches at this shape
        am = torch.randn(B * Ho * Wo, ks * ks * Ci, device=dev).to(torch.bfloat16)
        bm = torch.randn(ks * ks * Ci, Co, device=dev).to(torch.bfloat16)
        t_mm = timeit(lambda: torch.mm(am, bm))
        del am, bm
        tf = lambda t: round(flop / t / 1e6, 1)  # noqa: E731  TFLOP/s
        print(json.dumps({"shape": list(shape), "gflop": round(flop / 1e9, 2), "wgrad_splits": ns, "dgrad_flip": nb > 0,
                          "miopen_us": [round(t_mf, 1), round(t_md, 1), round(t_mw, 1)],
                          "hip_us": [round(t_hf, 1), round(t_hd, 1), round(t_hw, 1)],
                          "miopen_tflops": [tf(t_mf), tf(t_md), tf(t_mw)], "hip_tflops": [tf(t_hf), tf(t_hd), tf(t_hw)],
                          "rel_err_vs_miopen": errs, "hipblaslt_gemm_us": round(t_mm, 1),
                          "hipblaslt_gemm_tflops": tf(t_mm),
                          "tuning": [a for a in sys.argv[1:] if "=" in a]}),
              flush=True)


if __name__ == "__main__":
    main()
