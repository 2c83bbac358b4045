"""Probe: the backbone's 1x1 convolutions (PResNet-50-vd at 1280x736, batch 8,
channels_last bf16) through MIOpen (F.conv2d, the shipped find-db) vs as plain
GEMMs on the NHWC view (y = x W^T by hipBLASLt; dX = dY W; dW = dY^T X as
chunked_wgrad's row-chunk bmm + fp32 sum).  Forward + backward (input and
weight gradients), device time per call from a replayed hipGraph.

    python tools/conv1x1_probe.py > gpurun_out/c1/probe.jsonl
"""
import json
import os
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT / "multimodal-moe_amd"))
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
os.environ.setdefault("MIOPEN_USER_DB_PATH", str(ROOT / "multimodal-moe_amd" / "miopen_db"))

import torch  # noqa: E402
import torch.nn.functional as F  # noqa: E402

SHAPES = [  # H, W, cin, cout (batch 8)
    (184, 320, 64, 64), (184, 320, 256, 64), (184, 320, 64, 256), (184, 320, 256, 128),
    (92, 160, 128, 512), (92, 160, 256, 512), (92, 160, 512, 128), (92, 160, 512, 256),
    (46, 80, 256, 1024), (46, 80, 512, 1024), (46, 80, 1024, 256), (46, 80, 1024, 512),
    (23, 40, 512, 2048), (23, 40, 1024, 2048), (23, 40, 2048, 512),
]


def timed(fn, reps=20):
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
    from src.rtdetr_moe.linear import chunked_wgrad

    torch.backends.cudnn.benchmark = True
    dev = torch.device("cuda", 0)
    tot = {"miopen": 0.0, "gemm": 0.0}
    for H, W, cin, cout in SHAPES:
        x = torch.randn(8, cin, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w = (torch.randn(cout, cin, 1, 1, device=dev, dtype=torch.bfloat16) * cin ** -0.5)
        gy = torch.randn(8, cout, H, W, device=dev, dtype=torch.bfloat16).contiguous(memory_format=torch.channels_last)
        x.requires_grad_(True)
        w.requires_grad_(True)

        def conv():
            y = F.conv2d(x, w)
            return torch.autograd.grad(y, (x, w), gy)

        x2 = x.detach().permute(0, 2, 3, 1).reshape(-1, cin)
        gy2 = gy.permute(0, 2, 3, 1).reshape(-1, cout)
        w2 = w.detach().view(cout, cin)

        def gemm():
            y = F.linear(x2, w2)
            dx = gy2.mm(w2)
            dw = chunked_wgrad(gy2, x2)
            return y, dx, dw

        r = {"H": H, "W": W, "cin": cin, "cout": cout}
        # agreement of the two formulations (fp32 sums, bf16 outputs)
        ref_y = F.conv2d(x.detach(), w.detach()).permute(0, 2, 3, 1).reshape(-1, cout).float()
        y, dx, dw = gemm()
        gx, gw = conv()
        r["y_rel"] = float((y.float() - ref_y).norm() / ref_y.norm())
        r["dx_rel"] = float((dx.float() - gx.permute(0, 2, 3, 1).reshape(-1, cin).float()).norm() / gx.float().norm())
        r["dw_rel"] = float((dw.float() - gw.view(cout, cin).float()).norm() / gw.float().norm())
        fw = lambda: F.conv2d(x.detach(), w.detach())  # noqa: E731
        r["miopen_fwd_us"] = round(timed(fw), 2)
        r["miopen_fwd_bwd_us"] = round(timed(conv), 2)
        r["gemm_fwd_us"] = round(timed(lambda: F.linear(x2, w2)), 2)
        r["gemm_dx_us"] = round(timed(lambda: gy2.mm(w2)), 2)
        r["gemm_dw_us"] = round(timed(lambda: chunked_wgrad(gy2, x2)), 2)
        r["gemm_fwd_bwd_us"] = round(timed(gemm), 2)
        tot["miopen"] += r["miopen_fwd_bwd_us"]
        tot["gemm"] += r["gemm_fwd_bwd_us"]
        print(json.dumps(r), flush=True)
    print(json.dumps({"total_fwd_bwd_us": tot}), flush=True)


if __name__ == "__main__":
    main()
