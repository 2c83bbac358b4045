"""The graphed evaluation forward alone (engine.EvalForward at C2: R50 +
8-expert top-2, batch 8, 1280x720 padded to 736, bf16 autocast), for a
rocprofv3 kernel trace of the inference path:

    rocprofv3 --kernel-trace --stats -d gpurun_out/eval_prof -- python3 tools/eval_prof.py
"""
from __future__ import annotations

import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)

import torch  # noqa: E402

from src.rtdetr_moe.data import SyntheticZOD  # noqa: E402
from src.rtdetr_moe.engine import EvalForward  # noqa: E402
from src.rtdetr_moe.model import RTDETRMoE  # noqa: E402


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    spec = sys.argv[2] if len(sys.argv) > 2 else "rtdetr-r50-moe8-top2"
    torch.manual_seed(1)
    model = RTDETRMoE(spec).cuda().to(memory_format=torch.channels_last)
    from src.rtdetr_moe.step import gemm_params

    for p in gemm_params(model):  # the trained model's bf16 GEMM / conv weights (TrainStep precision bf16)
        p.data = p.data.to(torch.bfloat16)
    model.eval()
    images, _, ctx = SyntheticZOD(batch=8, img_h=720, img_w=1280, seed=0).sample("cuda")
    images = images.contiguous(memory_format=torch.channels_last)
    fwd = EvalForward(model)
    fwd(images, ctx)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        fwd(images, ctx)
    torch.cuda.synchronize()
    dt = (time.perf_counter() - t0) / n
    print(f"eval forward: {1e3 * dt:.3f} ms / batch of 8, {8 / dt:.1f} images/s", flush=True)


if __name__ == "__main__":
    main()
