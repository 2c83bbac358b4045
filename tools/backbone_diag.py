"""Diagnostic (GPU box): backbone stage outputs, GPU bf16 vs CPU fp32, with and
without frozen-BN calibration."""
import copy
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "multimodal-moe_amd")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from src.rtdetr_moe.backbone import calibrate_frozen_bn  # noqa: E402
from src.rtdetr_moe.data import SyntheticZOD  # noqa: E402
from src.rtdetr_moe.model import RTDETRMoE  # noqa: E402
from src.rtdetr_moe.step import gemm_params  # noqa: E402


def rel(a, b):
    a = a.detach().float().cpu().reshape(-1)
    b = b.detach().float().cpu().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-20))


for calib in (False, True):
    torch.manual_seed(1)
    cpu = RTDETRMoE(sys.argv[1] if len(sys.argv) > 1 else "rtdetr-r50-moe8-top2")
    images, _, ctx = SyntheticZOD(batch=1, img_h=720, img_w=1280, seed=4).sample()
    if calib:
        calibrate_frozen_bn(cpu, images)
    for prec in ("bf16", "amp", "fp32-cpu-copy"):
        gpu = copy.deepcopy(cpu)
        if prec != "fp32-cpu-copy":
            gpu = gpu.cuda().to(memory_format=torch.channels_last)
        if prec == "bf16":
            for p in gemm_params(gpu):
                p.data = p.data.to(torch.bfloat16)
        img = images.clone()
        if prec != "fp32-cpu-copy":
            img = img.cuda().contiguous(memory_format=torch.channels_last)
        if prec == "bf16":
            img = img.to(torch.bfloat16)
        with torch.no_grad():
            fc = cpu.backbone(images)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=prec == "amp"):
                fg = gpu.backbone(img)
            st = [float(f.float().std()) for f in fc]
            print(f"calib={calib} {prec}: stage rel err", [round(rel(g, c), 5) for g, c in zip(fg, fc)], "std", [round(s, 4) for s in st])
            stem_c = cpu.backbone.stem(images)
            with torch.autocast("cuda", dtype=torch.bfloat16, enabled=prec == "amp"):
                stem_g = gpu.backbone.stem(img)
            print("   stem rel err", round(rel(stem_g, stem_c), 5))
