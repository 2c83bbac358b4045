"""Diagnostic (GPU box): where do the GPU (bf16) and CPU (fp32) whole-detector
runs diverge?  Per MoE layer: relative error of the layer input, output, the
gradient arriving at its output and leaving its input, the expert-weight
gradients, and the routing agreement.  Replays query selection + matching as
tests/test_gpu_model_parity.py does.  Usage: python tools/parity_diag.py spec B H W"""
import copy
import json
import sys
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT), str(ROOT / "multimodal-moe_amd"), str(ROOT / "tests")):
    sys.path.insert(0, p)
import torch  # noqa: E402

from src.rtdetr_moe.backbone import calibrate_frozen_bn  # noqa: E402
from src.rtdetr_moe.criterion import SetCriterion  # noqa: E402
from src.rtdetr_moe.data import SyntheticZOD  # noqa: E402
from src.rtdetr_moe.model import RTDETRMoE  # noqa: E402
from src.rtdetr_moe.step import gemm_params  # noqa: E402
from test_gpu_model_parity import _ReplayMatcher  # noqa: E402


def rel(a, b):
    a = a.detach().float().cpu().reshape(-1)
    b = b.detach().float().cpu().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-20))


def run(model, crit, images, ctx, targets, nb, autocast=False, rec=None):
    cap = {"x": [], "y": [], "gy": [], "gx": []}

    def fh(mod, inp, out):
        x = inp[0]
        cap["x"].append(x.detach())
        cap["y"].append(out.detach())
        if out.requires_grad:
            out.register_hook(lambda g: cap["gy"].append(g.detach()))
        if x.requires_grad:
            x.register_hook(lambda g: cap["gx"].append(g.detach()))
    hs = [m.register_forward_hook(fh) for m in model.moe_layers()]
    with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
        out = model(images, ctx)
    if rec is not None:
        orig = crit.matcher.match_many

        def r(s, t):
            x = orig(s, t)
            rec.extend(x)
            return x
        crit.matcher.match_many = r
    losses = crit(out, targets, nb)
    (sum(losses.values()) + model.moe_aux_loss()).backward()
    for h in hs:
        h.remove()
    cap["gy"].reverse()
    cap["gx"].reverse()
    return cap


def main():
    spec, B, H, W = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    prec = sys.argv[5] if len(sys.argv) > 5 else "bf16"
    torch.manual_seed(1)
    cpu = RTDETRMoE(spec)
    images, targets, ctx = SyntheticZOD(batch=B, img_h=H, img_w=W, seed=4).sample()
    if "--no-calib" not in sys.argv:
        calibrate_frozen_bn(cpu, images)
    gpu = copy.deepcopy(cpu).cuda().to(memory_format=torch.channels_last)
    if prec == "bf16":
        for p in gemm_params(gpu):
            p.data = p.data.to(torch.bfloat16)
    nb = max(1.0, float(sum(len(t["boxes"]) for t in targets)))
    pairs = []
    cc = run(cpu, SetCriterion(num_classes=1), images, ctx, targets, nb, rec=pairs)
    cg_ = SetCriterion(num_classes=1)
    cg_.matcher = _ReplayMatcher(pairs)
    gpu.decoder.query_override = cpu.decoder.last_topk.cuda()
    img = images.cuda().contiguous(memory_format=torch.channels_last)
    if prec == "bf16":
        img = img.to(torch.bfloat16)
    cg = run(gpu, cg_, img, ctx.cuda(), [{k: v.cuda() for k, v in t.items()} for t in targets], nb,
             autocast=prec == "amp")
    torch.cuda.synchronize()
    rows = []
    for i, (mc, mg) in enumerate(zip(cpu.moe_layers(), gpu.moe_layers())):
        r = {"layer": i, "x": rel(cg["x"][i], cc["x"][i]), "y": rel(cg["y"][i], cc["y"][i]),
             "gy": rel(cg["gy"][i], cc["gy"][i]) if i < len(cg["gy"]) and i < len(cc["gy"]) else None,
             "gx": rel(cg["gx"][i], cc["gx"][i]) if i < len(cg["gx"]) and i < len(cc["gx"]) else None,
             "gy_norm_cpu": float(cc["gy"][i].norm()) if i < len(cc["gy"]) else None,
             "gy_norm_gpu": float(cg["gy"][i].float().norm()) if i < len(cg["gy"]) else None}
        for n in ("wg", "w1", "w2", "b2"):
            r["d" + n] = rel(getattr(mg, n).grad, getattr(mc, n).grad)
            r["|d%s| gpu/cpu" % n] = float(getattr(mg, n).grad.float().norm() / getattr(mc, n).grad.norm())
        rows.append(r)
    dense = {}
    nc = dict(cpu.named_parameters())
    for n, p in gpu.named_parameters():
        if p.grad is not None and nc[n].grad is not None and ("ffn" not in n):
            dense[n] = rel(p.grad.contiguous(), nc[n].grad.contiguous())
    worst = sorted(dense.items(), key=lambda kv: -kv[1])[:12]
    print(json.dumps({"moe": rows, "dense_worst": worst,
                      "dense_median": sorted(dense.values())[len(dense) // 2]}, indent=1))


if __name__ == "__main__":
    main()
