"""Diagnostic (GPU box): per-module relative error of forward outputs and of
the gradients w.r.t. those outputs, GPU (bf16) and CPU-bf16-autocast (noise
floor) against CPU fp32, on the calibrated random-init detector with query
selection and matching replayed (as tests/test_gpu_model_parity.py).
Usage: python tools/grad_flow_diag.py spec B H W"""
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

WATCH = ("encoder.input_proj.2", "encoder.encoder.0.0.self_attn", "encoder.encoder.0.0.ffn", "encoder.encoder.0.0",
         "encoder.lateral_convs.0", "encoder.fpn_blocks.0", "encoder.lateral_convs.1", "encoder.fpn_blocks.1",
         "encoder.downsample_convs.0", "encoder.pan_blocks.0", "encoder.downsample_convs.1", "encoder.pan_blocks.1",
         "decoder.input_proj.0", "decoder.input_proj.1", "decoder.input_proj.2", "decoder.input_proj.2.0",
         "decoder.input_proj.2.1", "decoder.input_proj.1.0", "decoder.input_proj.1.1", "decoder.enc_output",
         "decoder.layers.0.cross_attn.value_proj", "decoder.layers.0.cross_attn", "decoder.layers.0",
         "decoder.layers.5.cross_attn.value_proj", "decoder.layers.5")


def rel(a, b):
    a = a.detach().float().cpu().reshape(-1)
    b = b.detach().float().cpu().reshape(-1)
    return float((a - b).norm() / max(float(b.norm()), 1e-20))


def run(model, crit, images, ctx, targets, nb, autocast=None, rec=None):
    cap = {}
    mods = dict(model.named_modules())

    def mk(name):
        def fh(mod, inp, out):
            o = out[0] if isinstance(out, tuple) else out
            if not torch.is_tensor(o):
                return
            cap.setdefault(name, {})["y"] = o.detach()
            if o.requires_grad:
                o.register_hook(lambda g: cap[name].__setitem__("g", g.detach()))
        return fh
    hs = [mods[n].register_forward_hook(mk(n)) for n in WATCH if n in mods]
    if autocast:
        with torch.autocast(autocast, dtype=torch.bfloat16):
            out = model(images, ctx)
    else:
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
    return cap


def _msda_fp32_accumulation():
    """--msda-fp32: unfused MSDA with fp32-atomic value gradients (A/B)."""
    from src.moe import _lib as L
    from src.rtdetr_moe import decoder as D

    D._FUSED_MSDA = False

    def bwd(ctx, grad_out):
        v, shapes_t, starts_t, lo, at = ctx.saved_tensors
        gv, gl, ga = L.msda_bwd(v, shapes_t, starts_t, lo, at, grad_out.to(torch.bfloat16).contiguous(),
                                bf16_grad_value=False)
        return gv.to(ctx.vdtype), None, None, gl, ga
    D._MSDAHip.backward = staticmethod(bwd)


def main():
    spec, B, H, W = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4])
    if "--msda-fp32" in sys.argv:
        _msda_fp32_accumulation()
    torch.manual_seed(1)
    cpu = RTDETRMoE(spec)
    images, targets, ctx = SyntheticZOD(batch=B, img_h=H, img_w=W, seed=4).sample()
    calibrate_frozen_bn(cpu, images)
    flo = copy.deepcopy(cpu)
    gpu = copy.deepcopy(cpu).cuda().to(memory_format=torch.channels_last)
    for p in gemm_params(gpu):
        p.data = p.data.to(torch.bfloat16)
    nb = max(1.0, float(sum(len(t["boxes"]) for t in targets)))
    pairs = []
    cc = run(cpu, SetCriterion(num_classes=1), images, ctx, targets, nb, rec=pairs)
    cf_ = SetCriterion(num_classes=1)
    cf_.matcher = _ReplayMatcher(pairs)
    flo.decoder.query_override = cpu.decoder.last_topk
    cf = run(flo, cf_, images, ctx, targets, nb, autocast="cpu")
    cg_ = SetCriterion(num_classes=1)
    cg_.matcher = _ReplayMatcher(pairs)
    gpu.decoder.query_override = cpu.decoder.last_topk.cuda()
    img = images.cuda().contiguous(memory_format=torch.channels_last).to(torch.bfloat16)
    cg = run(gpu, cg_, img, ctx.cuda(), [{k: v.cuda() for k, v in t.items()} for t in targets], nb)
    torch.cuda.synchronize()
    rows = []
    for n in WATCH:
        if n not in cc:
            continue
        r = {"module": n}
        for key in ("y", "g"):
            if key in cc[n] and key in cg.get(n, {}):
                yc = cc[n][key]
                yg = cg[n][key].float().cpu()
                if yg.shape != yc.shape and yg.numel() == yc.numel():
                    yg = yg.reshape(yc.shape) if yg.is_contiguous() else yg.contiguous().reshape(yc.shape)
                r[key + "_gpu"] = round(rel(yg, yc), 4)
                r[key + "_floor"] = round(rel(cf[n][key], yc), 4) if key in cf.get(n, {}) else None
        rows.append(r)
    print(json.dumps(rows, indent=0))


if __name__ == "__main__":
    main()
