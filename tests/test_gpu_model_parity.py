"""Whole-detector parity: the GPU path (HIP MoE kernels, bf16) against the CPU
path (fp32 torch, MoE layers through src/moe/eager.py) on identical weights
and an identical seeded ZOD-shaped batch -- north_star's acceptance criterion
("detector outputs/losses within a stated fp tolerance of the reference CPU
path on identical inputs"; the engine call this replaces is
/root/reference/src/models/vision/rtdetr.py:82-94).

Two discrete decisions are made from floating-point values and would turn a
bf16 rounding difference into a different computation: the decoder's top-300
query selection and the Hungarian matching.  Both are REPLAYED from the CPU
run on the GPU run (decoder.query_override; the criterion's matcher returns
the CPU's pairs), so outputs, losses and gradients are comparable element for
element.  MoE routing is NOT replayed: each path routes its own activations,
and the per-layer routing-agreement rate is measured (on all tokens, and on
tokens whose CPU top-(k+1) logit margin exceeds EPS_MARGIN), next to the
router kernel's agreement with the fp64 oracle on the GPU's own activations.

Configs: C1's model (R18 + 4-expert top-1) at 640x640, batch 2, and C2's
(R50 + 8-expert top-2) at 1280x720 (padded to 736), batch 2 and -- in bf16,
the bench precision -- C2's own batch 8, random-init
weights with the frozen backbone BatchNorm statistics calibrated on the batch
(backbone.calibrate_frozen_bn: the default mean-0 / var-1 statistics of a
random backbone let its features vanish, which amplifies any rounding
difference -- a pretrained backbone does not behave that way); GPU precision
"bf16" (bf16 weights, TrainStep's default) and "amp" (fp32 weights under bf16
autocast).

Tolerance.  A random-init detector amplifies rounding: bf16 mixed precision
alone moves its fp32 outputs and gradients by percents to tens of percent
(BatchNorm with batch statistics cancels most of a gradient, so what is left
is relatively noisy).  The test therefore measures that NOISE FLOOR in the same
run -- the CPU path again under torch.autocast("cpu", bfloat16), an
independent bf16 mixed-precision implementation of the same model -- and
requires, for every quantity q (relative Frobenius error against the fp32 CPU
run; losses: relative error):
    err_GPU(q) <= FLOOR_X * err_CPU-bf16(q) + ATOL[q]
for the pred_logits / pred_boxes of every decoder layer and the encoder
output, every loss term and the total, and the router / expert gradients of
every MoE layer, and the router INPUT of every MoE layer.  Routing: the router
kernel agrees with the fp64 oracle on the GPU's own activations (>= 0.999),
and every CPU-vs-GPU routing flip is explained by the router-input difference:
a token whose top-k set differs has a CPU top-(k+1) logit gap no larger than
2 max_e |logit_GPU - logit_CPU| (fp64 logits of each path's own input; at most
1e-3 of the tokens may be unexplained).  With the router inputs inside the
floor bound, routing then differs only where bf16 noise may move it.  The
agreement rates (all tokens, and tokens with CPU margin > EPS_MARGIN, next to
the CPU-bf16 run's) are reported, not bounded: the R50 detector's logit
perturbations exceed EPS_MARGIN on a few percent of its tokens.
Measured (profiles/r02/parity_model.json): the GPU's deviations are ~2x the
CPU-bf16 floor on activations (the GPU path stores EVERY activation and, in
"bf16" precision, every GEMM/conv weight in bf16; CPU autocast rounds only the
GEMM/conv inputs), hence FLOOR_X = 4; losses stay within 3.3 % of fp32 (ATOL 5 %).
Batch 2: at batch 1 the decoder's input_proj BatchNorm (training statistics over
one 23x40 map) has near-constant channels whose 1/sigma amplifies ANY
perturbation of the incoming gradient (on the CPU alone, 1 % noise on it moves
its input gradient by 140 %; tools/grad_flow_diag.py), which no precision
comparison survives.
Per-stage report: the same relative errors for the backbone outputs (S3-S5),
the AIFI layer, the encoder outputs (P3-P5), the selected memory projection and
every decoder layer, in forward order, with the first stage whose GPU error
exceeds 1.5x the CPU-bf16 floor (also bounded by FLOOR_X x floor + ATOL).
Set MOE_PARITY_REPORT=<path> to write the measured numbers as JSON
(profiles/r03/parity_model.json).
"""
from __future__ import annotations

import copy
import json
import os
from pathlib import Path

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"
EPS_MARGIN = 5e-2
FLOOR_X = 4.0                                        # GPU error <= FLOOR_X x the bf16 noise floor + ATOL
ATOL = {"logits": 2e-2, "boxes": 1e-3, "loss": 5e-2, "grad": 1e-1, "act": 1e-2}
_REPORT = {}


class _ReplayMatcher(torch.nn.Module):
    """Matcher stub: returns the pairs recorded from another criterion run."""

    def __init__(self, recorded):
        super().__init__()
        self.recorded = recorded

    def match_many(self, output_sets, targets):
        return self.recorded


def _stage_names(model):
    """Module names of the per-stage report, in forward order: backbone S3-S5,
    the AIFI layer, the encoder outputs P3-P5, the selected memory projection
    and every decoder layer."""
    names = ["backbone", "encoder.encoder.0.0", "encoder", "decoder.enc_output"]
    return names + [f"decoder.layers.{i}" for i in range(len(model.decoder.layers))]


def _stage_hooks(model, store):
    """Forward hooks that record the stage outputs (detached fp32 CPU copies)."""
    mods = dict(model.named_modules())
    hooks = []
    for n in _stage_names(model):
        def f(mod, inp, out, n=n):
            outs = list(out) if isinstance(out, (list, tuple)) else [out]
            for i, o in enumerate(outs):
                key = n if len(outs) == 1 else f"{n}[{i}]"
                store[key] = o.detach().float().cpu()
        hooks.append(mods[n].register_forward_hook(f))
    return hooks


def _run(model, crit, images, ctx, targets, nb, autocast=False, matcher_record=None, stages=None):
    captured = []
    hooks = [m.register_forward_hook(lambda mod, inp, out: captured.append(inp[0].detach().reshape(-1, inp[0].shape[-1])))
             for m in model.moe_layers()]
    if stages is not None:
        hooks += _stage_hooks(model, stages)
    try:
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=autocast):
            out = model(images, ctx)
        if matcher_record is not None:
            orig = crit.matcher.match_many

            def rec(sets, tg):
                r = orig(sets, tg)
                matcher_record.extend(r)
                return r
            crit.matcher.match_many = rec
        losses = crit(out, targets, nb)
        aux = model.moe_aux_loss()
        total = sum(losses.values()) + aux
        total.backward()
    finally:
        for h in hooks:
            h.remove()
    return out, losses, total, captured


def _sets(out):
    return [("final", out)] + [(f"aux{i}", o) for i, o in enumerate(out["aux_outputs"])] + [("enc", out["enc_outputs"])]


@pytest.mark.parametrize("precision", ["bf16", "amp"])
@pytest.mark.parametrize("spec,B,h,w", [("rtdetr-r18-moe4-top1", 2, 640, 640), ("rtdetr-r50-moe8-top2", 2, 720, 1280),
                                        ("rtdetr-r50-moe8-top2", 8, 720, 1280)])
def test_detector_gpu_vs_cpu(hip_lib, spec, B, h, w, precision):
    if B == 8 and precision != "bf16":
        pytest.skip("C2's batch 8 at the bench precision (bf16) only: the CPU runs take ~1 min")
    from oracle import moe_oracle as O
    from src.moe import _lib as L
    from src.moe import eager
    from src.rtdetr_moe.backbone import calibrate_frozen_bn
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.data import SyntheticZOD
    from src.rtdetr_moe.model import RTDETRMoE
    from src.rtdetr_moe.step import gemm_params

    torch.manual_seed(1)
    cpu = RTDETRMoE(spec)
    images, targets, ctx = SyntheticZOD(batch=B, img_h=h, img_w=w, seed=4).sample()
    calibrate_frozen_bn(cpu, images)  # well-conditioned backbone, as with pretrained statistics
    flo = copy.deepcopy(cpu)  # the bf16-autocast CPU run (noise floor)
    gpu = copy.deepcopy(cpu).to(DEV).to(memory_format=torch.channels_last)
    if precision == "bf16":
        for p in gemm_params(gpu):
            p.data = p.data.to(torch.bfloat16)
    nb = max(1.0, float(sum(len(t["boxes"]) for t in targets)))

    # CPU fp32 reference path (records the query selection and the matching)
    crit_c = SetCriterion(num_classes=1)
    pairs = []
    st_c, st_g, st_f = {}, {}, {}
    out_c, loss_c, tot_c, xs_c = _run(cpu, crit_c, images, ctx, targets, nb, matcher_record=pairs, stages=st_c)

    # GPU path, replaying the two discrete choices
    crit_g = SetCriterion(num_classes=1)
    crit_g.matcher = _ReplayMatcher(pairs)  # host index pairs, as the host matcher returns them
    gpu.decoder.query_override = cpu.decoder.last_topk.to(DEV)
    img_g = images.to(DEV).contiguous(memory_format=torch.channels_last)
    if precision == "bf16":
        img_g = img_g.to(torch.bfloat16)
    tg = [{k: v.to(DEV) for k, v in t.items()} for t in targets]
    out_g, loss_g, tot_g, xs_g = _run(gpu, crit_g, img_g, ctx.to(DEV), tg, nb, autocast=precision == "amp",
                                      stages=st_g)
    torch.cuda.synchronize()
    assert torch.equal(gpu.decoder.last_topk.cpu(), cpu.decoder.last_topk)

    # the noise floor: the CPU path again under bf16 autocast, same replayed choices
    flo.decoder.query_override = cpu.decoder.last_topk
    crit_f = SetCriterion(num_classes=1)
    crit_f.matcher = _ReplayMatcher(pairs)
    fh = _stage_hooks(flo, st_f)
    with torch.autocast("cpu", dtype=torch.bfloat16):
        out_f = flo(images, ctx)
    for hk in fh:
        hk.remove()
    loss_f = crit_f(out_f, targets, nb)
    tot_f = sum(loss_f.values()) + flo.moe_aux_loss()
    tot_f.backward()
    xs_f = []
    hooks = [m.register_forward_hook(lambda mod, inp, out: xs_f.append(inp[0].detach().reshape(-1, inp[0].shape[-1])))
             for m in flo.moe_layers()]
    with torch.no_grad(), torch.autocast("cpu", dtype=torch.bfloat16):
        flo(images, ctx)
    for hk in hooks:
        hk.remove()

    def rel(a, b):
        a = a.detach().float().cpu().reshape(-1)
        b = b.detach().float().cpu().reshape(-1)
        return float((a - b).norm() / max(float(b.norm()), 1e-12))

    rep = {"spec": spec, "batch": B, "img": f"{w}x{h}", "precision": precision, "floor_x": FLOOR_X, "atol": ATOL}
    checks = []  # (what, kind, gpu error, floor error)
    for (name, oc), (_, og), (_, of) in zip(_sets(out_c), _sets(out_g), _sets(out_f)):
        checks.append((f"pred_logits/{name}", "logits", rel(og["pred_logits"], oc["pred_logits"]),
                       rel(of["pred_logits"], oc["pred_logits"])))
        checks.append((f"pred_boxes/{name}", "boxes", rel(og["pred_boxes"], oc["pred_boxes"]),
                       rel(of["pred_boxes"], oc["pred_boxes"])))
    lrel = lambda a, b: abs(float(a) - float(b)) / max(abs(float(b)), 1e-3)  # noqa: E731
    for k in loss_c:
        checks.append((f"loss/{k}", "loss", lrel(loss_g[k], loss_c[k]), lrel(loss_f[k], loss_c[k])))
    checks.append(("loss/total", "loss", lrel(tot_g, tot_c), lrel(tot_f, tot_c)))
    named_c, named_f = dict(cpu.named_parameters()), dict(flo.named_parameters())
    for n, pg in gpu.named_parameters():
        if pg.grad is None or not any(s in n for s in (".ffn.wg", ".ffn.ctx_bias", ".ffn.w1", ".ffn.w2", ".ffn.b1",
                                                        ".ffn.b2")):
            continue
        gc, gf = named_c[n].grad, named_f[n].grad
        if gc is None or gf is None:
            continue
        gg = pg.grad.detach().float().contiguous().cpu().reshape(gc.shape)
        checks.append((f"grad/{n}", "grad", rel(gg, gc), rel(gf, gc)))

    # routing agreement per MoE layer
    ragree = []
    for li, (mc, mg, xc, xg, xf) in enumerate(zip(cpu.moe_layers(), gpu.moe_layers(), xs_c, xs_g, xs_f)):
        cfg = mc.cfg
        T = xc.shape[0]
        tpi = T // B
        ci = ctx.to(torch.int32)
        xgb = xg.to(torch.bfloat16).contiguous()
        idx_g = L.router_topk_fwd(xgb, mg.wg.detach().float().contiguous(), mg.ctx_bias.detach().float().contiguous(),
                                  ci.to(DEV), tpi, cfg.top_k, cfg.normalize)[0].cpu().numpy()
        xo = xgb.float().cpu().numpy().astype(np.float64)
        _, _, _, idx_o, _ = O.router_forward(xo, mg.wg.detach().double().cpu().numpy(),
                                             mg.ctx_bias.detach().double().cpu().numpy(), ci.numpy(), tpi,
                                             cfg.top_k, True)
        _, _, idx_c, _ = eager.route(xc, mc.wg.detach(), mc.ctx_bias.detach(), ci, tpi, cfg.top_k, cfg.normalize)
        _, _, idx_f, _ = eager.route(xf.float(), mc.wg.detach(), mc.ctx_bias.detach(), ci, tpi, cfg.top_k,
                                     cfg.normalize)
        bias = mc.ctx_bias.detach().double()[ci.long()].repeat_interleave(tpi, 0)
        logits_c = (xc.double() @ mc.wg.detach().double().t() + bias).numpy()
        logits_g = (xg.double().cpu() @ mg.wg.detach().double().cpu().t() +
                    mg.ctx_bias.detach().double().cpu()[ci.long()].repeat_interleave(tpi, 0)).numpy()
        delta = np.abs(logits_g - logits_c).max(1)
        checks.append((f"router_in/l{li}", "act", rel(xg, xc), rel(xf, xc)))
        srt = -np.sort(-logits_c, axis=1)[:, : min(cfg.top_k + 1, cfg.num_experts)]
        margin = np.min(np.abs(np.diff(srt, axis=1)), axis=1)
        s_g, s_o, s_c, s_f = (np.sort(a, 1) for a in (idx_g, idx_o, idx_c.numpy(), idx_f.numpy()))
        wide = margin > EPS_MARGIN
        e2e, flr = np.all(s_g == s_c, 1), np.all(s_f == s_c, 1)
        kth_gap = srt[:, cfg.top_k - 1] - srt[:, min(cfg.top_k, srt.shape[1] - 1)]
        unexplained = ~e2e & (kth_gap > 2 * delta + 1e-4)  # fp32-kernel slack
        ragree.append({"layer": li, "tokens": T, "kernel_vs_fp64_oracle": float(np.all(s_g == s_o, 1).mean()),
                       "flips_unexplained": float(unexplained.mean()),
                       "median_logit_delta": float(np.median(delta)), "median_kth_gap": float(np.median(kth_gap)),
                       "cpu_vs_gpu_all": float(e2e.mean()), "cpu_vs_cpu_bf16_all": float(flr.mean()),
                       "cpu_vs_gpu_margin_gt_eps": float(e2e[wide].mean()) if wide.any() else 1.0,
                       "cpu_vs_cpu_bf16_margin_gt_eps": float(flr[wide].mean()) if wide.any() else 1.0,
                       "frac_margin_gt_eps": float(wide.mean())})
    # per-stage activations in forward order: where does the GPU's deviation
    # from fp32 first exceed 1.5x the CPU-bf16 floor?
    stages = []
    for key in st_c:
        e, f = rel(st_g[key], st_c[key]), rel(st_f[key], st_c[key])
        stages.append({"stage": key, "gpu": round(e, 5), "cpu_bf16_floor": round(f, 5),
                       "ratio": round(e / max(f, 1e-12), 3)})
        checks.append((f"stage/{key}", "act", e, f))
    rep["stages"] = stages
    rep["first_stage_over_1.5x_floor"] = next((s_["stage"] for s_ in stages if s_["ratio"] > 1.5), None)
    rep["routing_agreement"] = ragree
    rep["checks"] = {w: {"gpu": round(e, 5), "cpu_bf16_floor": round(f, 5),
                         "limit": round(FLOOR_X * f + ATOL[kind], 5)} for w, kind, e, f in checks}
    _REPORT[f"{spec}/{precision}"] = rep

    bad = [(w, round(e, 4), round(FLOOR_X * f + ATOL[kind], 4)) for w, kind, e, f in checks
           if e > FLOOR_X * f + ATOL[kind]]
    assert not bad, f"{len(bad)} of {len(checks)} quantities beyond {FLOOR_X} x the bf16 floor + atol: {bad[:8]}"
    for r in ragree:
        assert r["kernel_vs_fp64_oracle"] >= 0.999, r
        assert r["flips_unexplained"] <= 1e-3, r


def teardown_module(module):
    path = os.environ.get("MOE_PARITY_REPORT")
    if path and _REPORT:
        p = Path(path)
        p = p.with_name(p.stem + "_model" + p.suffix)
        p.parent.mkdir(parents=True, exist_ok=True)
        p.write_text(json.dumps(_REPORT, indent=1, sort_keys=True))
