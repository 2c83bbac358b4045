"""Kernel microbenchmark for the MoE HIP kernels at the C2 shapes.

Times every kernel of one MoE layer (encoder T = 8*920, decoder T = 8*300;
E = 8, k = 2, d = 256, F = 1024) back to back on one stream, interleaving the
tuning variants in one process (median of rounds), and prints one JSON line
per (kernel, shape, variant) with us / TFLOP/s / GB/s.

  python multimodal-moe_amd/kbench.py [--reps 50] [--rounds 5] [--variants 1,2] [--stages 3,4]
"""
from __future__ import annotations

import argparse
import json
import statistics
import sys
from pathlib import Path

sys.path.insert(0, str(Path(__file__).resolve().parent))

import torch  # noqa: E402

from src.moe import _lib as L  # noqa: E402


_FLUSH = None


def timed(fn, reps):
    """Median kernel execution time (us) of `fn` over `reps` calls (the sum of
    its launches when it makes several), from the dispatch-stamped event pairs
    of libmoe_hip's profiler (hipExtLaunchKernel): no host overhead or
    inter-launch gaps included.  With --cold every call is preceded by a read
    of a buffer larger than the Infinity Cache (operands start in HBM, as in a
    training step where ~GBs pass between a layer's uses of its weights)."""
    fn()
    torch.cuda.synchronize()
    L.lib().moe_profile_enable(1)
    try:
        if _FLUSH is not None:
            _FLUSH.sum()
        fn()
        per = max(1, len(L.profile_records()))
        for _ in range(reps):
            if _FLUSH is not None:
                _FLUSH.sum()
            fn()
        recs = L.profile_records()
    finally:
        L.lib().moe_profile_enable(0)
    ms = [r[1] for r in recs]
    return 1e3 * statistics.median(sum(ms[i:i + per]) for i in range(0, len(ms) - per + 1, per))


SKEW = [0.0]


def setup(T, E, k, d, F, seed=0):
    g = torch.Generator(device="cuda").manual_seed(seed)
    x = torch.randn((T, d), device="cuda", generator=g).to(torch.bfloat16)
    wg = (torch.randn((E, d), device="cuda", generator=g) * 0.3).float()
    cb = torch.randn((6, E), device="cuda", generator=g).float() * 0.5
    # --skew: an expert preference in the context bias, so the routed counts
    # differ between experts as in a real model (C2 layers: max/mean 1.9-3.2x)
    cb += SKEW[0] * torch.linspace(0.0, 1.0, E, device="cuda")
    ci = torch.randint(0, 6, (T // 920 if T % 920 == 0 else T // 300,), device="cuda", generator=g).int()
    tpi = 920 if T % 920 == 0 else 300
    w1 = (torch.randn((E, F, d), device="cuda", generator=g) / 16).to(torch.bfloat16)
    w2 = (torch.randn((E, d, F), device="cuda", generator=g) / 32).to(torch.bfloat16)
    b1 = torch.zeros((E, F), device="cuda")
    b2 = torch.zeros((E, d), device="cuda")
    idx, w, probs, lse, lrank, bcnt, auxp = L.router_topk_fwd(x, wg, cb, ci, tpi, k, True)
    rank_base, hist, offsets = L.route_scan(bcnt, 0)
    rows = T * k
    xp, pos = L.permute_fwd(x, idx, lrank, rank_base, offsets, E, 0, rows)
    _, tok = L.route_index(idx, lrank, rank_base, offsets, E, 0, rows)
    _, _, _, _, gate, _, _ = L.route_dispatch(bcnt, idx, lrank, w, auxp, T, E, 0, rows, 1e-2, 1e-3, row_gate=True)
    h = L.grouped_gemm(xp, w1, offsets, E, rows, F, d, 1, L.EPI_BIAS_RELU, bias=b1)
    yp = L.grouped_gemm(h, w2, offsets, E, rows, d, F, 1, L.EPI_BIAS, bias=b2)
    dy = torch.randn((T, d), device="cuda", generator=g).to(torch.bfloat16)
    dyp, dw = L.combine_bwd(dy, yp, pos, w)
    dh = L.grouped_gemm(dyp, w2, offsets, E, rows, F, d, 0, L.EPI_RELU_MASK, aux=h)
    dxp = L.grouped_gemm(dh, w1, offsets, E, rows, d, F, 0, L.EPI_NONE)
    # MXFP8 expert path (C5 kernels) on the same routing
    xq, xs, _ = L.permute_fwd_mx(x, idx, lrank, rank_base, offsets, E, 0, rows)
    w1q, w1s = L.quantize_mx(w1)
    w2q, w2s = L.quantize_mx(w2)
    hq, hs = L.grouped_gemm_mx(xq, xs, w1q, w1s, offsets, E, rows, F, d, L.EPI_BIAS_RELU, bias=b1, out_mx=True)
    _, dlogits = L.token_bwd(dxp, pos, probs, idx, w, dw, lse, None, None, wg, True)
    return dict(dlogits=dlogits, T=T, E=E, k=k, d=d, F=F, x=x, gate=gate, wg=wg, cb=cb, ci=ci, tpi=tpi, w1=w1, w2=w2, b1=b1, b2=b2, idx=idx,
                auxp=auxp,
                w=w, probs=probs, lse=lse, lrank=lrank, bcnt=bcnt, rank_base=rank_base, offsets=offsets, rows=rows,
                xp=xp, pos=pos, tok=tok, h=h, yp=yp, dy=dy, dyp=dyp, dw=dw, dh=dh, dxp=dxp,
                xq=xq, xs=xs, w1q=w1q, w1s=w1s, w2q=w2q, w2s=w2s, hq=hq, hs=hs)


def layer_fwd_bwd(c):
    """One MoE layer forward + backward through ops._MoELayer (all its HIP launches)."""
    from src.moe.ops import moe_layer_hip

    x = c["x"].detach().requires_grad_(True)
    y, aux, raw, hist = moe_layer_hip(x, c["wg"], c["cb"], c["w1"], c["b1"], c["w2"], c["b2"], c["ci"], c["tpi"],
                                      c["k"], True, 0, aux_coefs=(1e-2, 1e-3))
    torch.autograd.backward([y, aux], [c["dy"], torch.ones_like(aux)])


def kernels(c):
    T, E, k, d, F, rows = c["T"], c["E"], c["k"], c["d"], c["F"], c["rows"]
    A = rows
    out = [
        ("router", lambda: L.router_topk_fwd(c["x"], c["wg"], c["cb"], c["ci"], c["tpi"], k, True), 0,
         512 * T + T * (4 * (E + 1) + 16 * k)),
        ("route_scan", lambda: L.route_scan(c["bcnt"], 0), 0, 8 * c["bcnt"].numel()),
        ("permute", lambda: L.permute_fwd(c["x"], c["idx"], c["lrank"], c["rank_base"], c["offsets"], E, 0, rows),
         0, 512 * (T + A) + 12 * A),
        ("gemm1_fwd", lambda: L.grouped_gemm(c["xp"], c["w1"], c["offsets"], E, rows, F, d, 1, L.EPI_BIAS_RELU,
                                             bias=c["b1"]), 2.0 * A * F * d, 0),
        ("gemm2_fwd", lambda: L.grouped_gemm(c["h"], c["w2"], c["offsets"], E, rows, d, F, 1, L.EPI_BIAS,
                                             bias=c["b2"]), 2.0 * A * F * d, 0),
        ("ffn_fwd_fused", lambda: L.expert_ffn_fwd(c["x"], c["tok"], c["w1"], c["b1"], c["w2"], c["b2"], c["offsets"],
                                                   E, rows), 4.0 * A * F * d, 0),
        ("route_index", lambda: L.route_index(c["idx"], c["lrank"], c["rank_base"], c["offsets"], E, 0, rows), 0,
         16 * A + 4 * A),
        ("gemm1_fwd_gather", lambda: L.grouped_gemm_gather(c["x"], c["tok"], c["w1"], c["offsets"], E, rows, F, d, 1,
                                                           L.EPI_BIAS_RELU, bias=c["b1"]), 2.0 * A * F * d, 0),
        # as the layer's backward runs it: dY rows gathered by token and scaled by the gate in both halves
        ("gemm_pair2", lambda: L.grouped_gemm_bwd_pair(c["dy"], c["w2"], c["offsets"], E, rows, F, d, L.EPI_RELU_MASK,
                                                       c["h"], c["dy"], c["h"], a_gather=c["tok"], row_scale=c["gate"],
                                                       wx_gather=c["tok"], wx_scale=c["gate"]), 4.0 * A * F * d, 0),
        ("gemm_pair1", lambda: L.grouped_gemm_bwd_pair(c["dh"], c["w1"], c["offsets"], E, rows, d, F, L.EPI_NONE,
                                                       None, c["dh"], c["x"], c["tok"]), 4.0 * A * F * d, 0),
        # the layer's backward since round 5: dH, then {dXp, dW2, dW1} in one grid (moe_expert_ffn_bwd)
        ("ffn_bwd2", lambda: L.expert_ffn_bwd(c["dy"], c["tok"], c["gate"], c["x"], c["h"], c["w1"], c["w2"],
                                              c["offsets"], E, rows), 8.0 * A * F * d, 0),
        ("route_dispatch", lambda: L.route_dispatch(c["bcnt"], c["idx"], c["lrank"], c["w"], c["auxp"], T, E, 0,
                                                    rows, 1e-2, 1e-3, row_gate=True), 0, 24 * A),
        ("moe_layer_fwd_bwd", lambda: layer_fwd_bwd(c), 6.0 * A * F * d, 0),
        ("combine", lambda: L.combine_fwd(c["yp"], c["pos"], c["w"], T), 0, 512 * (A + T) + 8 * A),
        ("combine_bwd", lambda: L.combine_bwd(c["dy"], c["yp"], c["pos"], c["w"]), 0, 512 * (T + 2 * A) + 12 * A),
        ("gemm_dgrad2", lambda: L.grouped_gemm(c["dyp"], c["w2"], c["offsets"], E, rows, F, d, 0, L.EPI_RELU_MASK,
                                               aux=c["h"]), 2.0 * A * F * d, 0),
        ("gemm_wgrad2", lambda: L.grouped_gemm_wgrad(c["dyp"], c["h"], c["offsets"], E), 2.0 * A * F * d, 0),
        ("gemm_dgrad1", lambda: L.grouped_gemm(c["dh"], c["w1"], c["offsets"], E, rows, d, F, 0, L.EPI_NONE),
         2.0 * A * F * d, 0),
        ("gemm_wgrad1", lambda: L.grouped_gemm_wgrad(c["dh"], c["xp"], c["offsets"], E), 2.0 * A * F * d, 0),
        # MXFP8 (C5) variants: bytes are the algorithmic ones of the fp8 operands
        ("permute_mx", lambda: L.permute_fwd_mx(c["x"], c["idx"], c["lrank"], c["rank_base"], c["offsets"], E, 0,
                                                rows), 0, 512 * T + (256 + 8) * A + 12 * A),
        ("quantize_w1_mx", lambda: L.quantize_mx(c["w1"]), 0, E * F * d * (2 + 1 + 1 / 32)),
        ("gemm1_fwd_mx", lambda: L.grouped_gemm_mx(c["xq"], c["xs"], c["w1q"], c["w1s"], c["offsets"], E, rows, F, d,
                                                   L.EPI_BIAS_RELU, bias=c["b1"], out_mx=True), 2.0 * A * F * d, 0),
        ("gemm2_fwd_mx", lambda: L.grouped_gemm_mx(c["hq"], c["hs"], c["w2q"], c["w2s"], c["offsets"], E, rows, d, F,
                                                   L.EPI_BIAS, bias=c["b2"]), 2.0 * A * F * d, 0),
        ("gemm_dgrad2_mx", lambda: L.grouped_gemm(c["dyp"], c["w2"], c["offsets"], E, rows, F, d, 0,
                                                  L.EPI_RELU_MASK_MX, aux=c["hq"]), 2.0 * A * F * d, 0),
        ("gemm_wgrad2_mx", lambda: L.grouped_gemm_wgrad_mx(c["dyp"], c["hq"], c["hs"], c["offsets"], E),
         2.0 * A * F * d, 0),
        ("gemm_wgrad1_mx", lambda: L.grouped_gemm_wgrad_mx(c["dh"], c["xq"], c["xs"], c["offsets"], E),
         2.0 * A * F * d, 0),
        ("router_wgrad", lambda: L.router_wgrad(c["dlogits"], c["x"], c["ci"], c["tpi"], 6), 0,
         4 * T * E + 512 * T + 4 * (E * d + 6 * E)),
        ("token_bwd", lambda: L.token_bwd(c["dxp"], c["pos"], c["probs"], c["idx"], c["w"], c["dw"], c["lse"],
                                          None, None, c["wg"], True), 0, 512 * (A + T) + 4 * (2 * E + 3 * k) * T),
    ]
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--reps", type=int, default=50)
    ap.add_argument("--rounds", type=int, default=5)
    ap.add_argument("--variants", default="0")
    ap.add_argument("--stages", default="0")
    ap.add_argument("--only", default="")
    ap.add_argument("--tune", action="append", default=[], help="key=value for moe_set_tuning (repeatable)")
    ap.add_argument("--config", choices=["c2", "c5"], default="c2", help="layer shapes (C2: E8 k2 bs8; C5: E32 k4 bs16)")
    ap.add_argument("--debug", default="0", help="comma list of gemm_debug modes (1 no C stores, 2 no main loop)")
    ap.add_argument("--bm", default="0", help="comma list of forced row-tile heights (0 = auto) for rows and wgrad")
    ap.add_argument("--xcd", default="0", help="comma list of ROWS tile->XCD maps (0 auto, 1 round-robin, 2 contiguous)")
    ap.add_argument("--ksplit", default="0", help="comma list of split-K factors (0 auto, 1 off, 2..8 forced)")
    ap.add_argument("--pair", default="1", help="comma list of gemm_pair modes (1 one launch, 0 two launches)")
    ap.add_argument("--wg", default="0:0", help="comma list of gathered-wgrad bodies dma:stages (dma 0 auto / 1 "
                                                "register-staged; stages 0 auto, 2, 3)")
    ap.add_argument("--skew", type=float, default=0.0, help="expert preference added to the context bias")
    ap.add_argument("--cold", action="store_true", help="flush the Infinity Cache (512 MiB read) before every call")
    ap.add_argument("--sweep", action="append", default=[],
                    help="key=v1,v2,... moe_set_tuning values interleaved per round (one knob; repeat the flag "
                         "for a cross product)")
    a = ap.parse_args()
    SKEW[0] = a.skew
    L.lib()
    for kv in a.tune:
        key, val = kv.split("=", 1)
        L.set_tuning(key, int(val))
    if a.cold:
        global _FLUSH
        _FLUSH = torch.zeros(128 << 20, device="cuda", dtype=torch.float32)
    configs = [(v, s, dbg, bm, xm, ks, pr, wg) for v in map(int, a.variants.split(",")) for s in map(int, a.stages.split(","))
               for dbg in map(int, a.debug.split(",")) for bm in map(int, a.bm.split(","))
               for xm in map(int, a.xcd.split(",")) for ks in map(int, a.ksplit.split(","))
               for pr in map(int, a.pair.split(",")) for wg in a.wg.split(",")
               if not (v == 1 and s != int(a.stages.split(",")[0]))]
    if a.config == "c5":  # 32 experts, top-4, bs 16 (no capacity drops here: cf only trims the tail)
        shapes = {"enc": setup(16 * 920, 32, 4, 256, 1024), "dec": setup(16 * 300, 32, 4, 256, 1024, seed=1)}
    else:
        shapes = {"enc": setup(8 * 920, 8, 2, 256, 1024), "dec": setup(8 * 300, 8, 2, 256, 1024, seed=1)}
    sweeps = [[]]
    for sw in a.sweep:
        key, vals = sw.split("=", 1)
        sweeps = [prev + [(key, int(v))] for prev in sweeps for v in vals.split(",")]
    res = {}
    for _ in range(a.rounds):
      for swv in sweeps:
        for key, val in swv:
            L.set_tuning(key, val)
        tag = ",".join(f"{k}={v}" for k, v in swv)
        for (v, s, dbg, bm, xm, ks, pr, wg) in configs:
            wd, ws = (int(u) for u in wg.split(":"))
            L.set_tuning("wgrad_dma", wd)
            L.set_tuning("wgrad_stages", ws)
            L.set_tuning("gemm_pair", pr)
            L.set_tuning("ksplit", ks)
            L.set_tuning("xcd_map", xm)
            L.set_tuning("rows_bm", bm)
            L.set_tuning("wgrad_bm", bm)
            L.set_tuning("gemm_variant", v)
            L.set_tuning("gemm_stages", s)
            L.set_tuning("gemm_debug", dbg)
            for sname, c in shapes.items():
                for name, fn, flops, byts in kernels(c):
                    if a.only and a.only not in name:
                        continue
                    if not name.startswith("gemm") and (v, s, dbg, bm, xm, ks, pr, wg) != configs[0]:
                        continue
                    if pr != 1 and "pair" not in name:
                        continue
                    res.setdefault((name, sname, v, s, dbg, bm, xm, ks, pr, wg, flops, byts, tag), []).append(
                        timed(fn, a.reps))
        for key, _ in swv:
            L.set_tuning(key, 0)
    L.set_tuning("ksplit", 0)
    L.set_tuning("gemm_pair", 1)
    L.set_tuning("gemm_debug", 0)
    L.set_tuning("rows_bm", 0)
    L.set_tuning("wgrad_bm", 0)
    L.set_tuning("xcd_map", 0)
    L.set_tuning("wgrad_dma", 0)
    L.set_tuning("wgrad_stages", 0)
    for (name, sname, v, s, dbg, bm, xm, ks, pr, wg, flops, byts, tag), ts in res.items():
        us = statistics.median(ts)
        d = {"kernel": name, "config": a.config, "shape": sname, "sweep": tag, "variant": v, "stages": s, "debug": dbg,
             "bm": bm,
             "xcd": xm, "ksplit": ks, "pair": pr, "wg": wg, "skew": a.skew, "cold": a.cold, "us": round(us, 2),
             "min_us": round(min(ts), 2)}
        if flops:
            d["tflops"] = round(flops / us / 1e6, 1)
            d["frac_bf16_peak"] = round(flops / us / 1e6 / 2500.0, 4)
        if byts:
            d["gbs"] = round(byts / us / 1e3, 1)
            d["frac_hbm_peak"] = round(byts / us / 1e3 / 8000.0, 4)
        print(json.dumps(d))


if __name__ == "__main__":
    main()
