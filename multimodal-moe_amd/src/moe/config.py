"""MoE knobs and the ``--model`` spec grammar.

The reference's ``--model`` flag names an Ultralytics hub weight
(scripts/train_rtdetr.py:40, src/models/vision/rtdetr.py:39).  Here it names a
local architecture spec (no network fetch), e.g.::

    rtdetr-r50-moe8-top2          C2/C3: R50, 8 experts, top-2, bf16
    rtdetr-r18-moe4-top1          C1: R18, 4 experts, top-1 (CPU plumbing)
    rtdetr-r50-moe16-top2-ep8     C4: 16 experts sharded over 8 ranks (slots sized per layer, below)
    rtdetr-r50-moe16-top2-ep8-epcf0    same, every layer lossless (T slots per source and expert)
    rtdetr-r50-moe16-top2-ep8-epmb0    same, every layer at ep_capacity_factor (no lossless budget)
    rtdetr-r50-moe32-top4-cf1.25-fp8   C5: capacity factor 1.25, fp8 experts
    rtdetr-r50                    dense FFN (no MoE)
"""
from __future__ import annotations

import math
import re
from dataclasses import dataclass, field


@dataclass
class MoEConfig:
    num_experts: int = 8
    top_k: int = 2
    hidden: int = 1024            # expert FFN width (RT-DETR dim_feedforward)
    capacity_factor: float = 0.0  # 0 -> no capacity limit (no drops)
    normalize: bool = True        # renormalise top-k gates to sum 1 (k > 1)
    expert_dtype: str = "bf16"    # "bf16" | "fp8"
    lb_coef: float = 1e-2         # load-balance loss coefficient
    z_coef: float = 1e-3          # router z-loss coefficient
    num_contexts: int = 6         # solar bins + missing
    use_context: bool = True
    ep_size: int = 1              # expert-parallel group size (C4)
    expert_parallel: bool = False  # route through ep.py (set by an -ep<n> spec token, n >= 1)
    # rows each rank may send to one expert in the fixed-capacity all-to-all
    # (layers with capacity_factor > 0 use their own capacity instead), sized
    # PER LAYER from its token count T:
    #  * lossless (S = T, the worst case: the EP layer equals the single-process
    #    layer) when that exchange buffer, E T d 2 bytes, fits ep_lossless_mb
    #    (default 32 MB: every C4 decoder layer, 16 x 2,400 x 512 B = 19.7 MB,
    #    where single-context batches skew the experts most -- round 4 measured
    #    22.7 % drops there at 2x the mean);
    #  * else ceil(ep_capacity_factor T k / E) (default 2.0, SURVEY 8(e)'s
    #    budget: the C4 encoder, 60 MB lossless -> 15 MB); assignments beyond it
    #    are dropped like capacity drops and counted (MoEFFN.last_ep_overflow,
    #    bench ep_overflow).
    # Spec tokens: -epcf<f> sets the factor (-epcf0: every layer lossless),
    # -epmb<MB> the lossless budget (-epmb0: every layer at the factor).
    ep_capacity_factor: float = 2.0
    ep_lossless_mb: float = 32.0
    router_init_std: float = 0.02
    ctx_init_scale: float = 0.5

    def capacity(self, tokens: int) -> int:
        if self.capacity_factor <= 0:
            return 0
        return int(math.ceil(self.capacity_factor * tokens * self.top_k / self.num_experts))

    def ep_slot_rows(self, tokens: int, d_model: int = 256) -> int:
        """Rows per (source rank, expert) of the expert-parallel exchange: the
        layer capacity when it has one; T (lossless) when the factor is 0, or
        when the lossless buffer E T d 2 bytes fits ep_lossless_mb; else
        ceil(ep_capacity_factor T k / E) -- never more than T (a token sends at
        most one row to an expert)."""
        cap = self.capacity(tokens)
        if cap > 0:
            return cap
        f = self.ep_capacity_factor
        lossless_bytes = self.num_experts * tokens * d_model * 2
        if f <= 0 or f * self.top_k >= self.num_experts or lossless_bytes <= self.ep_lossless_mb * 1e6:
            return max(1, tokens)
        return max(1, min(tokens, int(math.ceil(f * tokens * self.top_k / self.num_experts))))


@dataclass
class ModelSpec:
    backbone: str = "r50"          # r18 | r34 | r50 | r101
    moe: MoEConfig | None = field(default_factory=MoEConfig)
    num_decoder_layers: int | None = None  # default by backbone (6 for r50, 3 for r18)
    raw: str = ""


_SPEC_RE = re.compile(r"^rtdetr-(r18|r34|r50|r101)((?:-[a-z0-9.]+)*)$")


def parse_moe_spec(spec: str) -> ModelSpec:
    """Parse ``rtdetr-<backbone>[-moe<E>][-top<k>][-cf<f>][-fp8][-ep<n>][-epcf<f>][-dec<L>]``."""
    s = spec.strip().lower()
    if s.endswith(".pt") or s.endswith(".pth"):
        raise ValueError(f"{spec!r} is a weights file, not an architecture spec")
    m = _SPEC_RE.match(s)
    if not m:
        raise ValueError(
            f"unknown model spec {spec!r}; expected e.g. 'rtdetr-r50-moe8-top2' "
            "(hub weight names such as 'rtdetr-l.pt' need a network fetch and are not supported)")
    out = ModelSpec(backbone=m.group(1), moe=None, raw=spec)
    moe = None
    for tok in [t for t in m.group(2).split("-") if t]:
        if tok.startswith("moe"):
            moe = moe or MoEConfig()
            moe.num_experts = int(tok[3:])
        elif tok.startswith("top"):
            moe = moe or MoEConfig()
            moe.top_k = int(tok[3:])
        elif tok.startswith("cf"):
            moe = moe or MoEConfig()
            moe.capacity_factor = float(tok[2:])
        elif tok == "fp8":
            moe = moe or MoEConfig()
            moe.expert_dtype = "fp8"
        elif tok == "noctx":
            moe = moe or MoEConfig()
            moe.use_context = False
        elif tok.startswith("epcf"):
            moe = moe or MoEConfig()
            moe.ep_capacity_factor = float(tok[4:])
        elif tok.startswith("epmb"):
            moe = moe or MoEConfig()
            moe.ep_lossless_mb = float(tok[4:])
        elif tok.startswith("ep"):
            moe = moe or MoEConfig()
            moe.ep_size = int(tok[2:])
            moe.expert_parallel = True
        elif tok.startswith("dec"):
            out.num_decoder_layers = int(tok[3:])
        else:
            raise ValueError(f"unknown token {tok!r} in model spec {spec!r}")
    if moe is not None:
        if moe.top_k > moe.num_experts:
            raise ValueError("top_k must be <= num_experts")
        if moe.num_experts % moe.ep_size:
            raise ValueError("num_experts must be divisible by ep_size")
    out.moe = moe
    return out
