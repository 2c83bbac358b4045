"""Seeded MoE-layer inputs at the BASELINE.json configs' shapes (test infrastructure).

Shared by the golden-fixture generator (tests/golden/make_moe_golden.py), the
CPU fixture check (tests/test_moe_golden.py) and the GPU parity tests
(tests/test_gpu_fullsize.py): inputs are regenerated from a seed with numpy's
PCG64 stream (stable across numpy versions), so fixtures store only the
oracle's OUTPUTS.

Inputs follow SURVEY.md 8(d) and are NOT filtered for routing margins (the
real routing distribution, near-ties included): x ~ N(0, 1) rounded to bf16;
router Wg ~ N(0, 0.02^2) (fp32); ctx_bias ~ 0.5 N(0, 1) (fp32); experts with
nn.Linear's init U(-1/sqrt(fan_in), 1/sqrt(fan_in)), weights rounded to bf16;
per-image solar-context ids drawn from the ZOD bin frequencies
(context_field_frequencies_final.csv:22-26), one bin for every image of a C4
("solar-context-binned") batch.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

from oracle import moe_oracle as O

D, F = 256, 1024
CTX_FREQ = np.array([0.1901, 0.0365, 0.1633, 0.4142, 0.1960])  # night, twilight, low, mid, high


@dataclass(frozen=True)
class LayerCase:
    name: str
    T: int           # tokens of the layer (images x tokens per image)
    tpi: int         # tokens per image (920 encoder at 1280x736, 300 decoder queries, 400 encoder at 640^2)
    E: int
    k: int
    cf: float        # capacity factor (0: no capacity limit)
    seed: int
    mx: bool = False  # MXFP8 expert GEMMs (config C5)
    single_ctx: bool = False

    @property
    def cap(self) -> int:
        return 0 if self.cf <= 0 else int(math.ceil(self.cf * self.T * self.k / self.E))

    @property
    def rows(self) -> int:
        return self.T * self.k if self.cap <= 0 else min(self.T * self.k, self.E * self.cap)


# Full-size MoE layers of every BASELINE.json config:
# C1 R18 moe4 top-1, 2 x 640^2; C2/C3 R50 moe8 top-2, bs 8 at 1280x736;
# C4 moe16 top-2 (one rank's batch, one context bin); C5 moe32 top-4 cf 1.25,
# bs 16, bf16 and MXFP8 experts.
FULL = {
    "c1_enc": LayerCase("c1_enc", 2 * 400, 400, 4, 1, 0.0, 11),
    "c1_dec": LayerCase("c1_dec", 2 * 300, 300, 4, 1, 0.0, 12),
    "c2_enc": LayerCase("c2_enc", 8 * 920, 920, 8, 2, 0.0, 21),
    "c2_dec": LayerCase("c2_dec", 8 * 300, 300, 8, 2, 0.0, 22),
    "c4_enc": LayerCase("c4_enc", 8 * 920, 920, 16, 2, 0.0, 41, single_ctx=True),
    "c4_dec": LayerCase("c4_dec", 8 * 300, 300, 16, 2, 0.0, 42, single_ctx=True),
    "c5_enc": LayerCase("c5_enc", 16 * 920, 920, 32, 4, 1.25, 51),
    "c5_enc_fp8": LayerCase("c5_enc_fp8", 16 * 920, 920, 32, 4, 1.25, 52, mx=True),
    "c5_dec_fp8": LayerCase("c5_dec_fp8", 16 * 300, 300, 32, 4, 1.25, 53, mx=True),
}

# Committed golden fixtures (tests/golden/moe_<name>.npz): the small configs at
# full size, the large ones at 2 images (same per-image shape, every expert
# populated) so each file stays < 2 MB.
GOLDEN = {
    "c1_enc": FULL["c1_enc"],
    "c1_dec": FULL["c1_dec"],
    "c2_enc_2img": LayerCase("c2_enc_2img", 2 * 920, 920, 8, 2, 0.0, 23),
    "c2_dec": FULL["c2_dec"],
    "c4_enc_2img": LayerCase("c4_enc_2img", 2 * 920, 920, 16, 2, 0.0, 43, single_ctx=True),
    "c5_enc_2img": LayerCase("c5_enc_2img", 2 * 920, 920, 32, 4, 1.25, 54),
    "c5_enc_2img_fp8": LayerCase("c5_enc_2img_fp8", 2 * 920, 920, 32, 4, 1.25, 55, mx=True),
    "c5_dec_fp8": FULL["c5_dec_fp8"],
}


def make_inputs(c: LayerCase) -> dict:
    """The layer's inputs and the incoming gradient dy (all bf16/fp32-exact float64)."""
    rng = np.random.default_rng(c.seed)
    n_img = c.T // c.tpi
    x = O.round_bf16(rng.standard_normal((c.T, D)))
    wg = rng.standard_normal((c.E, D)).astype(np.float32).astype(np.float64) * np.float32(0.02)
    wg = wg.astype(np.float32).astype(np.float64)
    ctx_bias = (rng.standard_normal((6, c.E)) * 0.5).astype(np.float32).astype(np.float64)
    if c.single_ctx:
        ctx_img = np.full(n_img, int(rng.choice(5, p=CTX_FREQ / CTX_FREQ.sum())), np.int32)
    else:
        ctx_img = rng.choice(5, size=n_img, p=CTX_FREQ / CTX_FREQ.sum()).astype(np.int32)
    b1_ = 1.0 / math.sqrt(D)
    b2_ = 1.0 / math.sqrt(F)
    w1 = O.round_bf16(rng.uniform(-b1_, b1_, (c.E, F, D)))
    b1 = rng.uniform(-b1_, b1_, (c.E, F)).astype(np.float32).astype(np.float64)
    w2 = O.round_bf16(rng.uniform(-b2_, b2_, (c.E, D, F)))
    b2 = rng.uniform(-b2_, b2_, (c.E, D)).astype(np.float32).astype(np.float64)
    dy = O.round_bf16(rng.standard_normal((c.T, D)) * 0.05)
    return dict(x=x, wg=wg, ctx_bias=ctx_bias, ctx_img=ctx_img, w1=w1, b1=b1, w2=w2, b2=b2, dy=dy)


G_LB, G_Z = 0.7, 0.3  # loss = <dy, y> + G_LB lb + G_Z z (gradients of both aux terms are exercised)


def run_oracle(c: LayerCase, inp: dict, fused_dgrad: bool = False):
    """fused_dgrad: emulate the single-GPU bf16 layer's gate-in-epilogue dgrad
    (oracle.moe_backward) -- the bf16 golden fixtures use it too
    (tests/golden/make_moe_golden.py); the EP and MXFP8 paths (which scatter a
    bf16 dYp) use the plain rounding points."""
    st = O.moe_forward(inp["x"], inp["wg"], inp["ctx_bias"], inp["w1"], inp["b1"], inp["w2"], inp["b2"],
                       inp["ctx_img"], c.tpi, c.k, True, c.cap, emulate_bf16=True, mx=c.mx)
    gr = O.moe_backward(st, inp["x"], inp["wg"], inp["w1"], inp["w2"], inp["ctx_img"], c.tpi, 6, inp["dy"],
                        g_lb=G_LB, g_z=G_Z, normalize=True, emulate_bf16=True, fused_dgrad=fused_dgrad)
    return st, gr


def topk_margin(logits: np.ndarray, k: int) -> np.ndarray:
    """Per token: the smallest gap between consecutive logits among the top k+1
    (how far the routing decision is from a tie)."""
    E = logits.shape[1]
    srt = -np.sort(-logits, axis=1)[:, : min(k + 1, E)]
    return np.min(np.abs(np.diff(srt, axis=1)), axis=1) if E > 1 else np.full(logits.shape[0], np.inf)


def bf16_bits(a) -> np.ndarray:
    """bf16-exact float64 -> uint16 bit patterns (lossless, half the bytes of fp32)."""
    return (np.asarray(a, np.float32).view(np.uint32) >> 16).astype(np.uint16)


def from_bf16_bits(b) -> np.ndarray:
    return (np.asarray(b, np.uint32) << 16).view(np.float32).astype(np.float64)


WROWS = 4  # expert-weight gradients are stored as WROWS output rows per expert + full-tensor checksums


def wsample(a: np.ndarray) -> np.ndarray:
    step = max(1, a.shape[1] // WROWS)
    return np.asarray(a[:, ::step], np.float32)


def tok_stride(T: int) -> int:
    """y / dx are stored for tokens t % stride == 0 (fixtures < 2 MB)."""
    return 1 if T <= 1000 else (2 if T <= 2000 else 4)


def summarize(c: LayerCase, st, gr) -> dict:
    """The fixture payload of one case (see tests/golden/make_moe_golden.py)."""
    return dict(
        idx=st.idx.astype(np.int8), pos=st.pos.astype(np.int32), hist=st.hist.astype(np.int32),
        offsets=st.offsets.astype(np.int32), margin=topk_margin(st.logits, c.k).astype(np.float32),
        lb=np.float64(st.lb), z=np.float64(st.z), tok_stride=np.int32(tok_stride(c.T)),
        y=bf16_bits(st.y[::tok_stride(c.T)]), dx=bf16_bits(gr["dx"][::tok_stride(c.T)]),
        y_sum=np.float64(st.y.sum()), dx_sum=np.float64(gr["dx"].sum()),
        dwg=gr["dwg"].astype(np.float32), dctx_bias=gr["dctx_bias"].astype(np.float32),
        db1=gr["db1"].astype(np.float32), db2=gr["db2"].astype(np.float32),
        dw1_rows=wsample(gr["dw1"]), dw2_rows=wsample(gr["dw2"]),
        dw1_sum=np.float64(gr["dw1"].sum()), dw1_sumsq=np.float64((gr["dw1"] ** 2).sum()),
        dw2_sum=np.float64(gr["dw2"].sum()), dw2_sumsq=np.float64((gr["dw2"] ** 2).sum()),
    )
