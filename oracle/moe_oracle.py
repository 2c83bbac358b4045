"""CPU oracle for the MoE-gated RT-DETR hot path -- TEST INFRASTRUCTURE ONLY.

Only tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg may import
this module, and only as the checker / CPU baseline.  The product path
(multimodal-moe_amd/src/moe) never imports it.

What it restates (numpy, float64, explicit loops over experts):
  a1  solar context bin      scripts/add_solar_context_bins.py:87-107
      (pd.cut(bins=[-1e9,-6,0,15,45,1e9], include_lowest, right-closed);
       NaN -> "missing"; duplicate at scripts/analyze_context_frequencies.py:68-83)
  a2  router                 SURVEY.md 8(a) row a2 (reference: planned only,
      notes/MoE_in_ZOD_Thesis_Proposal_revisedTimeline.txt:215-216 "Top-k
      routing"; context as an additive router-logit bias,
      notes/related_work.md:64-68)
  a3  aux losses             SURVEY.md 8(a) row a3 (load balance, z-loss:
      notes/related_work.md:72-75)
  a4  dispatch               SURVEY.md 8(a) row a4 (slot-major capacity priority)
  a5  expert FFN             SURVEY.md 8(a) row a5 ("Experts are standard MLP
      blocks", notes/related_work.md:23)
  a6  combine                SURVEY.md 8(a) row a6
  a7  backward               SURVEY.md 8(a) row a7 (hand-derived, checked
      against torch autograd in tests/test_oracle.py)

Parity status: a1 is PINNED against the reference itself (golden vectors in
tests/golden/reference_known_answers.json, made by tests/golden/make_golden.py
importing /root/reference).  a2-a7 are "parity unpinned": the reference has no
MoE code, so this restatement of the written spec is the
oracle, cross-checked against an independent torch-autograd formulation.

``emulate_bf16=True`` rounds the tensors the GPU path stores in bf16 (inputs,
H, Yp, y, dYp, dH, dXp, dx) at the same points, so GPU-vs-oracle differences
are only fp32-vs-fp64 accumulation order plus one final bf16 rounding.
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import numpy as np

# ----------------------------------------------------------------------------
# a1: solar context bins (scripts/add_solar_context_bins.py:90-107)
# ----------------------------------------------------------------------------
SOLAR_BINS = [-1e9, -6.0, 0.0, 15.0, 45.0, 1e9]
SOLAR_LABELS = [
    "night(<-6)",
    "twilight(-6..0)",
    "low_sun(0..15)",
    "mid_sun(15..45)",
    "high_sun(>45)",
]
CONTEXT_LABELS = SOLAR_LABELS + ["missing"]


def solar_context_bin(angle) -> str:
    """Label of one solar elevation angle, as pd.cut(..., include_lowest=True)."""
    try:
        a = float(angle)
    except (TypeError, ValueError):
        return "missing"
    if math.isnan(a):
        return "missing"
    # right-closed intervals (lo, hi]; include_lowest closes the first on the left
    if SOLAR_BINS[0] <= a <= SOLAR_BINS[1]:
        return SOLAR_LABELS[0]
    for i in range(1, len(SOLAR_LABELS)):
        if SOLAR_BINS[i] < a <= SOLAR_BINS[i + 1]:
            return SOLAR_LABELS[i]
    return "missing"  # outside [-1e9, 1e9]: pd.cut gives NaN -> fillna("missing")


def solar_context_id(angle) -> int:
    return CONTEXT_LABELS.index(solar_context_bin(angle))


# ----------------------------------------------------------------------------
# bf16 emulation (round-to-nearest-even, like v_cvt_pk_bf16_f32)
# ----------------------------------------------------------------------------
def round_bf16(a) -> np.ndarray:
    f = np.asarray(a, dtype=np.float32)
    u = f.view(np.uint32).astype(np.uint64)
    r = ((u + 0x7FFF + ((u >> 16) & 1)) >> 16) << 16
    out = r.astype(np.uint32).view(np.float32)
    out = np.where(np.isnan(f), np.float32(np.nan), out)
    return out.astype(np.float64)


# ----------------------------------------------------------------------------
# MXFP8 emulation (config C5 fp8 experts; include/moe_hip.h "MXFP8 expert path")
# OCP e4m3 elements, one E8M0 exponent per 32 consecutive elements of a row.
# ----------------------------------------------------------------------------
E4M3_MAX = 448.0
MX_BLOCK = 32


def mx_exponent(amax) -> np.ndarray:
    """Smallest e with amax <= 448 * 2^e, from amax's fp32 bits (1.75 = 448/2^8),
    clamped to the E8M0 range [-127, 127]; amax == 0 -> -127."""
    a = np.asarray(amax, dtype=np.float32)
    u = a.view(np.uint32).astype(np.int64)
    e = ((u >> 23) & 0xFF) - 127 - 8 + ((u & 0x7FFFFF) > 0x600000).astype(np.int64)
    e = np.where(a == 0, -127, e)
    return np.clip(e, -127, 127)


def e4m3_round(v) -> np.ndarray:
    """Round |v| <= 448 to the nearest OCP e4m3 value (ties to even; subnormal
    quantum 2^-9 below 2^-6)."""
    v = np.asarray(v, np.float64)
    a = np.abs(v)
    _, ex = np.frexp(np.where(a > 0, a, 1.0))   # a = m 2^ex, m in [0.5, 1)
    E = np.maximum(ex - 1, -6)
    q = np.exp2(E - 3)
    return np.round(v / q) * q


def mx_quantize(x):
    """x [..., K] (bf16-exact values) -> (e4m3 values [..., K] in block units,
    exponents int [..., K/32]).  Dequantised value = q * 2^e."""
    x = np.asarray(x, np.float64)
    K = x.shape[-1]
    xb = x.reshape(*x.shape[:-1], K // MX_BLOCK, MX_BLOCK)
    e = mx_exponent(np.abs(xb).max(axis=-1))
    q = e4m3_round(xb * np.exp2(-e)[..., None].astype(np.float64))
    return q.reshape(x.shape), e


def mx_dequantize(q, e) -> np.ndarray:
    q = np.asarray(q, np.float64)
    K = q.shape[-1]
    qb = q.reshape(*q.shape[:-1], K // MX_BLOCK, MX_BLOCK)
    return (qb * np.exp2(np.asarray(e, np.float64))[..., None]).reshape(q.shape)


def mx_round(x) -> np.ndarray:
    """Quantize-dequantize through MXFP8."""
    return mx_dequantize(*mx_quantize(x))


def e4m3_bytes(q) -> np.ndarray:
    """OCP e4m3 encoding (uint8) of e4m3-exact values (|q| <= 448)."""
    q = np.asarray(q, np.float64)
    sign = (q < 0) | ((q == 0) & np.signbit(q))
    a = np.abs(q)
    _, ex = np.frexp(np.where(a > 0, a, 1.0))
    E = ex - 1
    normal = (a >= 2.0 ** -6)
    exp_field = np.where(normal, E + 7, 0)
    mant = np.where(normal, a / np.exp2(E) - 1.0, a / 2.0 ** -6) * 8.0
    out = (sign.astype(np.int64) << 7) | (exp_field.astype(np.int64) << 3) | np.rint(mant).astype(np.int64)
    return np.where(a == 0, sign.astype(np.int64) << 7, out).astype(np.uint8)


def _maybe(a, on):
    return round_bf16(a) if on else np.asarray(a, dtype=np.float64)


# ----------------------------------------------------------------------------
# a2: router
# ----------------------------------------------------------------------------
def router_forward(x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize):
    """logits = x.wg^T + ctx_bias[ctx(t)]; softmax; top-k (ties -> lower id); gates."""
    x = np.asarray(x, np.float64)
    wg = np.asarray(wg, np.float64)
    T = x.shape[0]
    E = wg.shape[0]
    logits = x @ wg.T
    if ctx_bias is not None:
        img = np.arange(T) // int(tokens_per_image)
        logits = logits + np.asarray(ctx_bias, np.float64)[np.asarray(ctx_img)[img]]
    m = logits.max(axis=1, keepdims=True)
    ex = np.exp(logits - m)
    s = ex.sum(axis=1, keepdims=True)
    probs = ex / s
    lse = (m + np.log(s))[:, 0]
    # lexsort: last key primary -> by -logit, then by expert id (lowest first)
    eid = np.broadcast_to(np.arange(E), logits.shape)
    order = np.lexsort((eid, -logits), axis=1)
    idx = order[:, :k].astype(np.int64)
    psel = np.take_along_axis(probs, idx, axis=1)
    if normalize and k > 1:
        w = psel / psel.sum(axis=1, keepdims=True)
    else:
        w = psel.copy()
    return logits, probs, lse, idx, w


# ----------------------------------------------------------------------------
# a4: dispatch (slot-major, token order; capacity drop)
# ----------------------------------------------------------------------------
def dispatch_indices(idx, E, cap):
    """Returns (pos [T,k] (-1 = dropped), hist [E], offsets [E+1])."""
    idx = np.asarray(idx)
    T, k = idx.shape
    hist = np.bincount(idx.ravel(), minlength=E).astype(np.int64)
    kept = np.minimum(hist, cap) if cap and cap > 0 else hist.copy()
    offsets = np.concatenate([[0], np.cumsum(kept)]).astype(np.int64)
    rank = np.zeros((T, k), np.int64)
    seen = np.zeros(E, np.int64)
    for j in range(k):          # slot-major: every top-1 choice before any top-2
        for t in range(T):      # then token order
            e = idx[t, j]
            rank[t, j] = seen[e]
            seen[e] += 1
    if cap and cap > 0:
        pos = np.where(rank < cap, offsets[idx] + rank, -1)
    else:
        pos = offsets[idx] + rank
    return pos.astype(np.int64), hist, offsets


def permute(x, pos, rows):
    x = np.asarray(x, np.float64)
    T, k = pos.shape
    xp = np.zeros((rows, x.shape[1]))
    for t in range(T):
        for j in range(k):
            if pos[t, j] >= 0:
                xp[pos[t, j]] = x[t]
    return xp


# ----------------------------------------------------------------------------
# a5: expert FFN
# ----------------------------------------------------------------------------
def expert_ffn(xp, offsets, w1, b1, w2, b2, emulate_bf16=False, mx=False):
    """Per expert H = relu(xp W1^T + b1), Yp = H W2^T + b2.

    mx=True is the MXFP8 expert path (include/moe_hip.h): xp, W1, W2 and the
    bf16-rounded H enter the GEMMs quantize-dequantized through MXFP8 (blocks
    of 32 along each GEMM's K); the returned H is that MXFP8 H (what the
    backward reads)."""
    rows = int(offsets[-1])
    E = w1.shape[0]
    d = w2.shape[1]
    F = w1.shape[1]
    H = np.zeros((rows, F))
    Y = np.zeros((rows, d))
    if mx:
        xp = mx_round(xp)
        w1 = mx_round(w1)
        w2 = mx_round(w2)
    for e in range(E):
        a, b = int(offsets[e]), int(offsets[e + 1])
        if b <= a:
            continue
        h = np.maximum(xp[a:b] @ np.asarray(w1[e], np.float64).T + b1[e], 0.0)
        H[a:b] = _maybe(h, emulate_bf16 or mx)
        if mx:
            H[a:b] = mx_round(H[a:b])
        Y[a:b] = _maybe(H[a:b] @ np.asarray(w2[e], np.float64).T + b2[e], emulate_bf16)
    return H, Y


# ----------------------------------------------------------------------------
# a6: combine
# ----------------------------------------------------------------------------
def combine(yp, pos, w, emulate_bf16=False):
    T, k = pos.shape
    y = np.zeros((T, yp.shape[1]))
    for j in range(k):
        keep = pos[:, j] >= 0
        y[keep] += w[keep, j][:, None] * yp[pos[keep, j]]
    return _maybe(y, emulate_bf16)


# ----------------------------------------------------------------------------
# a3: aux losses
# ----------------------------------------------------------------------------
def aux_losses(probs, lse, hist, k):
    T, E = probs.shape
    f = hist / max(T * k, 1)
    P = probs.mean(axis=0) if T > 0 else np.zeros(E)
    lb = E * float((f * P).sum())
    z = float((lse ** 2).mean()) if T > 0 else 0.0
    return lb, z


@dataclass
class MoEState:
    logits: np.ndarray
    probs: np.ndarray
    lse: np.ndarray
    idx: np.ndarray
    w: np.ndarray
    pos: np.ndarray
    hist: np.ndarray
    offsets: np.ndarray
    xp: np.ndarray
    H: np.ndarray
    Yp: np.ndarray
    y: np.ndarray
    lb: float
    z: float


def moe_forward(x, wg, ctx_bias, w1, b1, w2, b2, ctx_img, tokens_per_image, k,
                normalize=True, cap=0, emulate_bf16=False, mx=False) -> MoEState:
    """Full routed FFN of one layer (a2-a6).  Shapes: x [T,d], wg [E,d],
    ctx_bias [C,E] | None, w1 [E,F,d], b1 [E,F], w2 [E,d,F], b2 [E,d].
    mx=True: MXFP8 expert GEMMs (st.xp and st.H are then the MXFP8 values the
    backward uses)."""
    E = np.asarray(wg).shape[0]
    x = _maybe(x, emulate_bf16)
    logits, probs, lse, idx, w = router_forward(x, wg, ctx_bias, ctx_img, tokens_per_image, k, normalize)
    pos, hist, offsets = dispatch_indices(idx, E, cap)
    xp = permute(x, pos, int(offsets[-1]))
    if emulate_bf16:
        w1 = round_bf16(w1)
        w2 = round_bf16(w2)
    H, Yp = expert_ffn(xp, offsets, w1, b1, w2, b2, emulate_bf16, mx)
    if mx:
        xp = mx_round(xp)
    y = combine(Yp, pos, w, emulate_bf16)
    lb, z = aux_losses(probs, lse, hist, k)
    return MoEState(logits, probs, lse, idx, w, pos, hist, offsets, xp, H, Yp, y, lb, z)


# ----------------------------------------------------------------------------
# a7: backward (hand-derived)
# ----------------------------------------------------------------------------
def moe_backward(st: MoEState, x, wg, w1, w2, ctx_img, tokens_per_image, n_ctx, dy,
                 g_lb=0.0, g_z=0.0, normalize=True, emulate_bf16=False, fused_dgrad=False):
    """Gradients of  <dy, y> + g_lb * lb + g_z * z  w.r.t. every input.

    fused_dgrad (with emulate_bf16): emulate the single-GPU bf16 path's fused
    combine transpose, whose dgrad GEMM reads the UNSCALED bf16 dy rows and
    applies the gate as an fp32 epilogue row scale, dH = relu'(H) * w (dy W2^T),
    instead of multiplying by a bf16-rounded dYp = w dy; the weight gradient
    dW2 = H^T dYp and db2 still see the rounded dYp (the MFMA operand).  Same
    value in exact arithmetic; only the rounding point moves.

    Returns dict(dx, dwg, dctx_bias, dw1, db1, dw2, db2)."""
    x = _maybe(x, emulate_bf16)
    dy = _maybe(dy, emulate_bf16)
    if emulate_bf16:
        w1 = round_bf16(w1)
        w2 = round_bf16(w2)
    w1 = np.asarray(w1, np.float64)
    w2 = np.asarray(w2, np.float64)
    wg = np.asarray(wg, np.float64)
    T, d = x.shape
    E, F = w1.shape[0], w1.shape[1]
    k = st.idx.shape[1]
    rows = int(st.offsets[-1])
    # combine transpose
    dYp = np.zeros((rows, d))
    dw = np.zeros((T, k))
    for j in range(k):
        for t in range(T):
            p = st.pos[t, j]
            if p >= 0:
                dYp[p] = st.w[t, j] * dy[t]
                dw[t, j] = float(dy[t] @ st.Yp[p])
    dYp_exact = dYp
    dYp = _maybe(dYp, emulate_bf16)
    dYp_dgrad = dYp_exact if fused_dgrad else dYp
    # expert FFN backward
    dH = np.zeros((rows, F))
    dXp = np.zeros((rows, d))
    dw1 = np.zeros_like(w1)
    dw2 = np.zeros_like(w2)
    db1 = np.zeros((E, F))
    db2 = np.zeros((E, d))
    for e in range(E):
        a, b = int(st.offsets[e]), int(st.offsets[e + 1])
        if b <= a:
            continue
        dh = (dYp_dgrad[a:b] @ w2[e]) * (st.H[a:b] > 0)
        dH[a:b] = _maybe(dh, emulate_bf16)
        dXp[a:b] = _maybe(dH[a:b] @ w1[e], emulate_bf16)
        dw2[e] = dYp[a:b].T @ st.H[a:b]
        dw1[e] = dH[a:b].T @ st.xp[a:b]
        db2[e] = dYp[a:b].sum(axis=0)
        db1[e] = dH[a:b].sum(axis=0)
    # router backward
    dprobs = np.zeros((T, E))
    psel = np.take_along_axis(st.probs, st.idx, axis=1)
    if normalize and k > 1:
        S = psel.sum(axis=1, keepdims=True)
        wdw = (st.w * dw).sum(axis=1, keepdims=True)
        dpsel = (dw - wdw) / S
    else:
        dpsel = dw
    for j in range(k):
        dprobs[np.arange(T), st.idx[:, j]] += dpsel[:, j]
    if g_lb:
        f = st.hist / max(T * k, 1)
        dprobs += g_lb * E * f[None, :] / max(T, 1)
    dlogits = st.probs * (dprobs - (st.probs * dprobs).sum(axis=1, keepdims=True))
    if g_z:
        dlogits += g_z * 2.0 * st.lse[:, None] * st.probs / max(T, 1)
    # dispatch transpose + router input grad
    dx = dlogits @ wg
    for j in range(k):
        for t in range(T):
            p = st.pos[t, j]
            if p >= 0:
                dx[t] += dXp[p]
    dx = _maybe(dx, emulate_bf16)
    dwg = dlogits.T @ x
    dctx = None
    if ctx_img is not None and n_ctx:
        dctx = np.zeros((n_ctx, E))
        img = np.arange(T) // int(tokens_per_image)
        np.add.at(dctx, np.asarray(ctx_img)[img], dlogits)
    return dict(dx=dx, dwg=dwg, dctx_bias=dctx, dw1=dw1, db1=db1, dw2=dw2, db2=db2,
                dlogits=dlogits, dw=dw)
