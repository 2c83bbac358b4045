"""GPU parity of the HIP MoE kernels against the CPU oracle (oracle/moe_oracle.py).

Every test calls libmoe_hip.so through its C-ABI (src/moe/_lib.py -> ctypes)
and compares with the float64 oracle run on the same bf16-representable
inputs (``emulate_bf16=True`` rounds the same intermediates the GPU stores in
bf16).  Tolerances (stated per check below):
  integer outputs (top-k ids, pos, hist, offsets, permuted rows): bit-exact;
  fp32 router outputs (probs, lse, gates): |err| <= 2e-6;
  bf16 tensors: |err| <= 1e-2 * max|ref| + 1 bf16 ulp of the value
  (fp32 accumulation order differs from the fp64 oracle, then one rounding);
  fp32 weight gradients: relative Frobenius error <= 5e-3.
Integer-valued GEMM checks are exact (small integers are exact in bf16 and
their fp32 sums are exact).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import moe_oracle as O

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _bf16(a):
    return torch.from_numpy(np.asarray(O.round_bf16(a), np.float32)).to(torch.bfloat16)


def _np(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def make_case(T, d, E, F, k, tpi, seed, C=6, wg_std=0.3, ctx_scale=0.5, skew=None):
    """Random bf16-representable inputs whose top-(k) choice has a margin of
    at least 1e-3 in fp64 logits (so fp32 vs fp64 cannot flip a selection)."""
    rng = np.random.default_rng(seed)
    n_img = (T + tpi - 1) // tpi
    wg = O.round_bf16(rng.standard_normal((E, d)) * wg_std).astype(np.float32).astype(np.float64)
    ctx_bias = (rng.standard_normal((C, E)) * ctx_scale).astype(np.float32).astype(np.float64)
    if skew is not None:
        ctx_bias[:, :] = 0.0
        ctx_bias[:, skew] = 60.0  # steer every token to one expert
    ctx_img = rng.integers(0, C, size=n_img).astype(np.int32)
    x = O.round_bf16(rng.standard_normal((T, d)))
    for _ in range(50):
        logits, *_ = O.router_forward(x, wg, ctx_bias, ctx_img, tpi, k, True)
        srt = -np.sort(-logits, axis=1)
        gaps = np.min(np.abs(np.diff(srt[:, : min(k + 1, E)], axis=1)), axis=1) if E > 1 else np.ones(T)
        bad = gaps < 1e-3
        if not bad.any():
            break
        x[bad] = O.round_bf16(rng.standard_normal((int(bad.sum()), d)))
    else:
        raise RuntimeError("could not build a tie-free case")
    w1 = O.round_bf16(rng.standard_normal((E, F, d)) / np.sqrt(d))
    b1 = (rng.standard_normal((E, F)) * 0.1).astype(np.float32).astype(np.float64)
    w2 = O.round_bf16(rng.standard_normal((E, d, F)) / np.sqrt(F))
    b2 = (rng.standard_normal((E, d)) * 0.1).astype(np.float32).astype(np.float64)
    return dict(x=x, wg=wg, ctx_bias=ctx_bias, ctx_img=ctx_img, w1=w1, b1=b1, w2=w2, b2=b2, tpi=tpi)


def bf16_close(got, ref, what):
    """Layer outputs vs the oracle: tests/_tolreport.check_layer_output (one
    bf16 ulp per element plus 0.05 x RMS everywhere, 0.015 x RMS for 99.9 %)."""
    from _tolreport import check_layer_output

    check_layer_output(got, ref, what, "bf16")


def rel_fro(got, ref):
    got = np.asarray(got, np.float64)
    ref = np.asarray(ref, np.float64)
    return float(np.linalg.norm(got - ref) / max(np.linalg.norm(ref), 1e-12))


# ---------------------------------------------------------------------------
# grouped GEMM with exact integer data (layout / indexing checks)
# ---------------------------------------------------------------------------
def _int_tensor(rng, shape, lo=-3, hi=4):
    return rng.integers(lo, hi, size=shape).astype(np.float64)


# (gemm_variant, gemm_stages, ksplit[, deep_stages]); 0 = per-shape choice, ksplit 1 = no split-K;
# deep_stages: the ring depth of long-K sub-chip row GEMMs (default 3)
GEMM_CFGS = [(0, 0, 0), (0, 0, 1), (1, 2, 1), (2, 2, 1), (2, 3, 1), (2, 4, 1),
             (1, 2, 2), (2, 2, 3), (2, 3, 4), (1, 2, 5), (0, 0, 1, 4), (0, 0, 1, 6)]


@pytest.fixture
def gemm_cfg(request, hip_lib):
    from src.moe import _lib as L

    v, s, ks, *deep = request.param
    L.set_tuning("gemm_variant", v)
    L.set_tuning("gemm_stages", s)
    L.set_tuning("ksplit", ks)
    L.set_tuning("deep_stages", deep[0] if deep else 3)
    yield request.param
    L.set_tuning("gemm_variant", 0)  # back to the per-shape choice
    L.set_tuning("gemm_stages", 0)
    L.set_tuning("ksplit", 0)
    L.set_tuning("deep_stages", 3)
    # split-K arrival counters are left at zero by every launch
    torch.cuda.synchronize()
    for _ws, cnt in L._SPLIT_WS.values():
        assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("gemm_cfg", GEMM_CFGS, indirect=True)
@pytest.mark.parametrize("trans_b", [1, 0])
@pytest.mark.parametrize("rows_per_group", [[0, 1, 63, 64, 65, 200, 0, 130], [1000, 24, 0, 500]])
@pytest.mark.parametrize("N,K", [(1024, 256), (256, 1024), (128, 64)])
def test_grouped_gemm_exact(gemm_cfg, trans_b, rows_per_group, N, K):
    from src.moe import _lib as L

    rng = np.random.default_rng(7)
    G = len(rows_per_group)
    offsets = np.concatenate([[0], np.cumsum(rows_per_group)]).astype(np.int32)
    R = int(offsets[-1])
    A = _int_tensor(rng, (R + 5, K))  # extra rows beyond the groups must be ignored
    Bw = _int_tensor(rng, (G, N, K) if trans_b else (G, K, N))
    bias = _int_tensor(rng, (G, N))
    ref = np.zeros((R, N))
    for g in range(G):
        a, b = offsets[g], offsets[g + 1]
        Bg = Bw[g].T if trans_b else Bw[g]  # logical [K][N]
        ref[a:b] = A[a:b] @ Bg
    At = torch.from_numpy(A).to(torch.bfloat16).to(DEV)
    Bt = torch.from_numpy(Bw).to(torch.bfloat16).to(DEV).contiguous()
    off_t = torch.from_numpy(offsets).to(DEV)
    C = L.grouped_gemm(At, Bt, off_t, G, R + 5, N, K, trans_b, L.EPI_NONE)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(C)[:R], O.round_bf16(ref))  # exact fp32 sum, one RNE rounding
    # bias + relu epilogue
    bias_t = torch.from_numpy(bias).float().to(DEV)
    C2 = L.grouped_gemm(At, Bt, off_t, G, R + 5, N, K, trans_b, L.EPI_BIAS_RELU, bias=bias_t)
    gid = np.repeat(np.arange(G), rows_per_group)
    ref2 = np.maximum(ref + bias[gid], 0)
    # values are integers up to ~|3*3*K| -> may exceed bf16's exact range: compare in bf16
    np.testing.assert_array_equal(_np(C2)[:R], O.round_bf16(ref2))
    # relu-mask epilogue (mask from C2 > 0)
    C3 = L.grouped_gemm(At, Bt, off_t, G, R + 5, N, K, trans_b, L.EPI_RELU_MASK, aux=C2)
    np.testing.assert_array_equal(_np(C3)[:R], O.round_bf16(ref * (O.round_bf16(ref2) > 0)))


@pytest.mark.parametrize("gemm_cfg", GEMM_CFGS, indirect=True)
@pytest.mark.parametrize("rows_per_group", [[0, 1, 63, 64, 65, 200, 0, 130], [700, 0, 33], [1500, 40, 0, 1100]])
@pytest.mark.parametrize("M,N", [(256, 1024), (1024, 256), (64, 128)])
def test_grouped_gemm_wgrad_exact(gemm_cfg, rows_per_group, M, N):
    from src.moe import _lib as L

    rng = np.random.default_rng(11)
    G = len(rows_per_group)
    offsets = np.concatenate([[0], np.cumsum(rows_per_group)]).astype(np.int32)
    R = int(offsets[-1])
    X = _int_tensor(rng, (R + 3, M), -2, 3)
    Y = _int_tensor(rng, (R + 3, N), -2, 3)
    Xt = torch.from_numpy(X).to(torch.bfloat16).to(DEV)
    Yt = torch.from_numpy(Y).to(torch.bfloat16).to(DEV)
    off_t = torch.from_numpy(offsets).to(DEV)
    C, cs = L.grouped_gemm_wgrad(Xt, Yt, off_t, G)
    Cb, csb = L.grouped_gemm_wgrad(Xt, Yt, off_t, G, out_dtype=torch.bfloat16)  # bf16 out: RNE of the sums
    torch.cuda.synchronize()
    for g in range(G):
        a, b = offsets[g], offsets[g + 1]
        np.testing.assert_array_equal(_np(C[g]), X[a:b].T @ Y[a:b])
        np.testing.assert_array_equal(_np(cs[g]), X[a:b].sum(0))
        np.testing.assert_array_equal(_np(Cb[g]), O.round_bf16(X[a:b].T @ Y[a:b]))
        np.testing.assert_array_equal(_np(csb[g]), O.round_bf16(X[a:b].sum(0)))


# ---------------------------------------------------------------------------
# router / dispatch / combine / full layer against the oracle
# ---------------------------------------------------------------------------
CASES = [
    # T, d, E, F, k, tpi, cap_factor, seed
    (1, 256, 4, 1024, 1, 1, 0.0, 0),
    (200, 256, 4, 1024, 1, 100, 0.0, 1),
    (1000, 256, 8, 1024, 2, 250, 0.0, 2),
    (1300, 256, 8, 1024, 2, 130, 1.25, 3),
    (777, 256, 16, 1024, 2, 111, 0.0, 4),
    (640, 256, 32, 1024, 4, 64, 1.25, 5),
    (333, 128, 8, 256, 3, 333, 0.5, 6),
    (500, 384, 5, 256, 2, 100, 0.0, 7),  # d/128 = 3 row chunks, E not a power of two
    (300, 256, 64, 256, 8, 300, 0.0, 8),  # E = 64: 4-wave router blocks, 4 experts per lane
]


def _cap(T, k, E, cf):
    import math

    return 0 if cf <= 0 else int(math.ceil(cf * T * k / E))


@pytest.mark.parametrize("T,d,E,F,k,tpi,cf,seed", CASES)
def test_router_dispatch_combine(hip_lib, T, d, E, F, k, tpi, cf, seed):
    from src.moe import _lib as L

    c = make_case(T, d, E, F, k, tpi, seed)
    cap = _cap(T, k, E, cf)
    st = O.moe_forward(c["x"], c["wg"], c["ctx_bias"], c["w1"], c["b1"], c["w2"], c["b2"],
                       c["ctx_img"], tpi, k, True, cap, emulate_bf16=True)
    x = _bf16(c["x"]).to(DEV)
    wg = torch.from_numpy(c["wg"]).float().to(DEV)
    cb = torch.from_numpy(c["ctx_bias"]).float().to(DEV)
    ci = torch.from_numpy(c["ctx_img"]).to(DEV)
    idx, w, probs, lse, lrank, bcnt, auxp = L.router_topk_fwd(x, wg, cb, ci, tpi, k, True)
    rank_base, hist, offsets = L.route_scan(bcnt, cap)
    rows = T * k if cap <= 0 else min(T * k, E * cap)
    xp, pos = L.permute_fwd(x, idx, lrank, rank_base, offsets, E, cap, rows)
    torch.cuda.synchronize()
    # integer outputs: exact
    np.testing.assert_array_equal(idx.cpu().numpy(), st.idx)
    np.testing.assert_array_equal(hist.cpu().numpy(), st.hist)
    np.testing.assert_array_equal(offsets.cpu().numpy(), st.offsets)
    np.testing.assert_array_equal(pos.cpu().numpy(), st.pos)
    R = int(st.offsets[-1])
    np.testing.assert_array_equal(_np(xp)[:R], st.xp)
    # fp32 router outputs
    np.testing.assert_allclose(_np(probs), st.probs, atol=2e-6, rtol=0)
    np.testing.assert_allclose(_np(lse), st.lse, atol=2e-6 * max(1, np.abs(st.lse).max()), rtol=0)
    np.testing.assert_allclose(_np(w), st.w, atol=2e-6, rtol=0)
    # aux partials
    np.testing.assert_allclose(_np(auxp[:, :E].sum(0)), st.probs.sum(0), rtol=1e-5, atol=1e-4)
    np.testing.assert_allclose(float(auxp[:, E].sum()), float((st.lse ** 2).sum()), rtol=1e-5)
    # combine with the oracle's Yp (isolates the combine kernel)
    yp = _bf16(st.Yp if R > 0 else np.zeros((1, d))).to(DEV)
    y = L.combine_fwd(yp, pos, w, T)
    torch.cuda.synchronize()
    bf16_close(_np(y), st.y, "combine y")


@pytest.mark.parametrize("T,d,E,F,k,tpi,cf,seed", CASES)
def test_moe_layer_fwd_bwd(hip_lib, T, d, E, F, k, tpi, cf, seed):
    from src.moe.ops import moe_ffn_hip

    c = make_case(T, d, E, F, k, tpi, seed)
    cap = _cap(T, k, E, cf)
    rng = np.random.default_rng(100 + seed)
    dy = O.round_bf16(rng.standard_normal((T, d)))
    g_lb, g_z = 0.7, 0.3
    st = O.moe_forward(c["x"], c["wg"], c["ctx_bias"], c["w1"], c["b1"], c["w2"], c["b2"],
                       c["ctx_img"], tpi, k, True, cap, emulate_bf16=True)
    gr = O.moe_backward(st, c["x"], c["wg"], c["w1"], c["w2"], c["ctx_img"], tpi, 6, dy,
                        g_lb=g_lb, g_z=g_z, normalize=True, emulate_bf16=True)

    def P(a, dtype=torch.float32):
        return torch.from_numpy(np.asarray(a)).to(dtype).to(DEV).requires_grad_(True)

    x = P(c["x"], torch.bfloat16)
    wg, cb = P(c["wg"]), P(c["ctx_bias"])
    w1, b1, w2, b2 = P(c["w1"]), P(c["b1"]), P(c["w2"]), P(c["b2"])
    ci = torch.from_numpy(c["ctx_img"]).to(DEV)
    y, lb, z, hist = moe_ffn_hip(x, wg, cb, w1, b1, w2, b2, ci, tpi, k, True, cap)
    loss = (y.float() * _bf16(dy).float().to(DEV)).sum() + g_lb * lb + g_z * z
    loss.backward()
    torch.cuda.synchronize()
    bf16_close(_np(y), st.y, "y")
    assert abs(float(lb.detach()) - st.lb) <= 1e-5 * max(1.0, abs(st.lb))
    assert abs(float(z.detach()) - st.z) <= 1e-5 * max(1.0, abs(st.z))
    np.testing.assert_array_equal(hist.cpu().numpy(), st.hist)
    bf16_close(_np(x.grad), gr["dx"], "dx")
    for name, t in [("dwg", wg), ("dctx_bias", cb), ("dw1", w1), ("db1", b1), ("dw2", w2), ("db2", b2)]:
        ref = gr[name]
        e = rel_fro(_np(t.grad), ref)
        assert e <= 5e-3, f"{name}: relative Frobenius error {e:.2e}"


@pytest.mark.parametrize("T,d,E,F,k,tpi,cf,seed", [CASES[0], CASES[2], CASES[5]])
def test_moe_layer_residual_fused(hip_lib, T, d, E, F, k, tpi, cf, seed):
    """residual=True (moe_combine_res_fwd + moe_token_bwd_res): y = x + FFN(x)
    and dx = dy + the layer's dx, against the oracle (x + y, dx + dy) and
    against the unfused GPU path (x + y in torch, autograd's accumulation):
    outputs within one bf16 rounding of the unfused ones, every parameter
    gradient bit-identical (they see the same dy)."""
    from src.moe.ops import moe_ffn_hip

    c = make_case(T, d, E, F, k, tpi, seed)
    cap = _cap(T, k, E, cf)
    rng = np.random.default_rng(200 + seed)
    dy = O.round_bf16(rng.standard_normal((T, d)))
    st = O.moe_forward(c["x"], c["wg"], c["ctx_bias"], c["w1"], c["b1"], c["w2"], c["b2"],
                       c["ctx_img"], tpi, k, True, cap, emulate_bf16=True)
    gr = O.moe_backward(st, c["x"], c["wg"], c["w1"], c["w2"], c["ctx_img"], tpi, 6, dy,
                        g_lb=0.0, g_z=0.0, normalize=True, emulate_bf16=True)
    runs = {}
    for fused in (True, False):
        def P(a, dtype=torch.float32):
            return torch.from_numpy(np.asarray(a)).to(dtype).to(DEV).requires_grad_(True)

        x = P(c["x"], torch.bfloat16)
        ps = [P(c["wg"]), P(c["ctx_bias"]), P(c["w1"]), P(c["b1"]), P(c["w2"]), P(c["b2"])]
        ci = torch.from_numpy(c["ctx_img"]).to(DEV)
        if fused:
            out, *_ = moe_ffn_hip(x, *ps[:2], *ps[2:], ci, tpi, k, True, cap, residual=True)
        else:
            y, *_ = moe_ffn_hip(x, *ps[:2], *ps[2:], ci, tpi, k, True, cap)
            out = x + y
        (out.float() * _bf16(dy).float().to(DEV)).sum().backward()
        torch.cuda.synchronize()
        runs[fused] = (out, x.grad, [p.grad for p in ps])
    out, dx, grads = runs[True]
    out_u, dx_u, grads_u = runs[False]
    bf16_close(_np(out), c["x"] + st.y, "x + y")
    bf16_close(_np(dx), gr["dx"] + dy, "dx + dy")
    # the unfused path rounds the branch sum to bf16 before the add: the two
    # differ by at most half an ulp of the addends' scale plus one final rounding
    def ulp(m):
        return np.exp2(np.floor(np.log2(np.maximum(m, 1e-30))) - 7)

    x64, dy64 = c["x"], dy
    for name, a, b, addend in [("out", out, out_u, x64), ("dx", dx, dx_u, dy64)]:
        a, b = _np(a), _np(b)
        bound = ulp(np.abs(addend) + np.abs(b)) + ulp(np.maximum(np.abs(a), np.abs(b)))
        assert np.all(np.abs(a - b) <= bound), f"{name}: fused vs unfused beyond one bf16 rounding"
    for name, g, gu in zip(["dwg", "dctx_bias", "dw1", "db1", "dw2", "db2"], grads, grads_u):
        assert torch.equal(g, gu), f"{name}: fused residual changed a parameter gradient"


def test_skewed_routing_and_empty_experts(hip_lib):
    """Every token forced to one expert (others empty), with capacity drops."""
    from src.moe.ops import moe_ffn_hip

    T, d, E, F, k, tpi = 500, 256, 8, 1024, 2, 50
    c = make_case(T, d, E, F, k, tpi, 9, wg_std=0.05, skew=3)
    cap = _cap(T, k, E, 1.0)
    st = O.moe_forward(c["x"], c["wg"], c["ctx_bias"], c["w1"], c["b1"], c["w2"], c["b2"],
                       c["ctx_img"], tpi, k, True, cap, emulate_bf16=True)
    assert st.hist[3] == T and (st.pos[:, 0] >= 0).sum() == cap  # drops happen
    x = _bf16(c["x"]).to(DEV)
    f = lambda a: torch.from_numpy(np.asarray(a)).float().to(DEV)
    y, lb, z, hist = moe_ffn_hip(x, f(c["wg"]), f(c["ctx_bias"]), f(c["w1"]), f(c["b1"]), f(c["w2"]),
                                 f(c["b2"]), torch.from_numpy(c["ctx_img"]).to(DEV), tpi, k, True, cap)
    torch.cuda.synchronize()
    bf16_close(_np(y), st.y, "y (skewed)")
    np.testing.assert_array_equal(hist.cpu().numpy(), st.hist)


def test_library_reports_bad_shapes(hip_lib):
    from src.moe import _lib as L

    x = torch.zeros((10, 100), dtype=torch.bfloat16, device=DEV)  # d not a multiple of 128
    wg = torch.zeros((4, 100), dtype=torch.float32, device=DEV)
    with pytest.raises(L.MoEKernelError, match="multiple of 128"):
        L.router_topk_fwd(x, wg, None, None, 10, 1, True)


def test_library_profiler_records_gemm_work(hip_lib):
    """moe_profile_*: one record per launch, GEMM work = 2 N K x routed rows read from offsets[G]."""
    from src.moe import _lib as L

    rows_per_group = [100, 0, 37, 300]
    G, N, K = len(rows_per_group), 256, 128
    offsets = torch.tensor(np.concatenate([[0], np.cumsum(rows_per_group)]), dtype=torch.int32, device=DEV)
    R = int(sum(rows_per_group))
    A = torch.ones((R + 64, K), dtype=torch.bfloat16, device=DEV)
    B = torch.ones((G, N, K), dtype=torch.bfloat16, device=DEV)
    L.TIMER.start()
    try:
        L.grouped_gemm(A, B, offsets, G, R + 64, N, K, 1, L.EPI_NONE)
        L.grouped_gemm_wgrad(A[:R].contiguous(), torch.ones((R, N), dtype=torch.bfloat16, device=DEV), offsets, G)
        L.TIMER.harvest()
    finally:
        L.TIMER.stop()
    s = L.TIMER.summary()
    g = s["grouped_gemm"]
    assert g["launches"] == 2
    assert g["flops"] == 2.0 * R * N * K + 2.0 * R * K * N
    # bytes: fwd = weights + R rows of A and C; wgrad = fp32 C + colsum + R rows of X and Y
    assert g["bytes"] == (2.0 * G * N * K + R * (2 * K + 2 * N)) + (4.0 * G * K * N + 4.0 * G * K + R * 2 * (K + N))
    assert 0 < g["avg_us"] < 1e5
    assert lib_count_after_stop() == 0


def lib_count_after_stop():
    from src.moe import _lib as L

    return L.lib().moe_profile_count()


@pytest.mark.gpu
def test_fused_aux_loss_matches_torch(hip_lib):
    """moe_aux_loss_fwd (one launch) == ops.aux_losses (torch ops) in value
    and in its gradient w.r.t. the router partials."""
    from src.moe.ops import aux_loss_weighted, aux_losses

    g = torch.Generator(device=DEV).manual_seed(2)
    nblk, E, T, k = 37, 8, 2300, 2
    auxp = (torch.rand(nblk, E + 1, device=DEV, generator=g) * 10).requires_grad_(True)
    hist = torch.randint(0, 600, (E,), device=DEV, generator=g).int()
    lbc, zc = 1e-2, 1e-3
    lb, z = aux_losses(auxp, hist, T, k)
    ref = lbc * lb + zc * z
    (ga_ref,) = torch.autograd.grad(ref, auxp)
    aux, raw = aux_loss_weighted(auxp, hist, T, k, lbc, zc)
    (ga,) = torch.autograd.grad(aux * 3.0, auxp)
    torch.testing.assert_close(aux, ref, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(raw, torch.stack([lb, z]).detach(), rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(ga, 3.0 * ga_ref, rtol=1e-5, atol=1e-9)


# ---------------------------------------------------------------------------
# round 2: row gathers (no permuted copy) and paired backward launches
# ---------------------------------------------------------------------------
@pytest.mark.parametrize("rows_per_group", [[0, 1, 63, 64, 65, 200, 0, 130], [1000, 24, 0, 500]])
@pytest.mark.parametrize("ksplit", [0, 1, 2])
def test_grouped_gemm_gather_exact(hip_lib, rows_per_group, ksplit):
    """GEMM1 reading routed row r as token row x[tok[r]] == the GEMM on the
    permuted copy, bit for bit (integer data)."""
    from src.moe import _lib as L

    rng = np.random.default_rng(17)
    G, N, K = len(rows_per_group), 1024, 256
    offsets = np.concatenate([[0], np.cumsum(rows_per_group)]).astype(np.int32)
    R = int(offsets[-1])
    T = max(R // 2, 1) + 7
    X = _int_tensor(rng, (T, K))
    tok = rng.integers(0, T, size=R + 5).astype(np.int32)
    Bw = _int_tensor(rng, (G, N, K))
    bias = _int_tensor(rng, (G, N))
    Xt = torch.from_numpy(X).to(torch.bfloat16).to(DEV)
    tok_t = torch.from_numpy(tok).to(DEV)
    Bt = torch.from_numpy(Bw).to(torch.bfloat16).to(DEV)
    off_t = torch.from_numpy(offsets).to(DEV)
    bias_t = torch.from_numpy(bias).float().to(DEV)
    L.set_tuning("ksplit", ksplit)
    try:
        got = L.grouped_gemm_gather(Xt, tok_t, Bt, off_t, G, R + 5, N, K, 1, L.EPI_BIAS_RELU, bias=bias_t)
        ref = L.grouped_gemm(Xt[tok_t.long()].contiguous(), Bt, off_t, G, R + 5, N, K, 1, L.EPI_BIAS_RELU,
                             bias=bias_t)
        torch.cuda.synchronize()
    finally:
        L.set_tuning("ksplit", 0)
    assert torch.equal(got[:R], ref[:R])


@pytest.mark.parametrize("rows_per_group", [[0, 1, 63, 64, 65, 200, 0, 130], [1500, 40, 0, 1100]])
@pytest.mark.parametrize("epi", ["mask", "none"])
@pytest.mark.parametrize("pair", [1, 0])
def test_grouped_gemm_bwd_pair_exact(hip_lib, rows_per_group, epi, pair):
    """moe_grouped_gemm_bwd_pair (one launch, or two with gemm_pair=0) ==
    the separate dgrad and wgrad launches, bit for bit, including the wgrad
    operand gathered through a row map and split-K in both halves."""
    from src.moe import _lib as L

    rng = np.random.default_rng(23)
    G = len(rows_per_group)
    offsets = np.concatenate([[0], np.cumsum(rows_per_group)]).astype(np.int32)
    R = int(offsets[-1])
    N, K = (1024, 256) if epi == "mask" else (256, 1024)  # dH = dYp W2 (mask) / dXp = dH W1
    A = torch.from_numpy(_int_tensor(rng, (R + 3, K))).to(torch.bfloat16).to(DEV)
    Bw = torch.from_numpy(_int_tensor(rng, (G, K, N))).to(torch.bfloat16).to(DEV)
    aux = torch.from_numpy(_int_tensor(rng, (R + 3, N))).to(torch.bfloat16).to(DEV) if epi == "mask" else None
    Tt = max(R, 1) + 11
    Y = torch.from_numpy(_int_tensor(rng, (Tt, 256 if epi == "none" else N), -2, 3)).to(torch.bfloat16).to(DEV)
    tok = torch.from_numpy(rng.integers(0, Tt, size=R + 3).astype(np.int32)).to(DEV) if epi == "none" else None
    off_t = torch.from_numpy(offsets).to(DEV)
    e = L.EPI_RELU_MASK if epi == "mask" else L.EPI_NONE
    L.set_tuning("gemm_pair", pair)
    try:
        c, wc, cs = L.grouped_gemm_bwd_pair(A, Bw, off_t, G, R + 3, N, K, e, aux, A, Y, tok, out_dtype=torch.float32)
    finally:
        L.set_tuning("gemm_pair", 1)
    ref_c = L.grouped_gemm(A, Bw, off_t, G, R + 3, N, K, 0, e, aux=aux)
    Yr = Y[tok.long()].contiguous() if tok is not None else Y
    ref_wc, ref_cs = L.grouped_gemm_wgrad(A, Yr[:R + 3].contiguous() if tok is None else Yr, off_t, G)
    torch.cuda.synchronize()
    assert torch.equal(c[:R], ref_c[:R])
    assert torch.equal(wc, ref_wc) and torch.equal(cs, ref_cs)
    for _ws, cnt in L._SPLIT_WS.values():  # split-K arrival counters left at zero
        assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("rows_per_group", [[0, 1, 63, 64, 65, 200, 0, 130], [1500, 40, 0, 1100], [3000] * 4])
@pytest.mark.parametrize("wg", ["0:0", "0:3", "1:0"], ids=["dma2", "dma3", "regs"])
def test_grouped_gemm_bwd_pair_gathered(hip_lib, rows_per_group, wg):
    """The layer backward's pairs with gathered k-rows: (a) dH = gate * (dy[tok]
    W2) * mask with dW2 = bf16(gate * dy[tok])^T H (X gathered AND scaled), (b)
    dXp = dH W1 with dW1 = dH^T x[tok] (Y gathered).  The weight gradients
    equal the plain wgrad of the explicitly gathered (and bf16-scaled) rows
    bit for bit, for the LDS-DMA ring (2 or 3 stages, indices staged in LDS)
    and the register-staged body; split-K engages on the 3000-row groups."""
    from src.moe import _lib as L

    rng = np.random.default_rng(29)
    G = len(rows_per_group)
    offsets = np.concatenate([[0], np.cumsum(rows_per_group)]).astype(np.int32)
    R = int(offsets[-1])
    d, F = 256, 1024
    T = max(R, 1) // 2 + 7
    tok = torch.from_numpy(rng.integers(0, T, size=max(R, 1)).astype(np.int32)).to(DEV)
    # power-of-two gates: bf16(gate * dy) is exact and every fp32 sum below is exact, so split-K and
    # the explicit reference agree bit for bit whatever the summation order
    gate = torch.from_numpy(rng.choice([0.25, 0.5, 1.0, 2.0], size=max(R, 1)).astype(np.float32)).to(DEV)
    dy = torch.from_numpy(_int_tensor(rng, (T, d), -3, 4)).to(torch.bfloat16).to(DEV)
    x = torch.from_numpy(_int_tensor(rng, (T, d), -2, 3)).to(torch.bfloat16).to(DEV)
    h = torch.from_numpy(_int_tensor(rng, (max(R, 1), F), -2, 3)).to(torch.bfloat16).to(DEV)
    dh = torch.from_numpy(_int_tensor(rng, (max(R, 1), F), -2, 3)).to(torch.bfloat16).to(DEV)
    w2 = torch.from_numpy(_int_tensor(rng, (G, d, F))).to(torch.bfloat16).to(DEV)
    w1 = torch.from_numpy(_int_tensor(rng, (G, F, d))).to(torch.bfloat16).to(DEV)
    off_t = torch.from_numpy(offsets).to(DEV)
    dma, stages = (int(v) for v in wg.split(":"))
    L.set_tuning("wgrad_dma", dma)
    L.set_tuning("wgrad_stages", stages)
    try:
        c2, wc2, cs2 = L.grouped_gemm_bwd_pair(dy, w2, off_t, G, R, F, d, L.EPI_RELU_MASK, h, dy, h,
                                               out_dtype=torch.float32, a_gather=tok, row_scale=gate, wx_gather=tok,
                                               wx_scale=gate)
        c1, wc1, cs1 = L.grouped_gemm_bwd_pair(dh, w1, off_t, G, R, d, F, L.EPI_NONE, None, dh, x, tok,
                                               out_dtype=torch.float32)
        L.set_tuning("wgrad_dma", 1)
        L.set_tuning("wgrad_stages", 0)
        r2 = L.grouped_gemm_bwd_pair(dy, w2, off_t, G, R, F, d, L.EPI_RELU_MASK, h, dy, h, out_dtype=torch.float32,
                                     a_gather=tok, row_scale=gate, wx_gather=tok, wx_scale=gate)
    finally:
        L.set_tuning("wgrad_dma", 0)
        L.set_tuning("wgrad_stages", 0)
    dyp = (dy[tok.long()].float() * gate[:, None]).to(torch.bfloat16).contiguous()
    ref_wc2, ref_cs2 = L.grouped_gemm_wgrad(dyp, h, off_t, G)
    ref_wc1, ref_cs1 = L.grouped_gemm_wgrad(dh, x[tok.long()].contiguous(), off_t, G)
    torch.cuda.synchronize()
    assert torch.equal(wc2, ref_wc2) and torch.equal(cs2, ref_cs2)
    assert torch.equal(wc1, ref_wc1) and torch.equal(cs1, ref_cs1)
    assert torch.equal(c2[:R], r2[0][:R]) and torch.equal(wc2, r2[1])  # the dgrad half is unchanged
    for _ws, cnt in L._SPLIT_WS.values():
        assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("T,E,k,cf", [(1000, 8, 2, 0.0), (777, 16, 2, 0.0), (640, 32, 4, 1.25), (1, 4, 1, 0.0)])
def test_route_index_matches_permute(hip_lib, T, E, k, cf):
    """route_index's pos equals permute_fwd's, and src_tok inverts it: the
    gathered token rows are exactly the permuted copy."""
    from src.moe import _lib as L

    c = make_case(T, 256, E, 1024, k, max(T // 4, 1), 31)
    cap = _cap(T, k, E, cf)
    x = _bf16(c["x"]).to(DEV)
    idx, w, probs, lse, lrank, bcnt, auxp = L.router_topk_fwd(
        x, torch.from_numpy(c["wg"]).float().to(DEV), torch.from_numpy(c["ctx_bias"]).float().to(DEV),
        torch.from_numpy(c["ctx_img"]).to(DEV), max(T // 4, 1), k, True)
    rank_base, hist, offsets = L.route_scan(bcnt, cap)
    rows = T * k if cap <= 0 else min(T * k, E * cap)
    xp, pos = L.permute_fwd(x, idx, lrank, rank_base, offsets, E, cap, rows)
    pos2, tok = L.route_index(idx, lrank, rank_base, offsets, E, cap, rows)
    torch.cuda.synchronize()
    assert torch.equal(pos, pos2)
    R = int(offsets[-1])
    assert torch.equal(x[tok[:R].long()], xp[:R])


@pytest.mark.parametrize("T,E,k,cf", [(1000, 8, 2, 0.0), (777, 16, 2, 0.0), (640, 32, 4, 1.25), (1, 4, 1, 0.0),
                                      (14720, 32, 4, 1.25), (300, 64, 8, 0.0), (1300, 8, 2, 1.25)])
def test_route_dispatch_matches_scan_index_aux(hip_lib, T, E, k, cf):
    """moe_route_dispatch (one launch) == route_scan + route_index +
    aux_loss_fwd: integer outputs bit-exact, aux losses and their gradient
    coefficients equal (same fixed-order sums), row gates = topk_w at pos."""
    from src.moe import _lib as L

    tpi = max(T // 4, 1)
    c = make_case(T, 256, E, 1024, k, tpi, 37) if T <= 2000 else None
    if c is None:  # C5 encoder size: unfiltered random inputs
        g = torch.Generator(device=DEV).manual_seed(3)
        x = torch.randn((T, 256), device=DEV, generator=g).to(torch.bfloat16)
        wg = torch.randn((E, 256), device=DEV, generator=g) * 0.02
        cb = torch.randn((6, E), device=DEV, generator=g) * 0.5
        ci = torch.randint(0, 6, ((T + tpi - 1) // tpi,), device=DEV, generator=g).int()
    else:
        x = _bf16(c["x"]).to(DEV)
        wg = torch.from_numpy(c["wg"]).float().to(DEV)
        cb = torch.from_numpy(c["ctx_bias"]).float().to(DEV)
        ci = torch.from_numpy(c["ctx_img"]).to(DEV)
    cap = _cap(T, k, E, cf)
    idx, w, probs, lse, lrank, bcnt, auxp = L.router_topk_fwd(x, wg, cb, ci, tpi, k, True)
    rank_base, hist, offsets = L.route_scan(bcnt, cap)
    rows = T * k if cap <= 0 else min(T * k, E * cap)
    pos, tok = L.route_index(idx, lrank, rank_base, offsets, E, cap, rows)
    out, wcoef = L.aux_loss_fwd(auxp, hist, T, k, 1e-2, 1e-3)
    pos2, tok2, hist2, off2, gate2, out2, wcoef2 = L.route_dispatch(bcnt, idx, lrank, w, auxp, T, E, cap, rows,
                                                                    1e-2, 1e-3, row_gate=True)
    torch.cuda.synchronize()
    R = int(offsets[-1])
    assert torch.equal(hist, hist2) and torch.equal(offsets, off2) and torch.equal(pos, pos2)
    assert torch.equal(tok[:R], tok2[:R])
    assert torch.equal(out, out2) and torch.equal(wcoef, wcoef2)
    keep = pos2 >= 0
    assert torch.equal(gate2[pos2[keep].long()], w[keep])


@pytest.mark.parametrize("B,tpi,E,C", [(3, 920, 8, 6), (8, 300, 8, 6), (2, 17, 32, 4), (1, 130, 16, 1),
                                       (16, 920, 32, 5), (4, 333, 6, 3), (2, 2500, 64, 2), (8, 1, 8, 3)])
def test_router_wgrad_vs_fp64(hip_lib, B, tpi, E, C):
    """moe_router_wgrad: dWg = dlogits^T x and the per-context sums of
    dlogits (contexts repeated across images, one context unused) against an
    fp64 reference; fixed-order sums, so two launches are bitwise equal and dWg
    does not depend on whether dcb is formed."""
    from src.moe import _lib as L

    g = torch.Generator(device=DEV).manual_seed(B * tpi + E)
    T, d = B * tpi, 256
    dl = torch.randn((T, E), device=DEV, generator=g)
    x = torch.randn((T, d), device=DEV, generator=g).to(torch.bfloat16)
    ci = torch.randint(0, max(1, C - 1), (B,), device=DEV, generator=g).to(torch.int32)
    assert L.lib().moe_router_wgrad_workspace(B, tpi, E, d) == 0  # reserved since round 5
    dwg, dcb = L.router_wgrad(dl, x, ci, tpi, C)
    dwg2, dcb2 = L.router_wgrad(dl, x, ci, tpi, C)
    dwg0, dcb0 = L.router_wgrad(dl, x, None, tpi, 0)
    torch.cuda.synchronize()
    ref = dl.double().t() @ x.double()
    per_img = dl.double().view(B, tpi, E).sum(1)
    ref_cb = torch.zeros((C, E), dtype=torch.float64, device=DEV).index_add_(0, ci.long(), per_img)
    assert ((dwg.double() - ref).norm() / ref.norm()).item() < 1e-5
    assert (dcb.double() - ref_cb).abs().max().item() <= 1e-4 * max(1.0, ref_cb.abs().max().item())
    assert torch.equal(dwg, dwg2) and torch.equal(dcb, dcb2) and torch.equal(dwg, dwg0) and dcb0 is None


@pytest.mark.parametrize("gather", [False, True])
def test_grouped_gemm_bf16_bias_matches_fp32_bias(hip_lib, gather):
    """MOE_BIAS_BF16: a bf16 bias read by the kernel gives bitwise the result
    of the fp32 copy of the same values (the per-call cast it replaces)."""
    from src.moe import _lib as L

    g = torch.Generator(device=DEV).manual_seed(3)
    G, N, K, R = 4, 1024, 256, 700
    offsets = torch.tensor([0, 100, 100, 450, R], dtype=torch.int32, device=DEV)
    x = torch.randn((R, K), device=DEV, generator=g).to(torch.bfloat16)
    tok = torch.randperm(R, device=DEV, generator=g).to(torch.int32)
    w = (torch.randn((G, N, K), device=DEV, generator=g) / 16).to(torch.bfloat16)
    b16 = torch.randn((G, N), device=DEV, generator=g).to(torch.bfloat16)
    outs = []
    for b in (b16, b16.float()):
        for epi in (L.EPI_BIAS, L.EPI_BIAS_RELU):
            if gather:
                outs.append(L.grouped_gemm_gather(x, tok, w, offsets, G, R, N, K, 1, epi, bias=b))
            else:
                outs.append(L.grouped_gemm(x, w, offsets, G, R, N, K, 1, epi, bias=b))
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[2]) and torch.equal(outs[1], outs[3])
