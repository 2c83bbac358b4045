"""The fused expert FFN forward (moe_expert_ffn_fwd, csrc/expert_ffn.hip)
against the two-launch path it replaces (GEMM1 with the row gather + ReLU,
GEMM2) and a torch fp32 reference.

Tolerances: with small-integer data every fp32 sum is exact in any order, so
H and Yp must equal the two-launch outputs bit for bit.  H is bit-exact for
any data (the same MFMA accumulation order over K = 256 as GEMM1).  Yp on
random data: the two F halves of every chunk accumulate separately and are
added once, so it is compared with the fp32 reference (bf16(H) W2^T + b2) at
1e-2 of max|ref| + 1 bf16 ulp per element, and its relative Frobenius error
must not exceed 1.5x the two-launch path's + 1e-4.
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _ints(rng, shape, lo, hi):
    return torch.from_numpy(rng.integers(lo, hi, size=shape).astype(np.float32))


def _two_launch(L, x, tok, w1, b1, w2, b2, off, G, R):
    F, d = w1.shape[1], w1.shape[2]
    if tok is not None:
        h = L.grouped_gemm_gather(x, tok, w1, off, G, R, F, d, 1, L.EPI_BIAS_RELU, bias=b1)
    else:
        h = L.grouped_gemm(x, w1, off, G, R, F, d, 1, L.EPI_BIAS_RELU, bias=b1)
    yp = L.grouped_gemm(h, w2, off, G, R, d, F, 1, L.EPI_BIAS, bias=b2)
    return h, yp


@pytest.mark.parametrize("rows_per_group", [[0, 1, 63, 64, 65, 200, 0, 130], [1500, 40, 0, 1100],
                                            [7] * 32, [3000]])
@pytest.mark.parametrize("gather", [True, False])
@pytest.mark.parametrize("bias_bf16", [False, True])
@pytest.mark.parametrize("F", [1024, 384])
def test_expert_ffn_exact_vs_two_launch(hip_lib, rows_per_group, gather, bias_bf16, F):
    from src.moe import _lib as L

    rng = np.random.default_rng(5)
    G, d = len(rows_per_group), 256
    assert L.expert_ffn_supported(G, F, d)
    offsets = np.concatenate([[0], np.cumsum(rows_per_group)]).astype(np.int32)
    R = int(offsets[-1])
    T = max(R // 2, 1) + 3
    # |H| <= 2 * 256 before the bf16 rounding; |Yp| sums <= 512 * F < 2^24: exact fp32 in any order
    x = _ints(rng, (T if gather else R + 5, d), -2, 3).to(torch.bfloat16).to(DEV)
    tok = torch.from_numpy(rng.integers(0, T, size=R + 5).astype(np.int32)).to(DEV) if gather else None
    w1 = _ints(rng, (G, F, d), -1, 2).to(torch.bfloat16).to(DEV)
    w2 = _ints(rng, (G, d, F), -1, 2).to(torch.bfloat16).to(DEV)
    bdt = torch.bfloat16 if bias_bf16 else torch.float32
    b1 = _ints(rng, (G, F), -8, 9).to(bdt).to(DEV)
    b2 = _ints(rng, (G, d), -8, 9).to(bdt).to(DEV)
    off = torch.from_numpy(offsets).to(DEV)
    h, yp = L.expert_ffn_fwd(x, tok, w1, b1, w2, b2, off, G, R + 5)
    h_ref, yp_ref = _two_launch(L, x, tok, w1, b1, w2, b2, off, G, R + 5)
    torch.cuda.synchronize()
    assert torch.equal(h[:R], h_ref[:R])
    assert torch.equal(yp[:R], yp_ref[:R])
    # rows past offsets[G] are never written (the launch's row bound is a host upper bound)
    assert h.shape == (R + 5, F) and yp.shape == (R + 5, d)


@pytest.mark.parametrize("T,E,k", [(8 * 920, 8, 2), (8 * 300, 8, 2), (16 * 300, 32, 4), (2 * 400, 4, 1)])
def test_expert_ffn_random_vs_fp32(hip_lib, T, E, k):
    """C2 encoder / decoder, C5 (bf16) and C1 layer shapes with a random
    expert-major routing of every token k times."""
    from src.moe import _lib as L

    g = torch.Generator().manual_seed(T + E)
    d, F = 256, 1024
    R = T * k
    counts = torch.distributions.Multinomial(R, torch.ones(E)).sample().long()
    offsets = torch.cat([torch.zeros(1, dtype=torch.long), counts.cumsum(0)]).int()
    x = torch.randn(T, d, generator=g).to(torch.bfloat16)
    tok = torch.randint(0, T, (R,), generator=g).int()
    w1 = (torch.randn(E, F, d, generator=g) / 16).to(torch.bfloat16)
    w2 = (torch.randn(E, d, F, generator=g) / 32).to(torch.bfloat16)
    b1 = torch.randn(E, F, generator=g) * 0.1
    b2 = torch.randn(E, d, generator=g) * 0.1
    xd, tokd, w1d, w2d, b1d, b2d, offd = (t.to(DEV) for t in (x, tok, w1, w2, b1, b2, offsets))
    h, yp = L.expert_ffn_fwd(xd, tokd, w1d, b1d, w2d, b2d, offd, E, R)
    h2, yp2 = _two_launch(L, xd, tokd, w1d, b1d, w2d, b2d, offd, E, R)
    torch.cuda.synchronize()
    assert torch.equal(h, h2)
    ref = torch.empty(R, d)
    hf = h.float().cpu()
    off = offsets.tolist()
    for e in range(E):
        a, b = off[e], off[e + 1]
        ref[a:b] = hf[a:b] @ w2[e].float().T + b2[e]
    got, two = yp.float().cpu(), yp2.float().cpu()
    tol = 1e-2 * ref.abs().max() + ref.abs() * 2.0 ** -8
    assert ((got - ref).abs() <= tol).all()
    rel = float((got - ref).norm() / ref.norm())
    rel2 = float((two - ref).norm() / ref.norm())
    assert rel <= 1.5 * rel2 + 1e-4, (rel, rel2)


def test_expert_ffn_rejects_bad_shapes(hip_lib):
    from src.moe import _lib as L

    assert not L.expert_ffn_supported(8, 1000, 256)
    assert not L.expert_ffn_supported(8, 1024, 128)
    assert not L.expert_ffn_supported(65, 1024, 256)
    x = torch.zeros(4, 256, dtype=torch.bfloat16, device=DEV)
    w1 = torch.zeros(2, 1024, 256, dtype=torch.bfloat16, device=DEV)
    w2 = torch.zeros(2, 256, 1024, dtype=torch.bfloat16, device=DEV)
    off = torch.tensor([0, 2, 4], dtype=torch.int32, device=DEV)
    with pytest.raises(L.MoEKernelError):
        L.expert_ffn_fwd(x, None, w1, torch.zeros(2, 1024, device=DEV), w2,
                         torch.zeros(2, 256, device=DEV, dtype=torch.bfloat16), off, 2, 4)


@pytest.mark.parametrize("W,El,S", [(1, 16, 1840), (4, 2, 37), (8, 4, 5), (2, 1, 1)])
def test_ep_compaction_matches_torch_map(hip_lib, W, El, S):
    """moe_ep_compaction == ep.compaction_map (the torch index chain it
    replaces) on random received counts, incl. counts above S (capped)."""
    from src.moe import _lib as L
    from src.moe.ep import compaction_map

    g = torch.Generator().manual_seed(W * 100 + El)
    cnt = torch.randint(0, S + 3, (W, El), generator=g).int()
    E = W * El
    hist = torch.randint(0, 2 * S + 1, (E,), generator=g).int()
    g0 = L.ep_compaction(cnt.to(DEV), hist.to(DEV), S)[0]
    g0.fill_(-7)  # every entry must be (re)written: the map is allocated uninitialised (the
    del g0        # caching allocator hands this block back to the next call)
    gather, offs, ovf = L.ep_compaction(cnt.to(DEV), hist.to(DEV), S)
    g_ref, _inv, o_ref = compaction_map(cnt.clamp(max=S).to(torch.int64), S)
    torch.cuda.synchronize()
    n = int(o_ref[-1])
    assert torch.equal(offs.cpu(), o_ref.int())
    assert torch.equal(gather[:n].cpu(), g_ref[:n].cpu())
    assert bool((gather[n:] == 0).all())  # the tail points at received row 0
    assert int(ovf[0]) == int((hist - S).clamp(min=0).sum())


@pytest.mark.parametrize("rows_per_group", [[0, 1, 63, 64, 65, 200, 0, 130], [1500, 40, 0, 1100]])
def test_scatter_outputs_match_gather_after(hip_lib, rows_per_group):
    """Output-row scatter (EP received layout): the fused FFN's Yp and the
    paired dgrad's C written through c_rows equal the unscattered outputs
    moved by index, bit for bit."""
    from src.moe import _lib as L

    rng = np.random.default_rng(9)
    G, d, F = len(rows_per_group), 256, 1024
    offsets = np.concatenate([[0], np.cumsum(rows_per_group)]).astype(np.int32)
    R = int(offsets[-1])
    n_out = 2 * R + 16
    rows = torch.from_numpy(rng.permutation(n_out)[:R].astype(np.int32)).to(DEV)
    x = _ints(rng, (n_out, d), -2, 3).to(torch.bfloat16).to(DEV)
    w1 = _ints(rng, (G, F, d), -1, 2).to(torch.bfloat16).to(DEV)
    w2 = _ints(rng, (G, d, F), -1, 2).to(torch.bfloat16).to(DEV)
    b1 = _ints(rng, (G, F), -8, 9).to(DEV)
    b2 = _ints(rng, (G, d), -8, 9).to(DEV)
    off = torch.from_numpy(offsets).to(DEV)
    h, ys = L.expert_ffn_fwd(x, rows, w1, b1, w2, b2, off, G, R, yp_rows=rows, yp_n=n_out)
    h2, y2 = L.expert_ffn_fwd(x, rows, w1, b1, w2, b2, off, G, R)
    dy = _ints(rng, (n_out, d), -2, 3).to(torch.bfloat16).to(DEV)
    dh, _, _ = L.grouped_gemm_bwd_pair(dy, w2, off, G, R, F, d, L.EPI_RELU_MASK, h, dy, h, a_gather=rows,
                                       wx_gather=rows)
    dxs, _, _ = L.grouped_gemm_bwd_pair(dh, w1, off, G, R, d, F, L.EPI_NONE, None, dh, x, rows, c_rows=rows,
                                        c_n=n_out)
    dx2, _, _ = L.grouped_gemm_bwd_pair(dh, w1, off, G, R, d, F, L.EPI_NONE, None, dh, x, rows)
    torch.cuda.synchronize()
    assert torch.equal(h, h2)
    idx = rows.long()
    assert ys.shape == (n_out, d) and dxs.shape == (n_out, d)
    assert torch.equal(ys[idx], y2[:R])
    assert torch.equal(dxs[idx], dx2[:R])
    # the two-launch EP forward: GEMM1 gathering, GEMM2 scattering (moe_grouped_gemm_scatter)
    hg = L.grouped_gemm_gather(x, rows, w1, off, G, R, F, d, 1, L.EPI_BIAS_RELU, bias=b1)
    yg = L.grouped_gemm_scatter(hg, w2, off, G, R, d, F, 1, L.EPI_BIAS, rows,
                                torch.empty((n_out, d), dtype=torch.bfloat16, device=DEV), bias=b2)
    torch.cuda.synchronize()
    assert torch.equal(hg[:R], h[:R])
    assert torch.equal(yg[idx], y2[:R])


@pytest.mark.parametrize("rows_per_group", [[600] * 8, [1840] * 8, [1900, 300, 0, 650, 1, 64, 1200, 85],
                                            [0, 0, 0, 5], [3000, 10, 10, 10, 10, 10, 10, 10]],
                         ids=["dec", "enc", "skew", "sparse", "hot"])
@pytest.mark.parametrize("out_bf16", [True, False])
def test_expert_ffn_bwd_equals_paired_launches(hip_lib, rows_per_group, out_bf16):
    """moe_expert_ffn_bwd (dH, then {dXp, dW2, dW1} in one grid) against the
    two paired launches it replaces ({dH, dW2}, {dXp, dW1}): the same bodies
    summing in the same order, so every output is bitwise equal -- at the C2
    decoder / encoder shapes (the encoder's weight gradients split-K), skewed
    and empty experts."""
    from src.moe import _lib as L

    g = torch.Generator().manual_seed(sum(rows_per_group) + len(rows_per_group))
    G, d, F = len(rows_per_group), 256, 1024
    offsets = torch.tensor(np.concatenate([[0], np.cumsum(rows_per_group)]).astype(np.int32), device=DEV)
    R = int(offsets[-1])
    T = max(R // 2, 1)
    dy = (torch.randn(T, d, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    x = torch.randn(T, d, generator=g).to(torch.bfloat16).to(DEV)
    tok = torch.randint(0, T, (R,), generator=g, dtype=torch.int32).to(DEV)
    gate = torch.rand(R, generator=g).to(DEV)
    h = torch.relu(torch.randn(R, F, generator=g)).to(torch.bfloat16).to(DEV)
    w1 = (torch.randn(G, F, d, generator=g) * 0.05).to(torch.bfloat16).to(DEV)
    w2 = (torch.randn(G, d, F, generator=g) * 0.03).to(torch.bfloat16).to(DEV)
    odt = torch.bfloat16 if out_bf16 else torch.float32
    dh, dxp, dW1, db1, dW2, db2 = L.expert_ffn_bwd(dy, tok, gate, x, h, w1, w2, offsets, G, R, out_dtype=odt)
    rdh, rdW2, rdb2 = L.grouped_gemm_bwd_pair(dy, w2, offsets, G, R, F, d, L.EPI_RELU_MASK, h, dy, h, out_dtype=odt,
                                              a_gather=tok, row_scale=gate, wx_gather=tok, wx_scale=gate)
    rdxp, rdW1, rdb1 = L.grouped_gemm_bwd_pair(rdh, w1, offsets, G, R, d, F, L.EPI_NONE, None, rdh, x, tok,
                                               out_dtype=odt)
    torch.cuda.synchronize()
    assert torch.equal(dh[:R], rdh[:R])
    assert torch.equal(dxp[:R], rdxp[:R])
    for got, ref, n in ((dW1, rdW1, "dW1"), (db1, rdb1, "db1"), (dW2, rdW2, "dW2"), (db2, rdb2, "db2")):
        assert torch.equal(got, ref), n
    # and against fp32 torch: dYp = bf16(gate dy[tok]); dH = relu'(H) (dYp W2); dXp = dH W1
    lo = offsets.cpu().tolist()
    dyp = (gate[:, None] * dy[tok.long()].float()).to(torch.bfloat16).float()
    for e in range(G):
        a, b = lo[e], lo[e + 1]
        if b <= a:
            assert float(dW1[e].float().abs().max()) == 0.0 and float(dW2[e].float().abs().max()) == 0.0
            continue
        ref_w2 = dyp[a:b].t() @ h[a:b].float()
        assert (dW2[e].float() - ref_w2).norm() <= 5e-3 * ref_w2.norm() + 1e-6
