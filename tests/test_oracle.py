"""The oracle's hand-derived MoE backward vs an independent torch float64
autograd formulation, and the product CPU (eager) path vs the oracle.
CPU only; small sizes."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import moe_oracle as O


def _case(T=96, d=32, E=6, F=48, k=2, tpi=24, seed=0, C=6):
    rng = np.random.default_rng(seed)
    return dict(
        x=rng.standard_normal((T, d)), wg=rng.standard_normal((E, d)) * 0.5,
        ctx_bias=rng.standard_normal((C, E)) * 0.5, ctx_img=rng.integers(0, C, T // tpi).astype(np.int32),
        w1=rng.standard_normal((E, F, d)) / np.sqrt(d), b1=rng.standard_normal((E, F)) * 0.1,
        w2=rng.standard_normal((E, d, F)) / np.sqrt(F), b2=rng.standard_normal((E, d)) * 0.1,
        dy=rng.standard_normal((T, d)), tpi=tpi, k=k)


def _torch_ref(c, cap, g_lb, g_z):
    """Independent formulation: dense masks instead of index lists, autograd for grads."""
    t = {n: torch.tensor(c[n], dtype=torch.float64, requires_grad=True)
         for n in ("x", "wg", "ctx_bias", "w1", "b1", "w2", "b2")}
    T = c["x"].shape[0]
    E = c["wg"].shape[0]
    k = c["k"]
    img = torch.arange(T) // c["tpi"]
    logits = t["x"] @ t["wg"].T + t["ctx_bias"][torch.as_tensor(c["ctx_img"]).long()[img]]
    probs = torch.softmax(logits, -1)
    lse = torch.logsumexp(logits, -1)
    idx = torch.sort(logits.detach(), dim=-1, descending=True, stable=True).indices[:, :k]
    psel = probs.gather(1, idx)
    w = psel / psel.sum(-1, keepdim=True) if k > 1 else psel
    # capacity via the oracle's integer dispatch (integer part is not differentiable)
    pos, hist, _ = O.dispatch_indices(idx.numpy(), E, cap)
    keep = torch.as_tensor(pos >= 0)
    y = torch.zeros_like(t["x"])
    for j in range(k):
        for e in range(E):
            m = (idx[:, j] == e) & keep[:, j]
            if m.any():
                h = torch.relu(t["x"][m] @ t["w1"][e].T + t["b1"][e])
                ye = h @ t["w2"][e].T + t["b2"][e]
                y = y.index_add(0, torch.nonzero(m)[:, 0], w[m, j : j + 1] * ye)
    f = torch.as_tensor(hist, dtype=torch.float64) / (T * k)
    lb = E * (f * probs.mean(0)).sum()
    z = (lse ** 2).mean()
    loss = (y * torch.tensor(c["dy"])).sum() + g_lb * lb + g_z * z
    loss.backward()
    return y.detach().numpy(), float(lb), float(z), {n: v.grad.numpy() for n, v in t.items()}


@pytest.mark.parametrize("k,cf,seed", [(1, 0.0, 0), (2, 0.0, 1), (2, 1.0, 2), (3, 0.6, 3)])
def test_oracle_backward_matches_autograd(k, cf, seed):
    c = _case(k=k, seed=seed)
    T, E = c["x"].shape[0], c["wg"].shape[0]
    cap = 0 if cf <= 0 else int(np.ceil(cf * T * k / E))
    g_lb, g_z = 0.37, 0.21
    st = O.moe_forward(c["x"], c["wg"], c["ctx_bias"], c["w1"], c["b1"], c["w2"], c["b2"],
                       c["ctx_img"], c["tpi"], k, True, cap)
    gr = O.moe_backward(st, c["x"], c["wg"], c["w1"], c["w2"], c["ctx_img"], c["tpi"], 6, c["dy"],
                        g_lb=g_lb, g_z=g_z, normalize=True)
    y, lb, z, tg = _torch_ref(c, cap, g_lb, g_z)
    np.testing.assert_allclose(st.y, y, rtol=1e-10, atol=1e-10)
    assert abs(st.lb - lb) < 1e-12 and abs(st.z - z) < 1e-12
    pairs = [("dx", "x"), ("dwg", "wg"), ("dctx_bias", "ctx_bias"), ("dw1", "w1"), ("db1", "b1"),
             ("dw2", "w2"), ("db2", "b2")]
    for a, b in pairs:
        np.testing.assert_allclose(gr[a], tg[b], rtol=1e-9, atol=1e-9, err_msg=a)


def test_dispatch_slot_major_priority():
    # 4 tokens, k=2, 2 experts, cap 2: every top-1 choice outranks any top-2 choice
    idx = np.array([[0, 1], [1, 0], [0, 1], [0, 1]])
    pos, hist, offsets = O.dispatch_indices(idx, 2, 2)
    assert hist.tolist() == [4, 4]
    assert offsets.tolist() == [0, 2, 4]
    # expert 0 slot-0 tokens: 0, 2, 3 -> ranks 0, 1, 2 (token 3 dropped); slot-1 token 1 dropped
    assert pos.tolist() == [[0, 3], [2, -1], [1, -1], [-1, -1]]


def test_topk_tie_break_lowest_index():
    x = np.zeros((1, 4))
    wg = np.zeros((4, 4))
    _, probs, _, idx, w = O.router_forward(x, wg, None, None, 1, 2, True)
    assert idx.tolist() == [[0, 1]]
    np.testing.assert_allclose(w, [[0.5, 0.5]])


def test_round_bf16():
    v = np.array([1.0, 1.00390625, 1.005859375, -3.14159, 0.0, np.inf])
    r = O.round_bf16(v)
    ref = torch.tensor(v, dtype=torch.float32).to(torch.bfloat16).double().numpy()
    np.testing.assert_array_equal(r, ref)


@pytest.mark.parametrize("k,cf", [(1, 0.0), (2, 0.0), (2, 1.0)])
def test_eager_cpu_path_matches_oracle(k, cf):
    """The product's device='cpu' path (C1 plumbing) agrees with the oracle."""
    from src.moe.eager import moe_ffn_eager

    c = _case(k=k, seed=10 + k)
    T, E = c["x"].shape[0], c["wg"].shape[0]
    cap = 0 if cf <= 0 else int(np.ceil(cf * T * k / E))
    st = O.moe_forward(c["x"], c["wg"], c["ctx_bias"], c["w1"], c["b1"], c["w2"], c["b2"],
                       c["ctx_img"], c["tpi"], k, True, cap)
    gr = O.moe_backward(st, c["x"], c["wg"], c["w1"], c["w2"], c["ctx_img"], c["tpi"], 6, c["dy"],
                        g_lb=0.5, g_z=0.25, normalize=True)
    t = {n: torch.tensor(c[n], dtype=torch.float32, requires_grad=True)
         for n in ("x", "wg", "ctx_bias", "w1", "b1", "w2", "b2")}
    y, lb, z, hist = moe_ffn_eager(t["x"], t["wg"], t["ctx_bias"], t["w1"], t["b1"], t["w2"], t["b2"],
                                   torch.as_tensor(c["ctx_img"]), c["tpi"], k, True, cap)
    ((y * torch.tensor(c["dy"], dtype=torch.float32)).sum() + 0.5 * lb + 0.25 * z).backward()
    np.testing.assert_allclose(y.detach().numpy(), st.y, rtol=1e-4, atol=1e-4)
    np.testing.assert_array_equal(hist.numpy(), st.hist)
    for a, b in [("dx", "x"), ("dwg", "wg"), ("dctx_bias", "ctx_bias"), ("dw1", "w1"), ("db1", "b1"),
                 ("dw2", "w2"), ("db2", "b2")]:
        np.testing.assert_allclose(t[b].grad.numpy(), gr[a], rtol=2e-4, atol=2e-4, err_msg=a)
