"""MXFP8 (config C5 fp8 experts) on the CPU: the oracle's e4m3 / E8M0
restatement against torch's float8_e4m3fn conversion, and the product's
device='cpu' fp8 path (src/moe/eager.py) against the oracle.  CPU only."""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import moe_oracle as O


def test_e4m3_round_matches_torch_float8():
    rng = np.random.default_rng(0)
    v = np.concatenate([
        rng.uniform(-448, 448, 20000),
        rng.standard_normal(20000) * 2.0 ** -7,          # subnormal range (< 2^-6)
        np.arange(-448, 449, 0.5),
        [0.0, -0.0, 2 ** -9, 2 ** -10, 3 * 2 ** -10, 448.0, -448.0, 2 ** -6],
    ]).astype(np.float32).astype(np.float64)
    t = torch.from_numpy(v.astype(np.float32)).to(torch.float8_e4m3fn)
    np.testing.assert_array_equal(O.e4m3_round(v), t.float().numpy().astype(np.float64))
    np.testing.assert_array_equal(O.e4m3_bytes(O.e4m3_round(v)), t.view(torch.uint8).numpy())


def test_mx_exponent_rule():
    # smallest e with amax <= 448 * 2^e
    for amax in [1.0, 1.75, 1.7500001, 2.0, 448.0, 449.0, 3.0e-5, 1e30, 2.0 ** -140]:
        e = int(O.mx_exponent(np.float32(amax)))
        a32 = float(np.float32(amax))
        assert a32 <= 448.0 * 2.0 ** e or e == 127
        assert e == -127 or a32 > 448.0 * 2.0 ** (e - 1)
    assert int(O.mx_exponent(0.0)) == -127
    x = O.round_bf16(np.random.default_rng(1).standard_normal((16, 64)) * 1e3)
    q, e = O.mx_quantize(x)
    assert np.abs(q).max() <= 448.0
    # quantize-dequantize error is at most half an e4m3 ulp (relative 2^-4) of each block's scale
    err = np.abs(O.mx_dequantize(q, e) - x)
    assert (err <= np.repeat(np.exp2(e - 9.0), 32, axis=-1) + np.abs(x) * 2.0 ** -4).all()


def test_eager_mx_round_matches_oracle():
    from src.moe.eager import mx_round

    rng = np.random.default_rng(2)
    x = (rng.standard_normal((50, 256)) * np.exp2(rng.integers(-20, 20, (50, 1)))).astype(np.float32)
    np.testing.assert_array_equal(mx_round(torch.from_numpy(x)).numpy().astype(np.float64),
                                  O.mx_round(x.astype(np.float64)))


@pytest.mark.parametrize("k,cf", [(2, 0.0), (4, 1.25)])
def test_eager_fp8_path_matches_oracle(k, cf):
    """The product's device='cpu' fp8 experts agree with the oracle's MXFP8 emulation."""
    from src.moe.eager import moe_ffn_eager

    rng = np.random.default_rng(30 + k)
    T, d, E, F, tpi = 96, 64, 8, 128, 24
    c = dict(x=rng.standard_normal((T, d)), wg=rng.standard_normal((E, d)) * 0.5,
             ctx_bias=rng.standard_normal((6, E)) * 0.5, ctx_img=rng.integers(0, 6, T // tpi).astype(np.int32),
             w1=rng.standard_normal((E, F, d)) / 8, b1=rng.standard_normal((E, F)) * 0.1,
             w2=rng.standard_normal((E, d, F)) / 11, b2=rng.standard_normal((E, d)) * 0.1)
    for n in ("x", "wg", "ctx_bias", "w1", "b1", "w2", "b2"):
        c[n] = c[n].astype(np.float32).astype(np.float64)
    dy = rng.standard_normal((T, d))
    cap = 0 if cf <= 0 else int(np.ceil(cf * T * k / E))
    st = O.moe_forward(c["x"], c["wg"], c["ctx_bias"], c["w1"], c["b1"], c["w2"], c["b2"],
                       c["ctx_img"], tpi, k, True, cap, mx=True)
    gr = O.moe_backward(st, c["x"], c["wg"], c["w1"], c["w2"], c["ctx_img"], tpi, 6, dy,
                        g_lb=0.5, g_z=0.25, normalize=True)
    t = {n: torch.tensor(c[n], dtype=torch.float32, requires_grad=True)
         for n in ("x", "wg", "ctx_bias", "w1", "b1", "w2", "b2")}
    y, lb, z, hist = moe_ffn_eager(t["x"], t["wg"], t["ctx_bias"], t["w1"], t["b1"], t["w2"], t["b2"],
                                   torch.as_tensor(c["ctx_img"]), tpi, k, True, cap, "fp8")
    ((y * torch.tensor(dy, dtype=torch.float32)).sum() + 0.5 * lb + 0.25 * z).backward()
    np.testing.assert_array_equal(hist.numpy(), st.hist)

    def rel(a, b):
        return float(np.linalg.norm(np.asarray(a, np.float64) - b) / max(np.linalg.norm(b), 1e-12))

    assert rel(y.detach().numpy(), st.y) < 2e-3
    for a, b in [("dx", "x"), ("dwg", "wg"), ("dctx_bias", "ctx_bias"), ("dw1", "w1"), ("db1", "b1"),
                 ("dw2", "w2"), ("db2", "b2")]:
        assert rel(t[b].grad.numpy(), gr[a]) < 5e-3, a
