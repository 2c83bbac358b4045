"""GPU parity of the MXFP8 expert path (config C5) against the CPU oracle.

Format (include/moe_hip.h): OCP e4m3 elements, one E8M0 exponent per 32
consecutive elements of a row, exponent = smallest e with amax <= 448 * 2^e.
Tolerances:
  quantizer / permute outputs (e4m3 bytes, exponent bytes): bit-exact;
  GEMMs on e4m3-exact integer data with per-block exponents in {0, 1, 2}
  (every fp32 sum exact): bit-exact after the one bf16 rounding -- this pins
  the lane -> (row, k-block) map of v_mfma_scale_f32_16x16x128_f8f6f4 and of its
  scale operands;
  full fp8 layer vs the oracle's MXFP8 emulation (moe_forward(mx=True)): the
  bf16 tolerance of test_gpu_kernels.py (1e-2 max|ref| + 1 bf16 ulp) on all but
  0.1% of the elements plus relative Frobenius <= 1e-2 for y and dx, weight
  gradients relative Frobenius <= 1e-2 (an H element on an e4m3 rounding
  boundary or at the ReLU edge can land on the other side after fp32 vs fp64
  accumulation: a discrete step in the few outputs that read it).
"""
from __future__ import annotations

import numpy as np
import pytest
import torch

from oracle import moe_oracle as O

pytestmark = pytest.mark.gpu
DEV = "cuda"


def _np(t):
    return t.detach().float().cpu().numpy().astype(np.float64)


def _u8(a):
    return torch.from_numpy(np.ascontiguousarray(a, dtype=np.uint8)).to(DEV)


def _bf16(a):
    return torch.from_numpy(np.asarray(O.round_bf16(a), np.float32)).to(torch.bfloat16).to(DEV)


def _mx_int_operand(rng, shape, lo=-2, hi=3, emax=2):
    """e4m3-exact integers with random per-block exponents in [0, emax]:
    returns (bytes, exponent bytes, dequantised values)."""
    q = rng.integers(lo, hi, size=shape).astype(np.float64)
    e = rng.integers(0, emax + 1, size=shape[:-1] + (shape[-1] // 32,))
    return O.e4m3_bytes(q), (e + 127).astype(np.uint8), O.mx_dequantize(q, e)


def test_quantize_mx_bitexact(hip_lib):
    from src.moe import _lib as L

    rng = np.random.default_rng(0)
    R, K = 300, 256
    x = rng.standard_normal((R, K)) * np.exp2(rng.integers(-30, 30, size=(R, 1)))
    x[5] = 0.0                                   # all-zero block row
    x[6, :32] = 2.0 ** -133                      # bf16 subnormal block
    x[7, :] = 448.0 * np.sign(x[7, :])           # amax exactly 448
    x[8, :32] = 450.0                            # just above -> next exponent
    x = O.round_bf16(x)
    q, s = L.quantize_mx(_bf16(x))
    torch.cuda.synchronize()
    qr, er = O.mx_quantize(x)
    np.testing.assert_array_equal(s.cpu().numpy(), (er + 127).astype(np.uint8))
    np.testing.assert_array_equal(q.cpu().numpy(), O.e4m3_bytes(qr))


@pytest.mark.parametrize("stages", [0, 3])
@pytest.mark.parametrize("rows_per_group", [[0, 1, 63, 64, 65, 200, 0, 130], [1000, 24, 0, 500]])
@pytest.mark.parametrize("N,K", [(1024, 256), (256, 1024), (128, 128)])
def test_grouped_gemm_mx_exact(hip_lib, stages, rows_per_group, N, K):
    from src.moe import _lib as L

    L.set_tuning("gemm_stages", stages)
    try:
        rng = np.random.default_rng(3)
        G = len(rows_per_group)
        offsets = np.concatenate([[0], np.cumsum(rows_per_group)]).astype(np.int32)
        R = int(offsets[-1])
        aq, as_, A = _mx_int_operand(rng, (R + 5, K))
        bq, bs, B = _mx_int_operand(rng, (G, N, K))
        bias = rng.integers(-3, 4, size=(G, N)).astype(np.float64)
        ref = np.zeros((R, N))
        for g in range(G):
            a, b = offsets[g], offsets[g + 1]
            ref[a:b] = A[a:b] @ B[g].T
        off_t = torch.from_numpy(offsets).to(DEV)
        args = (_u8(aq), _u8(as_), _u8(bq), _u8(bs), off_t, G, R + 5, N, K)
        C = L.grouped_gemm_mx(*args, L.EPI_NONE)
        torch.cuda.synchronize()
        np.testing.assert_array_equal(_np(C)[:R], O.round_bf16(ref))
        gid = np.repeat(np.arange(G), rows_per_group)
        ref2 = O.round_bf16(np.maximum(ref + bias[gid], 0))
        bias_t = torch.from_numpy(bias).float().to(DEV)
        C2 = L.grouped_gemm_mx(*args, L.EPI_BIAS_RELU, bias=bias_t)
        np.testing.assert_array_equal(_np(C2)[:R], ref2)
        # MXFP8 output (quantized from the bf16-rounded result)
        Cq, Cs = L.grouped_gemm_mx(*args, L.EPI_BIAS_RELU, bias=bias_t, out_mx=True)
        torch.cuda.synchronize()
        qr, er = O.mx_quantize(ref2)
        np.testing.assert_array_equal(Cs.cpu().numpy()[:R], (er + 127).astype(np.uint8))
        np.testing.assert_array_equal(Cq.cpu().numpy()[:R], O.e4m3_bytes(qr))
    finally:
        L.set_tuning("gemm_stages", 0)


@pytest.mark.parametrize("rows_per_group", [[0, 1, 63, 64, 65, 200, 0, 130], [700, 0, 33]])
@pytest.mark.parametrize("M,N", [(256, 1024), (1024, 256), (64, 128)])
def test_grouped_gemm_wgrad_mx_exact(hip_lib, rows_per_group, M, N):
    from src.moe import _lib as L

    rng = np.random.default_rng(5)
    G = len(rows_per_group)
    offsets = np.concatenate([[0], np.cumsum(rows_per_group)]).astype(np.int32)
    R = int(offsets[-1])
    X = rng.integers(-2, 3, size=(R + 3, M)).astype(np.float64)
    yq, ys, Y = _mx_int_operand(rng, (R + 3, N))
    C, cs = L.grouped_gemm_wgrad_mx(_bf16(X), _u8(yq), _u8(ys), torch.from_numpy(offsets).to(DEV), G)
    torch.cuda.synchronize()
    for g in range(G):
        a, b = offsets[g], offsets[g + 1]
        np.testing.assert_array_equal(_np(C[g]), X[a:b].T @ Y[a:b])
        np.testing.assert_array_equal(_np(cs[g]), X[a:b].sum(0))


def test_relu_mask_from_e4m3(hip_lib):
    from src.moe import _lib as L

    rng = np.random.default_rng(9)
    rows_per_group = [70, 0, 129]
    G, N, K = len(rows_per_group), 256, 128
    offsets = np.concatenate([[0], np.cumsum(rows_per_group)]).astype(np.int32)
    R = int(offsets[-1])
    A = rng.integers(-3, 4, size=(R, K)).astype(np.float64)
    Bw = rng.integers(-3, 4, size=(G, K, N)).astype(np.float64)
    hq = rng.integers(-3, 4, size=(R, N)).astype(np.float64)  # e4m3 values incl. 0 and negatives
    hb = O.e4m3_bytes(hq)
    hb[0, :4] = 0x80  # -0 does not pass the mask
    ref = np.zeros((R, N))
    for g in range(G):
        a, b = offsets[g], offsets[g + 1]
        ref[a:b] = A[a:b] @ Bw[g]
    keep = (hb != 0) & (hb < 0x80)
    C = L.grouped_gemm(_bf16(A), _bf16(Bw), torch.from_numpy(offsets).to(DEV), G, R, N, K, 0,
                       L.EPI_RELU_MASK_MX, aux=_u8(hb))
    torch.cuda.synchronize()
    np.testing.assert_array_equal(_np(C), O.round_bf16(ref * keep))


def test_permute_mx_matches_oracle(hip_lib):
    from src.moe import _lib as L

    from test_gpu_kernels import make_case

    T, d, E, F, k, tpi = 900, 256, 32, 1024, 4, 90
    c = make_case(T, d, E, F, k, tpi, 21)
    import math

    cap = int(math.ceil(1.25 * T * k / E))
    st = O.moe_forward(c["x"], c["wg"], c["ctx_bias"], c["w1"], c["b1"], c["w2"], c["b2"],
                       c["ctx_img"], tpi, k, True, cap, emulate_bf16=True)
    x = _bf16(c["x"])
    idx, w, probs, lse, lrank, bcnt, auxp = L.router_topk_fwd(
        x, torch.from_numpy(c["wg"]).float().to(DEV), torch.from_numpy(c["ctx_bias"]).float().to(DEV),
        torch.from_numpy(c["ctx_img"]).to(DEV), tpi, k, True)
    rank_base, hist, offsets = L.route_scan(bcnt, cap)
    rows = min(T * k, E * cap)
    xq, xs, pos = L.permute_fwd_mx(x, idx, lrank, rank_base, offsets, E, cap, rows)
    torch.cuda.synchronize()
    np.testing.assert_array_equal(pos.cpu().numpy(), st.pos)
    Rk = int(st.offsets[-1])
    qr, er = O.mx_quantize(st.xp)
    np.testing.assert_array_equal(xq.cpu().numpy()[:Rk], O.e4m3_bytes(qr))
    np.testing.assert_array_equal(xs.cpu().numpy()[:Rk], (er + 127).astype(np.uint8))


def _bf16_close(got, ref, what):
    """MXFP8 layer outputs vs the oracle's MX emulation:
    tests/_tolreport.check_layer_output with the mxfp8 limits (an H element on
    an e4m3 rounding boundary, or at the ReLU edge, can land on the other side
    after fp32 vs fp64 accumulation, moving the outputs that read it by an e4m3
    step), and relative Frobenius error <= 1e-2."""
    from _tolreport import check_layer_output

    check_layer_output(got, ref, what, "mxfp8")
    assert _rel_fro(got, ref) <= 1e-2, f"{what}: relative Frobenius error {_rel_fro(got, ref):.2e}"


def _rel_fro(got, ref):
    return float(np.linalg.norm(np.asarray(got) - ref) / max(np.linalg.norm(ref), 1e-12))


@pytest.mark.parametrize("T,E,k,tpi,cf,seed", [(640, 32, 4, 64, 1.25, 5), (1000, 8, 2, 250, 0.0, 2),
                                             (300, 16, 2, 100, 0.5, 7)])
def test_moe_layer_fp8_fwd_bwd(hip_lib, T, E, k, tpi, cf, seed):
    import math

    from src.moe.ops import moe_ffn_hip

    from test_gpu_kernels import make_case

    d, F = 256, 1024
    c = make_case(T, d, E, F, k, tpi, seed)
    cap = 0 if cf <= 0 else int(math.ceil(cf * T * k / E))
    rng = np.random.default_rng(200 + seed)
    dy = O.round_bf16(rng.standard_normal((T, d)))
    st = O.moe_forward(c["x"], c["wg"], c["ctx_bias"], c["w1"], c["b1"], c["w2"], c["b2"],
                       c["ctx_img"], tpi, k, True, cap, emulate_bf16=True, mx=True)
    gr = O.moe_backward(st, c["x"], c["wg"], c["w1"], c["w2"], c["ctx_img"], tpi, 6, dy,
                        g_lb=0.7, g_z=0.3, normalize=True, emulate_bf16=True)

    def P(a, dtype=torch.float32):
        return torch.from_numpy(np.asarray(a)).to(dtype).to(DEV).requires_grad_(True)

    x = P(c["x"], torch.bfloat16)
    wg, cb = P(c["wg"]), P(c["ctx_bias"])
    w1, b1, w2, b2 = P(c["w1"]), P(c["b1"]), P(c["w2"]), P(c["b2"])
    ci = torch.from_numpy(c["ctx_img"]).to(DEV)
    y, lb, z, hist = moe_ffn_hip(x, wg, cb, w1, b1, w2, b2, ci, tpi, k, True, cap, "fp8")
    loss = (y.float() * _bf16(dy).float()).sum() + 0.7 * lb + 0.3 * z
    loss.backward()
    torch.cuda.synchronize()
    np.testing.assert_array_equal(hist.cpu().numpy(), st.hist)
    _bf16_close(_np(y), st.y, "y (fp8)")
    _bf16_close(_np(x.grad), gr["dx"], "dx (fp8)")
    for name, t in [("dwg", wg), ("dctx_bias", cb), ("dw1", w1), ("db1", b1), ("dw2", w2), ("db2", b2)]:
        e = _rel_fro(_np(t.grad), gr[name])
        assert e <= 1e-2, f"{name} (fp8): relative Frobenius error {e:.2e}"
