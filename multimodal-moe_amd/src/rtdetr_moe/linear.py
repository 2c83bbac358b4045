"""Linear layer for inputs with a very large row count (the decoder's value
projection over all B*S encoder-memory tokens: 154,560 rows at 1280x736,
batch 8).

The weight gradient dW = dY^T X reduces over all rows.  As one GEMM with a
256x256 output, hipBLASLt picks a tiling that puts only 16 workgroups on the
chip (~380 us on MI355X); split into S row chunks as a batched GEMM
(S independent [256, K/S] x [K/S, 256] products, then a fp32 sum over S) it
fills the chip (~50 us, tools/mm_probe.py).  Forward and input gradient are
the usual GEMMs.  Every linear layer of the RT-DETR body is a TokenLinear on
the GPU: its bias gradient comes from rtdetr_bias_grad (deterministic
two-launch column sum) instead of torch's reduce kernel.
"""
from __future__ import annotations

import contextlib
import math
import os

import torch
import torch.nn.functional as F
from torch import nn

BIG_ROWS = 65536  # below this, the plain GEMM is already well shaped
DENSE_WGRAD_ROWS = [512]  # from this many rows, conforming shapes use libmoe_hip's wgrad (list: A/B switch)
# GraphedStep defers conforming dense weight gradients to one batched launch
# after the backward (MOE_DEFER_WGRAD=0: one launch per layer, as before)
DEFER_WGRAD = [os.environ.get("MOE_DEFER_WGRAD", "1") != "0"]
# the narrow heads' gradients deferred too, batched into one launch pair
# (MOE_NARROW_DEFER=0: one launch pair per head, as before)
NARROW_DEFER = [os.environ.get("MOE_NARROW_DEFER", "1") != "0"]
# narrow heads (N <= 8 outputs, or K <= 8 inputs) through rtdetr_linear_narrow_fwd /
# _dgrad instead of hipBLASLt's 1-8-column GEMMs + a ReLU (backward) launch
NARROW_LINEAR = [os.environ.get("MOE_NARROW_LINEAR", "1") != "0"]


def _narrow_fwd_ok(x, w, b):
    from ..moe import _lib as L

    return (NARROW_LINEAR[0] and x.is_cuda and x.dtype == w.dtype == torch.bfloat16 and x.numel() > 0
            and (b is None or b.dtype in (torch.bfloat16, torch.float32)) and L.linear_narrow_ok(w.shape[1], w.shape[0]))


def _narrow_dgrad_ok(g2, w):
    return (NARROW_LINEAR[0] and g2.is_cuda and g2.dtype == w.dtype == torch.bfloat16 and w.shape[0] <= 8
            and w.shape[1] % 8 == 0 and g2.shape[0] > 0)
_ACTIVE: list = [None]  # the DeferredWgrad collecting during a backward, or None


def _row_target(t: torch.Tensor):
    """(leaf parameter, first row) of a weight / bias that is the parameter
    itself or a contiguous row slice of it (TokenSelfAttention's in_proj
    slices); None otherwise."""
    if t.is_leaf:
        return t, 0
    base = t._base
    if base is None or not base.is_leaf or not t.is_contiguous() or not base.is_contiguous():
        return None
    if t.dim() != base.dim() or t.shape[1:] != base.shape[1:]:
        return None
    row = t[0].numel() if t.dim() > 1 else 1
    off = t.storage_offset() - base.storage_offset()
    if off % row != 0:
        return None
    return base, off // row


class DeferredWgrad:
    """Dense weight + bias gradients collected during one backward and computed
    afterwards in as few launches as possible (rtdetr_linear_wgrad_batch: up to
    24 layers of mixed shapes per launch, each with its rows split so that the
    batch fills the chip).  One at a time, every such gradient is a short
    split-K GEMM whose fixed cost -- launch, first tile, split-K merge -- is most
    of its ~15 us (54 per C2 step); batched, the fixed cost is paid twice.
    ``flush()`` returns {id(parameter): gradient} for the leaf parameters."""

    def __init__(self):
        self.items = []  # (gy, x, out dtype, (weight leaf, row), (bias leaf, row))
        self.narrow = []  # the same for narrow heads (rtdetr_linear_wgrad_narrow_batch)
        self.ln = []  # (row-pass partials fp32 [P, 2d], weight leaf, bias leaf): LayerNorm finals

    def add(self, gy, x, odt, wt, bt):
        self.items.append((gy, x, odt, wt, bt))

    def add_ln(self, parts, w, b):
        self.ln.append((parts, w, b))

    def _flush_ln(self):
        """Every deferred LayerNorm's [dgamma; dbeta] in one launch
        (rtdetr_add_layer_norm_final_batch) instead of one final per norm."""
        from ..moe import _lib as L

        out, jobs = {}, []
        for parts, w, b in self.ln:
            dwb = torch.empty((2, w.shape[0]), dtype=w.dtype, device=parts.device)
            jobs.append((parts, dwb))
            for p_, g in ((w, dwb[0]), (b, dwb[1])):
                out[id(p_)] = g if id(p_) not in out else out[id(p_)] + g  # (a norm applied twice)
        self.ln = []
        if jobs:
            L.add_layer_norm_final_batch(jobs)
        return out

    def add_narrow(self, gy, x, odt, wt, bt):
        self.narrow.append((gy, x, odt, wt, bt))

    def _flush_narrow(self):
        """The narrow heads' gradients in one launch pair per 32 problems: a
        head applied several times (the query position head, once per decoder
        layer) is one group whose gradient sums its uses in fp32 (rounded
        once), instead of one gradient per use summed by autograd."""
        from ..moe import _lib as L

        keys = {}
        for gy, x, odt, (wp, _), (bp, _) in self.narrow:
            k = (id(wp), id(bp), odt)
            if k not in keys:
                keys[k] = [wp, bp, odt, []]
            keys[k][3].append((gy, x))
        self.narrow = []
        out, by_dtype = {}, {}
        for wp, bp, odt, probs in keys.values():
            dw = torch.empty(wp.shape, dtype=odt, device=wp.device)
            db = torch.empty(bp.shape, dtype=odt, device=wp.device)
            by_dtype.setdefault(odt, []).append((probs, dw, db))
            out[id(wp)], out[id(bp)] = dw, db
        for odt, groups in by_dtype.items():
            L.linear_wgrad_narrow_batch(groups, odt)
        return out

    def flush(self):
        from ..moe import _lib as L

        if not self.items:
            out = self._flush_narrow() if self.narrow else {}
            if self.ln:
                out.update(self._flush_ln())
            return out
        # a parameter whose rows receive more than one layer's gradient (a
        # layer applied several times, e.g. a shared head) is summed in fp32
        # and rounded once; the others are written in place, in their dtype
        seen, shared = set(), set()
        for gy, x, odt, wt, bt in self.items:
            for p_, r0 in (wt, bt):
                if (id(p_), r0) in seen:
                    shared.add(id(p_))
                seen.add((id(p_), r0))
        # rows each parameter receives: a buffer whose rows are all written by
        # the kernel needs no zero fill
        rows = {}
        for gy, x, odt, (wp, wr), (bp, br) in self.items:
            for p_, r0 in ((wp, wr), (bp, br)):
                rows.setdefault(id(p_), []).append((r0, r0 + gy.shape[1]))

        def covered(p_):
            spans = sorted(rows[id(p_)])
            end = 0
            for a, b in spans:
                if a != end:
                    return False
                end = b
            return end == p_.shape[0]

        grads, acc = {}, {}
        direct = {torch.bfloat16: [], torch.float32: []}
        summed = []
        # a shared layer whose every use covers its whole weight and bias (a
        # head applied once per decoder layer): each use's fp32 gradient goes
        # to its own slot of a stacked buffer, summed once over the uses
        # (one reduction instead of a zero fill and one add per use)
        uses = {}
        for gy, x, odt, (wp, wr), (bp, br) in self.items:
            key = (id(wp), id(bp))
            full = wr == 0 and br == 0 and gy.shape[1] == wp.shape[0] == bp.shape[0]
            u = uses.setdefault(key, [0, True, wp, bp, odt])
            u[0] += 1
            u[1] = u[1] and full and id(wp) in shared and id(bp) in shared
        stacked = {}
        for key, (n, ok, wp, bp, odt) in uses.items():
            if ok and n > 1 and sum(1 for k2 in uses if id(wp) in k2 or id(bp) in k2) == 1:
                stacked[key] = [torch.empty((n,) + tuple(wp.shape), dtype=torch.float32, device=wp.device),
                                torch.empty((n,) + tuple(bp.shape), dtype=torch.float32, device=wp.device), 0, odt]
        for gy, x, odt, (wp, wr), (bp, br) in self.items:
            M, N = gy.shape[1], x.shape[1]
            st = stacked.get((id(wp), id(bp)))
            if st is not None:
                direct[torch.float32].append((gy, x, st[0][st[2]], st[1][st[2]]))
                st[2] += 1
                continue
            for p_ in (wp, bp):
                if id(p_) in shared:
                    if id(p_) not in acc:
                        acc[id(p_)] = (torch.zeros(p_.shape, dtype=torch.float32, device=gy.device), odt)
                elif id(p_) not in grads:
                    alloc = torch.empty if covered(p_) else torch.zeros
                    grads[id(p_)] = alloc(p_.shape, dtype=odt, device=gy.device)
            if id(wp) in shared or id(bp) in shared:
                dw = torch.empty((M, N), dtype=torch.float32, device=gy.device)
                db = torch.empty((M,), dtype=torch.float32, device=gy.device)
                direct[torch.float32].append((gy, x, dw, db))
                summed.append((dw, db, wp, wr, bp, br, odt))
            else:
                direct[odt].append((gy, x, grads[id(wp)][wr:wr + M], grads[id(bp)][br:br + M]))
        for dt, batch in direct.items():
            if batch:
                L.linear_wgrad_batch(batch, dt)
        for dw, db, wp, wr, bp, br, odt in summed:
            for p_, r0, part in ((wp, wr, dw), (bp, br, db)):
                if id(p_) in acc:
                    acc[id(p_)][0][r0:r0 + part.shape[0]] += part
                else:
                    grads[id(p_)][r0:r0 + part.shape[0]] += part.to(odt)
        for k, (a, odt) in acc.items():
            grads[k] = a.to(odt)
        for (kw, kb), (bw, bb, _, odt) in stacked.items():
            grads[kw] = bw.sum(0).to(odt)
            grads[kb] = bb.sum(0).to(odt)
        self.items.clear()
        extra = {}
        if self.narrow:
            extra.update(self._flush_narrow())
        if self.ln:
            extra.update(self._flush_ln())
        for k, g in extra.items():
            grads[k] = g if k not in grads else grads[k] + g.to(grads[k].dtype)
        return grads


@contextlib.contextmanager
def deferred_weight_grads():
    """Collect conforming TokenLinear weight gradients during the backward run
    inside this context (the collector's ``flush()`` computes them)."""
    d = DeferredWgrad() if DEFER_WGRAD[0] else None
    prev = _ACTIVE[0]
    _ACTIVE[0] = d
    try:
        yield d
    finally:
        _ACTIVE[0] = prev


def merge_deferred(params, grads, deferred: DeferredWgrad | None):
    """grads (torch.autograd.grad's output for params) with the deferred
    gradients flushed in: substituted where autograd had none, added where a
    parameter also received a regular gradient."""
    if deferred is None:
        return list(grads)
    extra = deferred.flush()
    out = []
    for p, g in zip(params, grads):
        e = extra.get(id(p))
        if e is None:
            out.append(g)
        elif g is None:
            out.append(e.to(p.dtype) if e.dtype != p.dtype else e)
        else:
            out.append(g + e.to(g.dtype))
    return out


def chunked_wgrad(gy: torch.Tensor, x: torch.Tensor, target_chunk: int = 2560) -> torch.Tensor:
    """sum_r gy[r, :]^T x[r, :] -> fp32 [m, n] as a batched GEMM over row chunks."""
    K, m = gy.shape
    n = x.shape[1]
    S = max(1, min(256, K // target_chunk))
    kc = K // S
    head = S * kc
    out = torch.bmm(gy[:head].view(S, kc, m).transpose(1, 2), x[:head].view(S, kc, n)).sum(0, dtype=torch.float32)
    if head < K:
        out += gy[head:].t().float().mm(x[head:].float())
    return out


def bias_grad(g2: torch.Tensor, dtype: torch.dtype) -> torch.Tensor:
    """Column sum of the bf16 output gradient [M, N] in the bias dtype: the HIP
    kernel pair rtdetr_bias_grad (fixed-order fp32 accumulation, two launches)
    on bf16 CUDA gradients; torch's sum elsewhere (fp32 layers)."""
    M, N = g2.shape
    if not (g2.is_cuda and g2.dtype == torch.bfloat16 and dtype in (torch.bfloat16, torch.float32)
            and M > 0 and (N % 8 == 0 and N <= 2048 or N <= 256)):
        return g2.sum(0, dtype=torch.float32).to(dtype)
    from ..moe import _lib as L

    if N % 8 == 0 and g2.data_ptr() % 16 != 0:
        g2 = g2.clone()  # 16-B row vectors
    lib = L.lib()
    P = int(lib.rtdetr_bias_grad_parts(M, N))
    parts = torch.empty((P, N), dtype=torch.float32, device=g2.device)
    out = torch.empty((N,), dtype=dtype, device=g2.device)
    L._check(lib.rtdetr_bias_grad(g2.data_ptr(), M, N, parts.data_ptr(), P, out.data_ptr(),
                                  int(dtype == torch.bfloat16), L._stream()), "rtdetr_bias_grad")
    return out


def L_narrow_ok(M: int, N: int) -> bool:
    """Shapes rtdetr_linear_wgrad_narrow takes (M outputs, N inputs)."""
    return (M <= 128 and N % 2 == 0 and N <= 4096) or (N <= 128 and M % 2 == 0 and M <= 4096)


def _defer_targets(weight, bias, x):
    """Where a deferred weight gradient would land (the leaf parameters), or
    None; the backward decides whether to defer (GraphedStep's forward runs
    outside the collecting context)."""
    if DEFER_WGRAD[0] and bias is not None and bias.dtype == weight.dtype and x.is_cuda:
        wt, bt = _row_target(weight), _row_target(bias)
        if wt is not None and bt is not None:
            return (wt, bt)
    return None


def _linear_wgrad(g2, x2, weight_dtype, bias_dtype, has_bias, need_w, need_b, targets):
    """(gw, gb) of one dense linear from its 2-D output gradient and input, or
    (None, None) when deferred (linear.DeferredWgrad collects them)."""
    K, M = g2.shape
    N = x2.shape[1]
    if (need_w and has_bias and need_b and g2.is_cuda and g2.dtype == x2.dtype == torch.bfloat16
            and M % 64 == 0 and N % 128 == 0 and DENSE_WGRAD_ROWS[0] <= K < BIG_ROWS and x2.is_contiguous()):
        # weight + bias gradient in one libmoe_hip launch (split over rows):
        # hipBLASLt's dY^T X on these few-tile outputs plus the bias column
        # sum took ~31 us at 2,400 rows, this ~14 us (tools/mm_probe_small.py)
        from ..moe import _lib as L

        odt = torch.bfloat16 if weight_dtype == torch.bfloat16 else torch.float32
        if _ACTIVE[0] is not None and targets is not None and weight_dtype == odt:
            _ACTIVE[0].add(g2, x2, odt, *targets)  # computed after the backward, batched
            return None, None
        gw, gb = L.linear_wgrad(g2, x2, odt)
        return gw, gb.to(bias_dtype)
    if (need_w and has_bias and need_b and g2.is_cuda and g2.dtype == x2.dtype == torch.bfloat16
            and L_narrow_ok(M, N) and 0 < K < BIG_ROWS and x2.is_contiguous()):
        # narrow heads (M = 1 / 4 / 96 outputs, or the query position
        # head's 4 inputs): hipBLASLt ran dY^T X on 1-8 workgroups, 25-34
        # us each; rtdetr_linear_wgrad_narrow splits the rows over the
        # whole chip and adds the bias column sum
        from ..moe import _lib as L

        odt = torch.bfloat16 if weight_dtype == torch.bfloat16 else torch.float32
        if (_ACTIVE[0] is not None and targets is not None and weight_dtype == odt and NARROW_DEFER[0]
                and targets[0][1] == 0 and targets[1][1] == 0 and M == targets[0][0].shape[0]
                and M == targets[1][0].shape[0] and g2.is_contiguous()):
            _ACTIVE[0].add_narrow(g2, x2, odt, *targets)  # batched after the backward
            return None, None
        gw, gb = L.linear_wgrad_narrow(g2, x2, odt)
        return gw, gb.to(bias_dtype)
    gw = gb = None
    if need_w:
        gw = chunked_wgrad(g2, x2) if x2.shape[0] >= BIG_ROWS else g2.t().mm(x2)
    if has_bias and need_b:
        gb = bias_grad(g2, bias_dtype)
    return gw, gb


class _TokenLinear(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, weight, bias, dtype):
        xc, wc = x.to(dtype), weight.to(dtype)
        bc = bias.to(dtype) if bias is not None else None
        ctx.save_for_backward(xc, wc)
        ctx.has_bias = bias is not None
        ctx.bias_dtype = bias.dtype if bias is not None else None
        ctx.weight_dtype = weight.dtype
        ctx.targets = _defer_targets(weight, bias, x)
        if _narrow_fwd_ok(xc, wc, bc) and wc.shape[0] <= 8:
            from ..moe import _lib as L

            y = L.linear_narrow_fwd(xc.reshape(-1, xc.shape[-1]).contiguous(), wc.contiguous(), bc)
            return y.view(*xc.shape[:-1], wc.shape[0])
        return F.linear(xc, wc, bc)

    @staticmethod
    def backward(ctx, gy):
        xc, wc = ctx.saved_tensors
        g2 = gy.reshape(-1, gy.shape[-1]).to(wc.dtype).contiguous()
        x2 = xc.reshape(-1, xc.shape[-1])
        gx = None
        if ctx.needs_input_grad[0]:
            if _narrow_dgrad_ok(g2, wc):
                from ..moe import _lib as L

                gx = L.linear_narrow_dgrad(g2, wc.contiguous()).view(xc.shape)
            else:
                gx = g2.mm(wc).view(xc.shape)
        gw, gb = _linear_wgrad(g2, x2, ctx.weight_dtype, ctx.bias_dtype, ctx.has_bias, ctx.needs_input_grad[1],
                               ctx.needs_input_grad[2], ctx.targets)
        return gx, gw, gb, None


class _DualTokenLinear(torch.autograd.Function):
    """(x W1^T + b1, x W2^T + b2): two linears of the same input as one node
    (the deformable attention's sampling-offset and attention-weight heads on
    the query).  Forward: the two GEMMs TokenLinear issues.  Backward: x's
    gradient g1 W1 + g2 W2 with the second product accumulated in place by its
    GEMM (addmm_, beta = 1) instead of two products and autograd's add -- the
    first product is already rounded to bf16, so the sum is rounded twice,
    bitwise what the autograd add gave; the weight gradients as TokenLinear's (deferred)."""

    @staticmethod
    def forward(ctx, x, w1, b1, w2, b2, dtype):
        xc = x.to(dtype)
        w1c, w2c = w1.to(dtype), w2.to(dtype)
        y1 = F.linear(xc, w1c, b1.to(dtype))
        y2 = F.linear(xc, w2c, b2.to(dtype))
        ctx.save_for_backward(xc, w1c, w2c)
        ctx.meta = ((w1.dtype, b1.dtype, _defer_targets(w1, b1, x)), (w2.dtype, b2.dtype, _defer_targets(w2, b2, x)))
        ctx.set_materialize_grads(False)
        return y1, y2

    @staticmethod
    def backward(ctx, gy1, gy2):
        xc, w1c, w2c = ctx.saved_tensors
        x2 = xc.reshape(-1, xc.shape[-1])
        gx = None
        grads = [None] * 4
        for i, (gy, wc) in enumerate(((gy1, w1c), (gy2, w2c))):
            if gy is None:
                continue
            g2 = gy.reshape(-1, gy.shape[-1]).to(wc.dtype).contiguous()
            if ctx.needs_input_grad[0]:
                gx = g2.mm(wc) if gx is None else gx.addmm_(g2, wc)
            wdt, bdt, tg = ctx.meta[i]
            grads[2 * i], grads[2 * i + 1] = _linear_wgrad(g2, x2, wdt, bdt, True, ctx.needs_input_grad[1 + 2 * i],
                                                           ctx.needs_input_grad[2 + 2 * i], tg)
        return (None if gx is None else gx.view(xc.shape), *grads, None)


def dual_linear(x, lin1: nn.Linear, lin2: nn.Linear):
    """(lin1(x), lin2(x)): one autograd node on the GPU (_DualTokenLinear),
    the two modules elsewhere."""
    if x.is_cuda and x.numel() > 0 and lin1.bias is not None and lin2.bias is not None:
        dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
        with torch.autocast("cuda", enabled=False):
            return _DualTokenLinear.apply(x, lin1.weight, lin1.bias, lin2.weight, lin2.bias, dtype)
    return lin1(x), lin2(x)


_ROW_OFFSETS: dict = {}


def _row_offsets(rows, device):
    """[0, rows] int32 on the device (one group for the grouped GEMM), cached."""
    key = (int(rows), str(device))
    t = _ROW_OFFSETS.get(key)
    if t is None:
        t = _ROW_OFFSETS[key] = torch.tensor([0, int(rows)], dtype=torch.int32, device=device)
    return t


def _gemm_ok(N, K):
    return N % 128 == 0 and K % 64 == 0


class _MLPHip(torch.autograd.Function):
    """The detector's ReLU MLP heads (box heads, query-position head) in bf16
    as ONE autograd node: a hidden layer whose shape the grouped GEMM takes
    (N % 128 == 0, K % 64 == 0) runs on it with the bias + ReLU epilogue (no
    separate ReLU launch); in the backward the ReLU mask of layer i-1's output
    is applied in layer i's data-gradient epilogue (EPI_RELU_MASK, no
    threshold_backward launch); the weight gradients go through the same
    kernels as TokenLinear's (and the same deferral).  Other layers fall back
    to F.linear / torch ops inside the node."""

    @staticmethod
    def forward(ctx, x, n, *wb):
        from ..moe import _lib as L

        ws, bs = wb[0::2], wb[1::2]
        x2 = x.reshape(-1, x.shape[-1]).contiguous()
        rows = x2.shape[0]
        offs = _row_offsets(rows, x.device)
        ins = []
        h = x2
        for i in range(n):
            w, b = ws[i], bs[i]
            relu = i < n - 1
            ins.append(h)
            N, K = w.shape
            if _gemm_ok(N, K):
                h = L.grouped_gemm(h, w.contiguous(), offs, 1, rows, N, K, 1,
                                   L.EPI_BIAS_RELU if relu else L.EPI_BIAS, bias=b if b.dtype == torch.bfloat16 else b.float(),
                                   dense=True)
            elif _narrow_fwd_ok(h, w, b):  # the box heads' 256 -> 4, the query position head's 4 -> 512 (+ ReLU)
                h = L.linear_narrow_fwd(h.contiguous(), w.contiguous(), b, relu)
            else:
                h = F.linear(h, w, b)
                if relu:
                    h = F.relu(h)
        ctx.save_for_backward(*ins, *ws)
        ctx.n = n
        ctx.meta = [(b.dtype, w.dtype, _defer_targets(w, b, x)) for w, b in zip(ws, bs)]
        ctx.xshape = x.shape
        return h.view(*x.shape[:-1], h.shape[-1])

    @staticmethod
    def backward(ctx, gy):
        from ..moe import _lib as L

        n = ctx.n
        saved = ctx.saved_tensors
        ins, ws = saved[:n], saved[n:]
        g = gy.reshape(-1, gy.shape[-1]).to(torch.bfloat16).contiguous()
        rows = g.shape[0]
        offs = _row_offsets(rows, g.device)
        grads = [None] * (2 * n)
        gx = None
        for i in range(n - 1, -1, -1):
            w, xin = ws[i], ins[i]
            bdt, wdt, tg = ctx.meta[i]
            need_w = ctx.needs_input_grad[2 + 2 * i]
            need_b = ctx.needs_input_grad[3 + 2 * i]
            # data gradient first (the weight gradient may be deferred, and reads g as is)
            gin = None
            if i > 0 or ctx.needs_input_grad[0]:
                N_in = w.shape[1]
                if i > 0 and _gemm_ok(N_in, w.shape[0]):
                    # g_in = (g W) * (x_i > 0): the previous layer's ReLU mask in the epilogue
                    gin = L.grouped_gemm(g, w.contiguous(), offs, 1, rows, N_in, w.shape[0], 0, L.EPI_RELU_MASK,
                                         aux=xin, dense=True)
                elif _narrow_dgrad_ok(g, w):  # a narrow layer: the same, one elementwise-shaped pass
                    gin = L.linear_narrow_dgrad(g, w.contiguous(), xin.contiguous() if i > 0 else None)
                else:
                    gin = g.mm(w)
                    if i > 0:  # ReLU backward of layer i-1's output: one launch
                        gin = torch.ops.aten.threshold_backward(gin, xin, 0.0)
            gw, gb = _linear_wgrad(g, xin, wdt, bdt, True, need_w, need_b, tg)
            grads[2 * i], grads[2 * i + 1] = gw, gb
            g = gin
        if ctx.needs_input_grad[0]:
            gx = g.view(ctx.xshape)
        return (gx, None, *grads)


def mlp_hip_ok(x, layers) -> bool:
    """_MLPHip takes bf16 CUDA inputs with bf16 weights and biases (the bench
    precision; under autocast / fp32 weights the per-layer path runs)."""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.numel() > 0) or torch.is_autocast_enabled("cuda"):
        return False
    return all(m.weight.dtype == torch.bfloat16 and m.bias is not None and m.bias.dtype == torch.bfloat16
               for m in layers)


class TokenLinear(nn.Linear):
    """nn.Linear (same parameters and state dict) whose backward splits the
    weight-gradient reduction over row chunks when the input has many rows and
    takes the bias gradient from the HIP column-sum kernels (bias_grad)."""

    def forward(self, x):
        if x.is_cuda and x.numel() > 0:
            dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
            with torch.autocast("cuda", enabled=False):
                return _TokenLinear.apply(x, self.weight, self.bias, dtype)
        return super().forward(x)


class _SelfAttentionHIP(torch.autograd.Function):
    """softmax(q k^T / sqrt(32)) v per head on the bf16 MFMA
    (rtdetr_attn_fwd / rtdetr_attn_bwd, csrc/attn.hip), reading q and k in
    place from the fused [q | k] projection output [B, L, 2d] and v from
    [B, L, d]; o comes back as [B, L, d] (heads concatenated), so no head
    transposes in either direction.  Head dim 32 only (RT-DETR: d 256, 8 heads)."""

    @staticmethod
    def forward(ctx, qk, v, H):
        from ..moe import _lib as L

        B, T, d2 = qk.shape
        d = d2 // 2
        if d % H or d // H != 32:
            raise ValueError(f"rtdetr_attn: head dim must be 32 (d {d}, {H} heads)")
        ctx.in_dtypes = (qk.dtype, v.dtype)
        qk = qk.to(torch.bfloat16).contiguous()
        v = v.to(torch.bfloat16).contiguous()
        o = torch.empty((B, T, d), dtype=torch.bfloat16, device=qk.device)
        lse = torch.empty((B, H, T), dtype=torch.float32, device=qk.device)
        scale = 1.0 / math.sqrt(d // H)
        L._check(L.lib().rtdetr_attn_fwd(qk.data_ptr(), d2, qk.data_ptr() + 2 * d, d2, v.data_ptr(), d,
                                         o.data_ptr(), d, lse.data_ptr(), B, H, T, d // H, scale, L._stream()),
                 "rtdetr_attn_fwd")
        ctx.save_for_backward(qk, v, o, lse)
        ctx.H, ctx.scale = H, scale
        return o

    @staticmethod
    def backward(ctx, do):
        from ..moe import _lib as L

        qk, v, o, lse = ctx.saved_tensors
        B, T, d2 = qk.shape
        d = d2 // 2
        H = ctx.H
        do = do.to(torch.bfloat16).contiguous()
        dqk = torch.empty_like(qk)
        dv = torch.empty_like(v)
        delta = torch.empty_like(lse)
        L._check(L.lib().rtdetr_attn_bwd(qk.data_ptr(), d2, qk.data_ptr() + 2 * d, d2, v.data_ptr(), d,
                                         o.data_ptr(), d, do.data_ptr(), d, lse.data_ptr(), delta.data_ptr(),
                                         dqk.data_ptr(), d2, dqk.data_ptr() + 2 * d, d2, dv.data_ptr(), d,
                                         B, H, T, d // H, ctx.scale, L._stream()), "rtdetr_attn_bwd")
        return dqk.to(ctx.in_dtypes[0]), dv.to(ctx.in_dtypes[1]), None


def self_attention_hip(qk: torch.Tensor, v: torch.Tensor, num_heads: int) -> torch.Tensor:
    """Multi-head self-attention of [B, L, 2d] fused q|k and [B, L, d] v on the
    GPU (HIP kernels; no scaled_dot_product_attention)."""
    return _SelfAttentionHIP.apply(qk, v, num_heads)


class TokenSelfAttention(nn.Module):
    """Self-attention with nn.MultiheadAttention(batch_first=True)'s parameters
    and state-dict keys (in_proj_weight [3d, d], in_proj_bias, out_proj), for
    the RT-DETR layers' q = k = x + pos, v = x pattern: q and k come from ONE
    [d -> 2d] GEMM on x + pos and v from one [d -> d] GEMM on x (MHA's packed
    path needs q, k and v from one tensor and otherwise issues three), every
    projection through TokenLinear's backward (fused weight + bias gradient),
    then the attention (on the GPU the HIP kernels of csrc/attn.hip, reading
    q / k / v in place; on the CPU scaled_dot_product_attention) and the
    output projection.  Same math as nn.MultiheadAttention (dropout 0)."""

    def __init__(self, d: int, nhead: int):
        super().__init__()
        self.embed_dim, self.num_heads = d, nhead
        self.in_proj_weight = nn.Parameter(torch.empty(3 * d, d))
        self.in_proj_bias = nn.Parameter(torch.empty(3 * d))
        self.out_proj = TokenLinear(d, d)
        nn.init.xavier_uniform_(self.in_proj_weight)
        nn.init.zeros_(self.in_proj_bias)
        nn.init.zeros_(self.out_proj.bias)

    def _proj(self, x, lo, hi):
        w, b = self.in_proj_weight[lo:hi], self.in_proj_bias[lo:hi]
        if x.is_cuda and x.numel() > 0:
            dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else x.dtype
            with torch.autocast("cuda", enabled=False):
                return _TokenLinear.apply(x, w, b, dtype)
        return F.linear(x, w, b)

    def forward(self, qk_in: torch.Tensor, v_in: torch.Tensor) -> torch.Tensor:
        """qk_in = x + pos, v_in = x, both [B, L, d] -> [B, L, d]."""
        B, L, d = qk_in.shape
        H = self.num_heads
        qk = self._proj(qk_in, 0, 2 * d)
        v = self._proj(v_in, 2 * d, 3 * d)
        if qk.is_cuda and d % H == 0 and d // H == 32 and d % 8 == 0:
            # HIP attention (csrc/attn.hip, head_dim 32: RT-DETR's 256 / 8):
            # no Triton-generated SDPA kernels in the step
            return self.out_proj(self_attention_hip(qk, v, H))
        q, k = qk.split(d, -1)
        heads = lambda t: t.reshape(B, L, H, d // H).transpose(1, 2)  # noqa: E731
        o = F.scaled_dot_product_attention(heads(q), heads(k), heads(v))
        return self.out_proj(o.transpose(1, 2).reshape(B, L, d))
