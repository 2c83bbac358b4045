"""RT-DETR transformer decoder: IoU-free query selection (top-300 encoder
tokens), L decoder layers of {self-attention, multi-scale deformable
cross-attention, (MoE) FFN} with iterative box refinement.  The FFN of every
decoder layer is the MoE slot; deformable attention
samples 4 points x 3 levels x 8 heads with bilinear grid_sample (SURVEY.md
8(f).1 names it the next HIP-kernel candidate)."""
from __future__ import annotations

import math
import os

import torch
from torch import nn
import torch.nn.functional as F

from .linear import TokenLinear, TokenSelfAttention, _MLPHip, bias_grad, chunked_wgrad, dual_linear, mlp_hip_ok
from ..moe.config import MoEConfig
from .encoder import HybridEncoder, make_ffn
from .norm import AddLayerNorm
from .backbone import _FUSED_BN
from .conv import conv_module_stats
from .fused import bn_act_eval, bn_act_ok, bn_eval_ok


def inverse_sigmoid(x, eps=1e-5):
    x = x.clamp(min=0.0, max=1.0)
    return torch.log(x.clamp(min=eps) / (1 - x).clamp(min=eps))


class _BoxRefineHip(torch.autograd.Function):
    """(boxes, inter) = sigmoid(delta + inverse_sigmoid(ref)) twice over: the
    same values, ``boxes`` with a gradient to ``ref`` (the loss term) and
    ``inter`` without (the next layer's reference) -- the upstream decoder's
    two sigmoid(delta + inverse_sigmoid(.)) evaluations on ref and on
    ref.detach().  One HIP launch each way (rtdetr_box_refine_fwd/bwd)."""

    @staticmethod
    def forward(ctx, delta, ref, eps):
        from ..moe import _lib as L

        d = delta.contiguous()
        r = ref.float().contiguous()
        y = torch.empty(r.shape, dtype=torch.float32, device=r.device)
        L._check(L.lib().rtdetr_box_refine_fwd(d.data_ptr(), int(d.dtype == torch.bfloat16), r.data_ptr(), r.numel(),
                                               float(eps), y.data_ptr(), L._stream()), "rtdetr_box_refine_fwd")
        ctx.save_for_backward(y, r)
        ctx.eps, ctx.ddt, ctx.rdt = float(eps), d.dtype, ref.dtype
        return y, y.view_as(y)

    @staticmethod
    def backward(ctx, g_boxes, g_inter):
        from ..moe import _lib as L

        y, r = ctx.saved_tensors
        gb = g_boxes.float().contiguous() if g_boxes is not None else None
        gi = g_inter.float().contiguous() if g_inter is not None else None
        gd = torch.empty(y.shape, dtype=ctx.ddt, device=y.device)
        need_ref = ctx.needs_input_grad[1] and gb is not None
        gr = torch.empty_like(y) if need_ref else None
        L._check(L.lib().rtdetr_box_refine_bwd(None if gb is None else gb.data_ptr(),
                                               None if gi is None else gi.data_ptr(), y.data_ptr(), r.data_ptr(),
                                               y.numel(), ctx.eps, gd.data_ptr(), int(ctx.ddt == torch.bfloat16),
                                               None if gr is None else gr.data_ptr(), L._stream()),
                 "rtdetr_box_refine_bwd")
        return gd, (gr.to(ctx.rdt) if gr is not None else None), None


def box_refine(delta, ref, eps=1e-5):
    """-> (boxes, inter): sigmoid(delta + inverse_sigmoid(ref)), boxes with a
    gradient to ref, inter without (see _BoxRefineHip)."""
    if delta.is_cuda and delta.dtype in (torch.bfloat16, torch.float32) and _FUSED_BOXES:
        return _BoxRefineHip.apply(delta, ref, eps)
    d = delta.float()
    boxes = (d + inverse_sigmoid(ref, eps)).sigmoid()
    inter = (d + inverse_sigmoid(ref.detach(), eps)).sigmoid()
    return boxes, inter


class MLP(nn.Module):
    def __init__(self, din, dh, dout, n):
        super().__init__()
        dims = [din] + [dh] * (n - 1)
        self.layers = nn.ModuleList(TokenLinear(a, b) for a, b in zip(dims, dims[1:] + [dout]))

    def forward(self, x):
        if _FUSED_MLP and mlp_hip_ok(x, self.layers):
            # one autograd node: bias + ReLU in the GEMM epilogue, the ReLU mask in the
            # next layer's data-gradient epilogue (linear._MLPHip)
            wb = [t for m in self.layers for t in (m.weight, m.bias)]
            return _MLPHip.apply(x, len(self.layers), *wb)
        for i, layer in enumerate(self.layers):
            x = layer(x)
            if i < len(self.layers) - 1:
                x = F.relu(x)
        return x


def deformable_attention_core(value, shapes, sampling_locations, attention_weights):
    """value [B, S, H, Dh]; sampling_locations [B, Q, H, L, P, 2] in [0,1];
    attention_weights [B, Q, H, L, P] -> [B, Q, H*Dh]."""
    B, _, H, Dh = value.shape
    _, Q, _, L, P, _ = sampling_locations.shape
    splits = [h * w for h, w in shapes]
    values = value.split(splits, dim=1)
    grids = 2.0 * sampling_locations - 1.0
    sampled = []
    for lvl, (h, w) in enumerate(shapes):
        v = values[lvl].flatten(2).transpose(1, 2).reshape(B * H, Dh, h, w)
        g = grids[:, :, :, lvl].transpose(1, 2).flatten(0, 1)            # [B*H, Q, P, 2]
        sampled.append(F.grid_sample(v, g.to(v.dtype), mode="bilinear", padding_mode="zeros",
                                     align_corners=False))              # [B*H, Dh, Q, P]
    aw = attention_weights.transpose(1, 2).reshape(B * H, 1, Q, L * P)
    out = (torch.stack(sampled, dim=-2).flatten(-2) * aw.to(sampled[0].dtype)).sum(-1)
    return out.view(B, H * Dh, Q).transpose(1, 2)


class _MSDAHip(torch.autograd.Function):
    """HIP sampling core (libmoe_hip.so rtdetr_msda_fwd/bwd) for GPU tensors."""

    @staticmethod
    def forward(ctx, value, shapes_t, starts_t, loc, attn):
        from ..moe import _lib as L

        v = value.to(torch.bfloat16).contiguous()
        lo = loc.float().contiguous()
        at = attn.float().contiguous()
        out = L.msda_fwd(v, shapes_t, starts_t, lo, at)
        ctx.save_for_backward(v, shapes_t, starts_t, lo, at)
        ctx.vdtype = value.dtype
        return out

    @staticmethod
    def backward(ctx, grad_out):
        from ..moe import _lib as L

        v, shapes_t, starts_t, lo, at = ctx.saved_tensors
        # bf16 values (the training step): packed bf16 atomics give grad_value in
        # the value's dtype directly; an fp32 value keeps fp32 accumulation
        gv, gl, ga = L.msda_bwd(v, shapes_t, starts_t, lo, at, grad_out.to(torch.bfloat16).contiguous(),
                                bf16_grad_value=ctx.vdtype == torch.bfloat16)
        return gv.to(ctx.vdtype), None, None, gl, ga


class _MSDAFusedHip(torch.autograd.Function):
    """Decoder cross-attention core with the location / softmax prep fused
    into the HIP kernels (rtdetr_msda_fused_fwd/bwd): inputs are the raw
    sampling-offset and attention-weight linear outputs and the (detached)
    reference boxes."""

    @staticmethod
    def forward(ctx, value, shapes_t, starts_t, off, ref, logits, offset_scale, L, P):
        from ..moe import _lib as L_

        v, o, lg = value.contiguous(), off.contiguous(), logits.contiguous()
        r = ref.float().contiguous()
        out = L_.msda_fused_fwd(v, shapes_t, starts_t, o, r, lg, offset_scale, L, P)
        ctx.save_for_backward(v, shapes_t, starts_t, o, r, lg)
        ctx.cfg = (offset_scale, L, P)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        from ..moe import _lib as L_

        v, shapes_t, starts_t, o, r, lg = ctx.saved_tensors
        offset_scale, L, P = ctx.cfg
        gv, go, gl = L_.msda_fused_bwd(v, shapes_t, starts_t, o, r, lg, offset_scale, L, P,
                                       grad_out.to(torch.bfloat16).contiguous())
        return gv, None, None, go, None, gl, None, None, None


class _LevelMemory(torch.autograd.Function):
    """The decoder's memory [B, S, d]: the input projections' training
    BatchNorms (act none) of the n levels, each written straight into its rows
    of memory (rtdetr_bn_act_fwd_rows: image b, level l at rows
    [b S + start_l, b S + start_l + h_l w_l)), instead of n BatchNorm outputs
    concatenated (a copy of all of memory) whose backward hands every level a
    strided slice of d memory to copy back to channels_last.  Backward reads
    each level's rows of d memory in place (rtdetr_bn_act_bwd_rows).  Inputs:
    the conv outputs y_l (channels_last bf16), their conv-epilogue statistics
    partials (or None), then gammas and betas."""

    @staticmethod
    def forward(ctx, bns, parts, *args):
        from ..moe import _lib as L

        n = len(bns)
        ys, gammas, betas = args[:n], args[n:2 * n], args[2 * n:3 * n]
        B, C = ys[0].shape[:2]
        hws = [int(y.shape[2] * y.shape[3]) for y in ys]
        S = sum(hws)
        mem = torch.empty((B, S, C), dtype=torch.bfloat16, device=ys[0].device)
        saved, row0 = [], 0
        for y, g, b, bn, part, hw in zip(ys, gammas, betas, bns, parts, hws):
            saved.append(L.bn_act_fwd_rows(y, g, b, bn.running_mean, bn.running_var, 0, bn.eps, bn.momentum, part,
                                           mem, row0, hw, S))
            row0 += hw
        ctx.save_for_backward(*ys, *gammas, *saved)
        ctx.meta = (n, hws, S)
        return mem

    @staticmethod
    def backward(ctx, dmem):
        from ..moe import _lib as L

        n, hws, S = ctx.meta
        t = ctx.saved_tensors
        ys, gammas, saved = t[:n], t[n:2 * n], t[2 * n:]
        dmem = dmem.contiguous()
        dxs, dgs, dbs, row0 = [], [], [], 0
        for y, g, sv, hw in zip(ys, gammas, saved, hws):
            dx, dgb = L.bn_act_bwd_rows(dmem, row0, hw, S, y, g, sv, 0)
            dxs.append(dx)
            dgs.append(dgb[0, 0])
            dbs.append(dgb[0, 1])
            row0 += hw
        return (None, None, *dxs, *dgs, *dbs)


def _select_queries(rank, k):
    """Indices of the k best-ranked memory tokens per image, best first:
    libmoe_hip's rtdetr_topk_rows on the GPU (torch.topk ran one
    single-workgroup sort per image, ~128 us at C2), torch.topk elsewhere."""
    from ..moe import _lib as L

    if (_HIP_TOPK and rank.is_cuda and rank.dtype == torch.float32 and rank.dim() == 2
            and rank.shape[1] <= L.TOPK_MAX_N and 0 < k <= min(L.TOPK_MAX_K, rank.shape[1])):
        return L.topk_rows(rank, k)
    return torch.topk(rank, k, dim=1).indices


class _ValueProjAll(torch.autograd.Function):
    """The decoder layers' value projections over the encoder memory as ONE
    GEMM, [B*S, d] x [d, n d] with the n layers' weights concatenated per call
    (the parameters stay per layer).  Forward returns the values v_all
    [B, S, n d] (layer i reads columns [i d, (i+1) d) through the strided MSDA
    kernels), a zeroed gradient buffer of the same shape into which the layers'
    MSDA backward kernels ACCUMULATE their value gradients, and a scalar
    `token` every layer takes as an input (its zero gradient makes autograd run
    this backward after all of them).  Backward: d memory = G W (one GEMM, no
    per-layer gradient adds), dW = G^T memory (one row-chunked GEMM), db = the
    column sums of G, split back per layer.
    Also returns the query selection's rows, sel = memory[b, topk[b, q]] *
    vsel[b, q] (the encoder-output heads' input): its gradient is added into
    the rows of d memory in place (one scatter-add over the B Q selected rows)
    instead of autograd's zero-filled [B, S, d] scatter and full-size add."""

    @staticmethod
    def forward(ctx, memory, dtype, det, topk, vsel, *wb):
        n = len(wb) // 2
        ws, bs = wb[0::2], wb[1::2]
        B, S, d = memory.shape
        m2 = memory.reshape(B * S, d).to(dtype)
        W = torch.cat([w.to(dtype) for w in ws], 0)  # [n d, d]
        bias = torch.cat([b.to(dtype) for b in bs], 0)
        v_all = F.linear(m2, W, bias).view(B, S, n * d)
        # det: every layer's deterministic MSDA backward writes its whole
        # column slice (no zero fill of the [B, S, n d] buffer); else the
        # atomic backward accumulates into a zeroed buffer
        grad_all = torch.empty_like(v_all) if det else torch.zeros_like(v_all)
        token = torch.zeros((), dtype=torch.float32, device=memory.device)
        idx = topk[..., None].expand(-1, -1, d)
        sel = memory.gather(1, idx) * vsel
        ctx.save_for_backward(m2, W, idx, vsel)
        ctx.grad_all = grad_all
        ctx.meta = (B, S, d, n, memory.dtype, [w.dtype for w in ws], [b.dtype for b in bs])
        ctx.mark_non_differentiable(v_all, grad_all)
        ctx.set_materialize_grads(False)  # no zero-filled [B, S, n d] gradients for v_all / grad_all
        return v_all, grad_all, token, sel

    @staticmethod
    def backward(ctx, _gv, _gg, _gt, gsel):
        m2, W, idx, vsel = ctx.saved_tensors
        B, S, d, n, mdtype, wdt, bdt = ctx.meta
        G = ctx.grad_all.view(B * S, n * d)
        ctx.grad_all = None
        dmem = G.mm(W).view(B, S, d).to(mdtype) if ctx.needs_input_grad[0] else None
        if dmem is not None and gsel is not None:  # (top-k rows are distinct per image: one add per row)
            dmem.scatter_add_(1, idx, (gsel * vsel).to(mdtype))
        dW = chunked_wgrad(G, m2)  # fp32 [n d, d]
        grads = []
        if len(set(wdt)) == 1 and len(set(bdt)) == 1:
            # one cast of all layers' weights and the bias sums in their dtype:
            # 2 launches instead of 2 n (per-layer slices are views)
            dWc = dW.to(wdt[0])
            dbc = bias_grad(G, bdt[0])
            for i in range(n):
                grads += [dWc[i * d:(i + 1) * d], dbc[i * d:(i + 1) * d]]
        else:
            db = bias_grad(G, torch.float32)
            for i in range(n):
                grads += [dW[i * d:(i + 1) * d].to(wdt[i]), db[i * d:(i + 1) * d].to(bdt[i])]
        return (dmem, None, None, None, None, *grads)


class _MSDAFusedSlot(torch.autograd.Function):
    """_MSDAFusedHip on a column slice of _ValueProjAll's v_all; the value
    gradient is accumulated into the same slice of its shared buffer."""

    @staticmethod
    def forward(ctx, token, v_all, grad_all, col0, H, D, shapes_t, starts_t, off, ref, logits, offset_scale, L, P,
                hw=None):
        from ..moe import _lib as L_

        o, lg = off.contiguous(), logits.contiguous()
        r = ref.float().contiguous()
        out = L_.msda_fused_fwd_slice(v_all, col0, H, D, shapes_t, starts_t, o, r, lg, offset_scale, L, P)
        ctx.save_for_backward(v_all, shapes_t, starts_t, o, r, lg)
        ctx.grad_all = grad_all
        ctx.cfg = (col0, H, D, offset_scale, L, P, hw)
        return out

    @staticmethod
    def backward(ctx, grad_out):
        from ..moe import _lib as L_

        v_all, shapes_t, starts_t, o, r, lg = ctx.saved_tensors
        col0, H, D, offset_scale, L, P, hw = ctx.cfg
        g = grad_out.to(torch.bfloat16).contiguous()
        if hw is not None:  # deterministic: writes the slice (fixed-order fp32 sums)
            go, gl = L_.msda_fused_bwd_slice_det(v_all, ctx.grad_all, col0, H, D, shapes_t, starts_t, hw, o, r, lg,
                                                 offset_scale, L, P, g)
        else:  # atomic: accumulates into the zeroed slice
            go, gl = L_.msda_fused_bwd_slice(v_all, ctx.grad_all, col0, H, D, shapes_t, starts_t, o, r, lg,
                                             offset_scale, L, P, g)
        ctx.grad_all = None
        # (no gradient for `token`: it only orders _ValueProjAll's backward after this one)
        return (None,) * 8 + (go, None, gl) + (None,) * 4


_LEVEL_CACHE = {}
_FUSED_MSDA = os.environ.get("MOE_FUSED_MSDA", "1") != "0"  # A/B switch
_BATCHED_VALUE = os.environ.get("MOE_BATCHED_VALUE", "1") != "0"  # A/B switch: one value projection for all layers
_FUSED_BOXES = os.environ.get("MOE_FUSED_BOXES", "1") != "0"  # A/B switch
_FUSED_MLP = os.environ.get("MOE_FUSED_MLP", "1") != "0"  # A/B switch: ReLU MLP heads as one node (linear._MLPHip)
# MOE_DET_MSDA=0: the decoder's MSDA value gradients by packed bf16 atomics
# (arrival order) instead of the deterministic fixed-order fp32 sums (A/B)
_DET_MSDA = os.environ.get("MOE_DET_MSDA", "1") != "0"
# MOE_LEVEL_MEMORY=0: the input projections' BatchNorm outputs concatenated
# into memory by torch.cat (A/B switch for _LevelMemory)
_LEVEL_MEMORY = os.environ.get("MOE_LEVEL_MEMORY", "1") != "0"
# MOE_MASK_ROWS=0: the ranking's valid * memory as a full multiply (A/B switch)
_MASK_ROWS = os.environ.get("MOE_MASK_ROWS", "1") != "0"
# query selection top-k on libmoe_hip (rtdetr_topk_rows); 0: torch.topk
_HIP_TOPK = os.environ.get("MOE_HIP_TOPK", "1") != "0"


def _det_msda(L, P, D):
    """Whether the decoder's fused MSDA backward runs deterministically
    (_lib.msda_det_ok shapes, MOE_DET_MSDA on)."""
    from ..moe import _lib as L_

    return _DET_MSDA and L_.msda_det_ok(L, P, D)


def _level_tensors(shapes, device):
    key = (tuple(shapes), device)
    if key not in _LEVEL_CACHE:
        starts, s = [], 0
        for h, w in shapes:
            starts.append(s)
            s += h * w
        _LEVEL_CACHE[key] = (torch.tensor(shapes, dtype=torch.int32, device=device),
                             torch.tensor(starts, dtype=torch.int32, device=device))
    return _LEVEL_CACHE[key]


def deformable_attention(value, shapes, sampling_locations, attention_weights):
    """GPU: HIP kernel; CPU: the grid_sample formulation above."""
    if value.is_cuda:
        st, so = _level_tensors(shapes, value.device)
        return _MSDAHip.apply(value, st, so, sampling_locations, attention_weights)
    return deformable_attention_core(value, shapes, sampling_locations, attention_weights)


class MSDeformableAttention(nn.Module):
    def __init__(self, d=256, nhead=8, nlevels=3, npoints=4, offset_scale=0.5):
        super().__init__()
        self.d, self.nhead, self.nlevels, self.npoints = d, nhead, nlevels, npoints
        self.offset_scale = offset_scale
        self.sampling_offsets = TokenLinear(d, nhead * nlevels * npoints * 2)
        self.attention_weights = TokenLinear(d, nhead * nlevels * npoints)
        self.value_proj = TokenLinear(d, d)  # runs over all B*S memory tokens
        self.output_proj = TokenLinear(d, d)
        self._reset()

    def _reset(self):
        nn.init.zeros_(self.sampling_offsets.weight)
        thetas = torch.arange(self.nhead, dtype=torch.float32) * (2.0 * math.pi / self.nhead)
        grid = torch.stack([thetas.cos(), thetas.sin()], -1)
        grid = grid / grid.abs().max(-1, keepdim=True).values
        grid = grid.view(self.nhead, 1, 1, 2).tile(1, self.nlevels, self.npoints, 1)
        grid *= torch.arange(1, self.npoints + 1, dtype=torch.float32).view(1, 1, -1, 1)
        with torch.no_grad():
            self.sampling_offsets.bias.copy_(grid.flatten())
        nn.init.zeros_(self.attention_weights.weight)
        nn.init.zeros_(self.attention_weights.bias)
        nn.init.xavier_uniform_(self.value_proj.weight)
        nn.init.zeros_(self.value_proj.bias)
        nn.init.xavier_uniform_(self.output_proj.weight)
        nn.init.zeros_(self.output_proj.bias)

    def forward(self, query, ref_boxes, value, shapes, vslot=None):
        """query [B,Q,d]; ref_boxes [B,Q,4] (cx,cy,w,h in [0,1]); value [B,S,d].
        vslot = (v_all, grad_all, token, col0): the projected values come from
        the decoder's batched value projection (_ValueProjAll) instead."""
        B, Q, _ = query.shape
        H, L, P = self.nhead, self.nlevels, self.npoints
        if vslot is not None:
            v_all, g_all, token, col0 = vslot
            off, logits = dual_linear(query, self.sampling_offsets, self.attention_weights)
            if not (off.dtype == logits.dtype == torch.bfloat16 and not ref_boxes.requires_grad and L * P <= 16):
                raise RuntimeError("the batched value projection needs the fused bf16 MSDA path")
            st, so = _level_tensors(shapes, v_all.device)
            det = _det_msda(L, P, self.d // H)  # (the same rule _value_slots applied to every layer)
            hw = tuple(int(h) * int(w) for h, w in shapes) if det else None
            out = _MSDAFusedSlot.apply(token, v_all, g_all, col0, H, self.d // H, st, so, off, ref_boxes, logits,
                                       float(self.offset_scale), L, P, hw)
            return self.output_proj(out)
        v = self.value_proj(value).view(B, value.shape[1], H, self.d // H)
        off, logits = dual_linear(query, self.sampling_offsets, self.attention_weights)
        if (_FUSED_MSDA and v.is_cuda and v.dtype == off.dtype == logits.dtype == torch.bfloat16
                and not ref_boxes.requires_grad and L * P <= 16):
            st, so = _level_tensors(shapes, v.device)
            out = _MSDAFusedHip.apply(v, st, so, off, ref_boxes, logits, float(self.offset_scale), L, P)
            return self.output_proj(out)
        off = off.view(B, Q, H, L, P, 2)
        aw = F.softmax(logits.view(B, Q, H, L * P).float(), -1).view(B, Q, H, L, P)
        ref = ref_boxes[:, :, None, None, None, :]
        loc = ref[..., :2] + off / P * ref[..., 2:] * self.offset_scale
        return self.output_proj(deformable_attention(v, shapes, loc, aw))


class TransformerDecoderLayer(nn.Module):
    def __init__(self, d=256, nhead=8, hidden=1024, nlevels=3, npoints=4, moe: MoEConfig | None = None):
        super().__init__()
        self.self_attn = TokenSelfAttention(d, nhead)
        self.norm1 = AddLayerNorm(d)  # LayerNorm(a + b), fused on the GPU (norm.py)
        self.cross_attn = MSDeformableAttention(d, nhead, nlevels, npoints)
        self.norm2 = AddLayerNorm(d)
        self.ffn = make_ffn(d, hidden, moe, act="relu")
        self.norm3 = AddLayerNorm(d)

    def forward(self, tgt, ref_boxes, memory, shapes, query_pos, ctx, vslot=None):
        # t1 and the cross-attention query t1 + query_pos from one LayerNorm launch
        tgt, q = self.norm1.with_pos(tgt, self.self_attn(tgt + query_pos, tgt), query_pos)
        tgt = self.norm2(tgt, self.cross_attn(q, ref_boxes, memory, shapes, vslot))
        tgt = self.norm3(self.ffn(tgt, ctx, residual=True))  # tgt + FFN(tgt)
        return tgt


class RTDETRDecoder(nn.Module):
    def __init__(self, num_classes=1, hidden=256, feat_channels=(256, 256, 256), feat_strides=(8, 16, 32),
                 num_queries=300, num_layers=6, nhead=8, dim_feedforward=1024, npoints=4,
                 moe: MoEConfig | None = None):
        super().__init__()
        self.hidden = hidden
        self.num_queries = num_queries
        self.num_classes = num_classes
        self.nlevels = len(feat_channels)
        self.input_proj = nn.ModuleList(
            [nn.Sequential(nn.Conv2d(c, hidden, 1, bias=False), nn.BatchNorm2d(hidden)) for c in feat_channels])
        self.layers = nn.ModuleList([
            TransformerDecoderLayer(hidden, nhead, dim_feedforward, self.nlevels, npoints, moe)
            for _ in range(num_layers)])
        self.query_pos_head = MLP(4, 2 * hidden, hidden, 2)
        self.enc_output = nn.Sequential(TokenLinear(hidden, hidden), AddLayerNorm(hidden))
        self.enc_score_head = TokenLinear(hidden, num_classes)
        self.enc_bbox_head = MLP(hidden, hidden, 4, 3)
        self.dec_score_head = nn.ModuleList([TokenLinear(hidden, num_classes) for _ in range(num_layers)])
        self.dec_bbox_head = nn.ModuleList([MLP(hidden, hidden, 4, 3) for _ in range(num_layers)])
        self._anchor_cache = {}
        # query selection of the last forward ([B, Q] token indices), and an
        # optional override replayed instead of the top-k (tests/test_gpu_model_parity.py
        # feeds the CPU run's selection to the GPU run so both decode the same queries)
        self.last_topk = None
        self.query_override = None
        self._reset()

    def _reset(self):
        bias = -math.log((1 - 0.01) / 0.01)
        nn.init.constant_(self.enc_score_head.bias, bias)
        for h in self.dec_score_head:
            nn.init.constant_(h.bias, bias)
        for m in [self.enc_bbox_head, *self.dec_bbox_head]:
            nn.init.zeros_(m.layers[-1].weight)
            nn.init.zeros_(m.layers[-1].bias)

    def _anchors(self, shapes, device, dtype, grid_size=0.05, eps=1e-2):
        key = (tuple(shapes), device, dtype)
        if key not in self._anchor_cache:
            anchors = []
            for lvl, (h, w) in enumerate(shapes):
                gy, gx = torch.meshgrid(torch.arange(h, dtype=torch.float32), torch.arange(w, dtype=torch.float32),
                                        indexing="ij")
                xy = torch.stack([(gx + 0.5) / w, (gy + 0.5) / h], -1)
                wh = torch.full_like(xy, grid_size * 2.0 ** lvl)
                anchors.append(torch.cat([xy, wh], -1).reshape(-1, 4))
            a = torch.cat(anchors, 0)[None]
            valid = ((a > eps) & (a < 1 - eps)).all(-1, keepdim=True)
            # (the invalid rows' indices, from the host copy: no device sync later)
            self._anchor_cache[("inv",) + key] = (~valid[0, :, 0]).nonzero().flatten().to(device)
            a, valid = a.to(device), valid.to(device)
            a = torch.log(a / (1 - a))
            a = torch.where(valid, a, torch.full_like(a, float("inf")))
            self._anchor_cache[key] = (a.to(dtype), valid.to(dtype))
        return self._anchor_cache[key]

    def _enc_output_masked(self, memory, inv, vmask):
        """enc_output(valid * memory) for the query ranking (no autograd).  GPU
        bf16: the linear runs on memory itself and only the invalid-anchor rows
        of its output are overwritten with the bias -- a zero input row's
        output, bf16(0 W^T + b) = b exactly -- instead of multiplying all of
        memory by the mask ([B, S, d], ~40 us at C2); the same values."""
        lin_, ln_ = self.enc_output[0], self.enc_output[1]
        if not (_MASK_ROWS and memory.is_cuda and memory.dtype == torch.bfloat16 and isinstance(lin_, TokenLinear)
                and lin_.bias is not None and not torch.is_autocast_enabled("cuda")):
            return self.enc_output(vmask * memory)
        y = lin_(memory)
        if inv.numel():
            y[:, inv] = lin_.bias.to(y.dtype)
        return ln_(y)

    def _value_slots(self, memory, topk, vsel):
        """GPU bf16 path: all layers' value projections as one GEMM
        (_ValueProjAll, which also gathers the selected rows) -> (slots, sel);
        elsewhere None (each layer projects its own values)."""
        n = len(self.layers)
        dtype = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled("cuda") else memory.dtype
        if not (_BATCHED_VALUE and _FUSED_MSDA and memory.is_cuda and dtype == torch.bfloat16 and n > 1):
            return None
        vps = [layer.cross_attn.value_proj for layer in self.layers]
        det = all(_det_msda(la.cross_attn.nlevels, la.cross_attn.npoints, la.cross_attn.d // la.cross_attn.nhead)
                  for la in self.layers)
        with torch.autocast("cuda", enabled=False):
            v_all, g_all, token, sel = _ValueProjAll.apply(memory, dtype, det, topk, vsel,
                                                           *[t for m in vps for t in (m.weight, m.bias)])
        return [(v_all, g_all, token, i * self.hidden) for i in range(n)], sel

    def _memory(self, feats):
        """(memory [B, S, d], level shapes): the input projections (1x1 conv +
        training BatchNorm) of every level, flattened and concatenated over
        the levels.  GPU bf16 with the fused BatchNorm: each level's
        BatchNorm writes its rows of memory directly (_LevelMemory), its
        statistics summed in the convolution's epilogue."""
        if _FUSED_BN and feats[0].is_cuda and not torch.is_grad_enabled():
            from . import evalfold

            # inference: each level's 1x1 conv with its BN folded writes its rows of the memory in place
            if all(evalfold.folded(p, f) is not None and evalfold.folded(p, f)[3] == 1
                   for p, f in zip(self.input_proj, feats)):
                shapes = [tuple(f.shape[-2:]) for f in feats]
                S = sum(h * w for h, w in shapes)
                B = feats[0].shape[0]
                mem = torch.empty((B, S, self.input_proj[0][0].out_channels), dtype=torch.bfloat16,
                                  device=feats[0].device)
                row = 0
                for p, f, (h, w) in zip(self.input_proj, feats, shapes):
                    evalfold.conv_folded(p, f, out=mem, out_row=row)
                    row += h * w
                return mem, shapes
        if _FUSED_BN and _LEVEL_MEMORY and feats[0].is_cuda:
            ys, parts, bns = [], [], []
            for p, f in zip(self.input_proj, feats):
                y, part = conv_module_stats(p[0], f)
                ys.append(y)
                parts.append(part)
                bns.append(p[1])
            if all(bn_act_ok([y], [bn]) for y, bn in zip(ys, bns)) and len({y.shape[:2] for y in ys}) == 1:
                mem = _LevelMemory.apply(bns, parts, *ys, *[bn.weight for bn in bns], *[bn.bias for bn in bns])
                return mem, [tuple(y.shape[-2:]) for y in ys]
            # inference: running statistics in one HIP pass per level
            proj = [bn_act_eval([y], [bn], None) if bn_eval_ok([y], [bn]) else bn(y) for y, bn in zip(ys, bns)]
        else:
            # conv + training BatchNorm through libmoe_hip's bn_act (as the encoder's
            # input projections): MIOpen's BN backward at batch 1 lost the gradient
            # (relative error 1.4 vs 0.09 for a bf16 CPU run, tools/grad_flow_diag.py)
            proj = [HybridEncoder._proj(p, f) for p, f in zip(self.input_proj, feats)]
        shapes = [tuple(f.shape[-2:]) for f in proj]
        return torch.cat([f.flatten(2).permute(0, 2, 1) for f in proj], 1).contiguous(), shapes  # [B, S, d]

    def forward(self, feats, ctx):
        memory, shapes = self._memory(feats)
        B = memory.shape[0]
        anchors, valid = self._anchors(shapes, memory.device, torch.float32)
        vmask = valid.to(memory.dtype)  # [1, S, 1]
        # Query selection.  Only the top-k rows of the encoder-output heads are
        # used downstream (their logits/boxes and the detached decoder targets),
        # so the heads run over all S tokens once without autograd, to rank
        # them, and again with autograd on the B*Q selected rows only.  Same
        # values and gradients as running the heads over all tokens, without
        # the three [B*S, 256] weight-gradient GEMMs and activation storage.
        if self.query_override is not None:  # parity checks: replay another run's query selection
            topk = self.query_override.to(memory.device)
        else:
            with torch.no_grad():
                inv = self._anchor_cache[("inv", tuple(shapes), memory.device, torch.float32)]
                enc_rank = self.enc_score_head(self._enc_output_masked(memory, inv, vmask)).float().max(-1).values
            topk = _select_queries(enc_rank, self.num_queries)
        self.last_topk = topk
        # (valid * memory) at the selected rows: the mask applied after the
        # gather (same products), so the backward multiplies [B, Q, d], not [B, S, d]
        vsel = vmask.expand(B, -1, -1).gather(1, topk[..., None])
        vs = self._value_slots(memory, topk, vsel)
        if vs is not None:
            vslots, sel_in = vs
        else:
            vslots = [None] * len(self.layers)
            sel_in = memory.gather(1, topk[..., None].expand(-1, -1, memory.shape[-1])) * vsel
        sel = self.enc_output(sel_in)
        enc_topk_logits = self.enc_score_head(sel)
        ref_unact = self.enc_bbox_head(sel).float() + anchors.expand(B, -1, -1).gather(
            1, topk[..., None].expand(-1, -1, 4))
        enc_topk_boxes = ref_unact.sigmoid()
        tgt = sel.detach()
        ref_detach = ref_unact.detach().sigmoid()
        ref = ref_detach
        dec_logits, dec_boxes = [], []
        for i, layer in enumerate(self.layers):
            query_pos = self.query_pos_head(ref_detach.to(tgt.dtype))
            tgt = layer(tgt, ref_detach, memory, shapes, query_pos, ctx, vslots[i])
            # boxes_i = sigmoid(delta_i + inverse_sigmoid(ref)) with a gradient to
            # the previous layer's boxes; the next reference is the same value
            # without it (upstream: inter on ref_detach, boxes on ref)
            boxes, inter = box_refine(self.dec_bbox_head[i](tgt), ref)
            dec_logits.append(self.dec_score_head[i](tgt))
            dec_boxes.append(boxes)
            ref = inter
            ref_detach = inter.detach()
        out = {"pred_logits": dec_logits[-1], "pred_boxes": dec_boxes[-1],
               "aux_outputs": [{"pred_logits": a, "pred_boxes": b} for a, b in zip(dec_logits[:-1], dec_boxes[:-1])],
               "enc_outputs": {"pred_logits": enc_topk_logits, "pred_boxes": enc_topk_boxes}}
        return out
