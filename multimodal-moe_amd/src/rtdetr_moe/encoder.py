"""RT-DETR HybridEncoder: AIFI transformer layer on S5 (its FFN is the MoE
slot) + CCFM cross-scale fusion (FPN + PAN of
CSPRep layers).  Dimensions follow Appendix A of SURVEY.md (hidden 256, FFN
1024, 8 heads, one encoder layer on stride 32)."""
from __future__ import annotations

import torch
from torch import nn
import torch.nn.functional as F

from ..moe.config import MoEConfig
from ..moe.layer import MoEFFN
from .norm import AddLayerNorm
from .backbone import _FUSED_BN, ConvNormLayer, stage_taps
from . import evalfold
from .conv import GradSlot, conv_module, conv_pair
from .fused import bn_act, bn_act_eval, bn_act_ok, bn_eval_ok
from .linear import TokenLinear, TokenSelfAttention


class _UpCat(torch.autograd.Function):
    """cat([nearest x2 upsample of high (cropped to low's size), low], dim=1)
    over channels_last bf16: rtdetr_upcat_nhwc_fwd / _bwd, one launch each way."""

    @staticmethod
    def forward(ctx, high, low):
        from ..moe import _lib as L

        B, Ch, Hh, Wh = high.shape
        Cl, H, W = low.shape[1:]
        out = torch.empty((B, Ch + Cl, H, W), dtype=low.dtype, device=low.device, memory_format=torch.channels_last)
        L._check(L.lib().rtdetr_upcat_nhwc_fwd(high.data_ptr(), low.data_ptr(), B, H, W, Hh, Wh, Ch, Cl,
                                               out.data_ptr(), L._stream()), "rtdetr_upcat_nhwc_fwd")
        ctx.dims = (B, H, W, Hh, Wh, Ch, Cl)
        return out

    @staticmethod
    def backward(ctx, g):
        from ..moe import _lib as L

        B, H, W, Hh, Wh, Ch, Cl = ctx.dims
        g = g.contiguous(memory_format=torch.channels_last)
        if g.data_ptr() % 16:
            g = g.clone(memory_format=torch.channels_last)
        dhigh = torch.empty((B, Ch, Hh, Wh), dtype=g.dtype, device=g.device, memory_format=torch.channels_last)
        dlow = torch.empty((B, Cl, H, W), dtype=g.dtype, device=g.device, memory_format=torch.channels_last)
        L._check(L.lib().rtdetr_upcat_nhwc_bwd(g.data_ptr(), B, H, W, Hh, Wh, Ch, Cl, dhigh.data_ptr(),
                                               dlow.data_ptr(), L._stream()), "rtdetr_upcat_nhwc_bwd")
        return dhigh, dlow


def up_cat(high, low):
    """The FPN top-down input: torch.cat([F.interpolate(high, scale_factor=2,
    mode="nearest") cropped to low, low], dim=1).  channels_last bf16 GPU
    tensors take the fused HIP pair (_UpCat); anything else the torch ops."""
    B, Ch, Hh, Wh = high.shape
    H, W = low.shape[-2:]
    if (high.is_cuda and high.dtype == low.dtype == torch.bfloat16 and low.shape[0] == B and Ch % 8 == 0
            and low.shape[1] % 8 == 0 and H <= 2 * Hh and W <= 2 * Wh and Hh <= H and Wh <= W
            and high.is_contiguous(memory_format=torch.channels_last)
            and low.is_contiguous(memory_format=torch.channels_last)
            and high.data_ptr() % 16 == 0 and low.data_ptr() % 16 == 0):
        return _UpCat.apply(high, low)
    up = F.interpolate(high, scale_factor=2.0, mode="nearest")
    if up.shape[-2:] != low.shape[-2:]:
        up = up[..., :H, :W]
    return torch.cat([up, low], dim=1)


class DenseFFN(nn.Module):
    def __init__(self, d, hidden, act="relu"):
        super().__init__()
        self.linear1 = TokenLinear(d, hidden)
        self.linear2 = TokenLinear(hidden, d)
        self.act = nn.GELU() if act == "gelu" else nn.ReLU()

    def forward(self, x, ctx=None, residual=False):
        y = self.linear2(self.act(self.linear1(x)))
        return x + y if residual else y


def make_ffn(d, hidden, moe: MoEConfig | None, act="relu"):
    return MoEFFN(d, moe) if moe is not None else DenseFFN(d, hidden, act)


class TransformerEncoderLayer(nn.Module):
    """Post-norm encoder layer (AIFI): self-attention with 2-D sin-cos position
    added to q/k, then the (MoE) FFN."""

    def __init__(self, d=256, nhead=8, hidden=1024, moe: MoEConfig | None = None):
        super().__init__()
        self.self_attn = TokenSelfAttention(d, nhead)
        self.ffn = make_ffn(d, hidden, moe, act="relu")
        self.norm1 = AddLayerNorm(d)  # LayerNorm(a + b), fused on the GPU (norm.py)
        self.norm2 = AddLayerNorm(d)

    def forward(self, src, pos, ctx):
        src = self.norm1(src, self.self_attn(src + pos, src))
        src = self.norm2(self.ffn(src, ctx, residual=True))  # src + FFN(src)
        return src


class RepVggBlock(nn.Module):
    def __init__(self, cin, cout):
        super().__init__()
        self.conv1 = ConvNormLayer(cin, cout, 3, 1)
        self.conv2 = ConvNormLayer(cin, cout, 1, 1)

    def forward(self, x, resid=None):
        """silu(BN1(conv3x3 x) + BN2(conv1x1 x)) [+ resid: the CSPRep
        shortcut branch, added in the same pass on the fused path]."""
        if _FUSED_BN:
            norms = [self.conv1.norm, self.conv2.norm]
            if not self.conv1.norm.training and not torch.is_grad_enabled():  # inference: running statistics
                y = evalfold.conv_folded(self, x, resid)  # both branches + BNs folded: one 3x3 conv + SiLU (+ r)
                if y is not None:
                    return y
                y1, y2 = conv_pair(self.conv1.conv, self.conv2.conv, x)
                if bn_eval_ok([y1, y2], norms):  # both BNs + sum + SiLU (+ shortcut) in one HIP pass
                    return bn_act_eval([y1, y2], norms, "silu", resid=resid)
                y = F.silu(self.conv1.norm(y1) + self.conv2.norm(y2))
                return y if resid is None else y + resid
            # one node: dx accumulated in the dgrad, the BN statistics in the forward epilogues
            y1, y2, parts = conv_pair(self.conv1.conv, self.conv2.conv, x, stats=True)
            if bn_act_ok([y1, y2], norms):  # both BNs + sum + SiLU in HIP
                return bn_act([y1, y2], norms, "silu", parts, resid=resid)
            y = F.silu(self.conv1.norm(y1) + self.conv2.norm(y2))
        else:
            y = F.silu(self.conv1(x) + self.conv2(x))
        return y if resid is None else y + resid


class CSPRepLayer(nn.Module):
    def __init__(self, cin, cout, num_blocks=3, expansion=1.0):
        super().__init__()
        hidden = int(cout * expansion)
        self.conv1 = ConvNormLayer(cin, hidden, 1, 1, "silu")
        self.conv2 = ConvNormLayer(cin, hidden, 1, 1, "silu")
        self.bottlenecks = nn.Sequential(*[RepVggBlock(hidden, hidden) for _ in range(num_blocks)])
        self.conv3 = ConvNormLayer(hidden, cout, 1, 1, "silu") if hidden != cout else nn.Identity()

    def forward(self, x):
        c1, c2 = self.conv1, self.conv2
        if _FUSED_BN and not c1.fold and not c2.fold:
            if not c1.norm.training and not torch.is_grad_enabled():  # inference: running statistics
                a1, a2 = evalfold.conv_folded(c1, x), evalfold.conv_folded(c2, x)  # BN + SiLU folded
                if a1 is not None and a2 is not None:
                    return self.conv3(self._bottlenecks_plus(a1, a2))
                y1, y2 = conv_pair(c1.conv, c2.conv, x)
                if bn_eval_ok([y1], [c1.norm]) and bn_eval_ok([y2], [c2.norm]):
                    a1, a2 = bn_act_eval([y1], [c1.norm], "silu"), bn_act_eval([y2], [c2.norm], "silu")
                else:
                    a1, a2 = c1.act(c1.norm(y1)), c2.act(c2.norm(y2))
                return self.conv3(self._bottlenecks_plus(a1, a2))
            y1, y2, parts = conv_pair(c1.conv, c2.conv, x, stats=True)  # (as RepVggBlock)
            if bn_act_ok([y1], [c1.norm]) and bn_act_ok([y2], [c2.norm]):
                p1, p2 = (None, None) if parts is None else (parts[0:1], parts[1:2])
                a1, a2 = bn_act([y1], [c1.norm], "silu", p1), bn_act([y2], [c2.norm], "silu", p2)
            else:
                a1, a2 = c1.act(c1.norm(y1)), c2.act(c2.norm(y2))
            return self.conv3(self._bottlenecks_plus(a1, a2))
        return self.conv3(self.bottlenecks(self.conv1(x)) + self.conv2(x))

    def _bottlenecks_plus(self, h, a2):
        """bottlenecks(h) + a2, the add in the last RepVgg block's BatchNorm
        pass (RepVggBlock resid)."""
        blocks = list(self.bottlenecks)
        if not blocks or not all(isinstance(b, RepVggBlock) for b in blocks):
            return self.bottlenecks(h) + a2
        for b in blocks[:-1]:
            h = b(h)
        return blocks[-1](h, resid=a2)


def sincos_pos_embed_2d(w, h, dim=256, temperature=10000.0, device=None, dtype=torch.float32):
    gw = torch.arange(w, dtype=torch.float32, device=device)
    gh = torch.arange(h, dtype=torch.float32, device=device)
    gw, gh = torch.meshgrid(gw, gh, indexing="ij")
    pos_dim = dim // 4
    omega = 1.0 / temperature ** (torch.arange(pos_dim, dtype=torch.float32, device=device) / pos_dim)
    out_w = gw.flatten()[:, None] @ omega[None]
    out_h = gh.flatten()[:, None] @ omega[None]
    # [w*h, dim] in (x-major) order; transpose to row-major (h, w) token order
    emb = torch.cat([out_w.sin(), out_w.cos(), out_h.sin(), out_h.cos()], dim=1)
    emb = emb.view(w, h, dim).transpose(0, 1).reshape(h * w, dim)
    return emb[None].to(dtype)


class HybridEncoder(nn.Module):
    def __init__(self, in_channels=(512, 1024, 2048), strides=(8, 16, 32), hidden=256, nhead=8,
                 dim_feedforward=1024, use_encoder_idx=(2,), num_encoder_layers=1,
                 expansion=1.0, depth_mult=1.0, moe: MoEConfig | None = None):
        super().__init__()
        self.hidden = hidden
        self.use_encoder_idx = list(use_encoder_idx)
        self.strides = list(strides)
        self.input_proj = nn.ModuleList(
            [nn.Sequential(nn.Conv2d(c, hidden, 1, bias=False), nn.BatchNorm2d(hidden)) for c in in_channels])
        self.encoder = nn.ModuleList([
            nn.ModuleList([TransformerEncoderLayer(hidden, nhead, dim_feedforward, moe)
                           for _ in range(num_encoder_layers)]) for _ in self.use_encoder_idx])
        nb = round(3 * depth_mult)
        n = len(in_channels)
        self.lateral_convs = nn.ModuleList([ConvNormLayer(hidden, hidden, 1, 1, "silu") for _ in range(n - 1)])
        self.fpn_blocks = nn.ModuleList([CSPRepLayer(hidden * 2, hidden, nb, expansion) for _ in range(n - 1)])
        self.downsample_convs = nn.ModuleList([ConvNormLayer(hidden, hidden, 3, 2, "silu") for _ in range(n - 1)])
        self.pan_blocks = nn.ModuleList([CSPRepLayer(hidden * 2, hidden, nb, expansion) for _ in range(n - 1)])
        self._pos_cache = {}

    def _pos(self, w, h, device, dtype):
        key = (w, h, device, dtype)
        if key not in self._pos_cache:
            self._pos_cache[key] = sincos_pos_embed_2d(w, h, self.hidden, device=device, dtype=dtype)
        return self._pos_cache[key]

    @staticmethod
    def _proj(p, f):
        conv, bn = p[0], p[1]
        if _FUSED_BN:
            y = evalfold.conv_folded(p, f)  # inference: the BN folded into the convolution
            if y is not None:
                return y
            y = conv_module(conv, f)
            if bn_eval_ok([y], [bn]):  # inference: running statistics, one HIP pass
                return bn_act_eval([y], [bn], None)
            return bn_act([y], [bn], None) if bn_act_ok([y], [bn]) else bn(y)
        return p(f)

    def forward(self, feats, ctx):
        feats = stage_taps(feats)  # backbone outputs with a GradLink: gradient handed over, not accumulated
        proj = [self._proj(p, f) for p, f in zip(self.input_proj, feats)]
        for i, enc_ind in enumerate(self.use_encoder_idx):
            B, C, h, w = proj[enc_ind].shape
            src = proj[enc_ind].flatten(2).permute(0, 2, 1).contiguous()   # [B, h*w, C]
            pos = self._pos(w, h, src.device, src.dtype)
            for layer in self.encoder[i]:
                src = layer(src, pos, ctx)
            proj[enc_ind] = src.permute(0, 2, 1).reshape(B, C, h, w).contiguous(memory_format=torch.channels_last)
        n = len(proj)
        inner = [proj[-1]]
        for idx in range(n - 1, 0, -1):
            high = self.lateral_convs[n - 1 - idx](inner[0])
            inner[0] = high
            inner.insert(0, self.fpn_blocks[n - 1 - idx](up_cat(high, proj[idx - 1])))
        outs = [inner[0]]
        for idx in range(n - 1):
            src = outs[-1]
            if torch.is_grad_enabled() and src.requires_grad and src.is_cuda:
                # src is also an encoder output (the decoder's input projection
                # consumes it): its gradient from there joins this convolution's
                # dgrad epilogue (GradSlot), not an autograd add
                src.grad_slot = GradSlot()
            down = self.downsample_convs[idx](src)
            outs.append(self.pan_blocks[idx](torch.cat([down, inner[idx + 1]], dim=1)))
        return outs
