"""PResNet-vd backbone (RT-DETR's R18/R34/R50/R101 body).

The reference trains RT-DETR through third-party engines that are absent here
(Ultralytics ``RTDETR``: src/models/vision/rtdetr.py:58-64, :82-94; RT-DETRv2
``rtdetrv2_r50vd`` configs named at scripts/train_rtdetr_thirdparty.py:30-35).
This is the build's own body for those configs:
ResNet-D stem (three 3x3 convs), AvgPool shortcut downsampling, stages
returning strides 8/16/32.  Runs channels_last under bf16 autocast (MIOpen
convolutions); nothing here is on the MoE hot path.
"""
from __future__ import annotations

import ctypes
import os

import torch
from torch import nn
import torch.nn.functional as F

from .conv import conv2d, conv2d_add_bias_relu_fork, conv2d_bias_relu, conv_module, conv_module_stats, hip_conv_ok_for
from .fused import AddBiasReLU, AddBiasReLUFork, BiasReLU, bn_act, bn_act_eval, bn_act_ok, bn_eval_ok

_FUSED_BN = os.environ.get("MOE_FUSED_BN", "1") != "0"  # A/B switch: training BN + SiLU in HIP
# A/B switch: frozen-BN shift + ReLU (+ residual add) in the HIP convolution's
# epilogue and ReLU backwards in the consumer's data-gradient epilogue
_FUSED_EPI = os.environ.get("MOE_CONV_EPI", "1") != "0"

_DEPTHS = {18: [2, 2, 2, 2], 34: [3, 4, 6, 3], 50: [3, 4, 6, 3], 101: [3, 4, 23, 3]}


class FrozenBatchNorm2d(nn.Module):
    """BatchNorm with fixed statistics and affine (RT-DETR ``freeze_norm``)."""

    def __init__(self, n, eps=1e-5):
        super().__init__()
        self.register_buffer("weight", torch.ones(n))
        self.register_buffer("bias", torch.zeros(n))
        self.register_buffer("running_mean", torch.zeros(n))
        self.register_buffer("running_var", torch.ones(n))
        self.eps = eps

    def scale_shift(self):
        """(scale, shift) of the frozen statistics, computed once and cached
        (recomputed only when a buffer changes, e.g. load_state_dict): five
        tiny kernels per layer per step otherwise, ~270 launches per C2 step."""
        key = (self.weight.device, self.weight._version, self.bias._version, self.running_mean._version,
               self.running_var._version)
        cache = getattr(self, "_ss_cache", None)
        if cache is None or cache[0] != key:
            with torch.no_grad():
                scale = self.weight * (self.running_var + self.eps).rsqrt()
                shift = self.bias - self.running_mean * scale
            if scale.is_cuda and torch.cuda.is_current_stream_capturing():
                return scale, shift  # first computed inside a capture: graph-owned, not cached
            cache = (key, scale, shift)
            self._ss_cache = cache
        # (a captured graph reads the cached tensors by address; frozen
        # statistics do not change while it is replayed)
        return cache[1], cache[2]

    def forward(self, x):
        scale, shift = self.scale_shift()
        # one fused multiply-add kernel (x * scale + shift)
        return torch.addcmul(shift.view(1, -1, 1, 1).to(x.dtype), x, scale.view(1, -1, 1, 1).to(x.dtype))


def _norm(n, frozen):
    return FrozenBatchNorm2d(n) if frozen else nn.BatchNorm2d(n)


class _FoldScale(torch.autograd.Function):
    """W' = W * scale[c_out] computed in fp32 and rounded once to W's dtype, in
    one kernel each way (TensorIterator promotes to fp32 and casts on store);
    the autograd chain float() -> mul -> to() it replaces took three kernels
    forward and three backward per convolution."""

    @staticmethod
    def forward(ctx, w, scale):
        s = scale.view(-1, *([1] * (w.dim() - 1)))
        out = torch.empty_like(w)
        torch.mul(w, s, out=out)
        ctx.save_for_backward(scale)
        return out

    @staticmethod
    def backward(ctx, g):
        from .conv import flush_wgrads

        flush_wgrads()  # g may be a deferred convolution weight gradient (conv.deferred_wgrads)
        (scale,) = ctx.saved_tensors
        s = scale.view(-1, *([1] * (g.dim() - 1)))
        gw = torch.empty_like(g)
        torch.mul(g, s, out=gw)
        return gw, None


class _FoldAll(torch.autograd.Function):
    """Every frozen-BN fold of the backbone (W'_l = W_l * scale_l) in ONE
    launch (rtdetr_fold_scale_multi) instead of one per convolution.  The
    folded weights live in buffers owned by the plan (fixed addresses: the
    device table is built once, outside any graph capture) and are returned
    as fresh views; the backward (dW_l = dW'_l * scale_l) is one kernel per
    tensor (the incoming gradients are new allocations)."""

    @staticmethod
    def forward(ctx, plan, *weights):
        plan.run()
        ctx.plan = plan
        outs = tuple(o.view_as(o) for o in plan.outs)
        frozen = [o for o, w in zip(outs, weights) if not w.requires_grad]
        if frozen:  # e.g. the frozen stem: no weight gradient is computed for it
            ctx.mark_non_differentiable(*frozen)
        ctx.set_materialize_grads(False)  # frozen folds: no zero-filled gradients
        return outs

    @staticmethod
    def backward(ctx, *grads):
        from .conv import flush_wgrads

        flush_wgrads()  # the convolutions' deferred weight-gradient sums land before they are scaled
        plan = ctx.plan
        out, jobs = [], []
        for g, sc in zip(grads, plan.scales):
            if g is None:
                out.append(None)
                continue
            gw = torch.empty_like(g)
            if _FOLD_BWD_BATCH and _fold_batch_ok(g, gw):
                jobs.append((g, sc, gw))  # bf16(g * scale[row]): one launch for all of them below
            else:
                torch.mul(g, sc.view(-1, *([1] * (g.dim() - 1))), out=gw)
            out.append(gw)
        if jobs:
            from ..moe import _lib as L

            for i in range(0, len(jobs), 64):
                part = jobs[i:i + 64]
                n = len(part)
                arr = [(ctypes.c_void_p * n)(*[t.data_ptr() for t in col]) for col in zip(*part)]
                rows = (ctypes.c_int * n)(*[g.shape[0] for g, _, _ in part])
                inner = (ctypes.c_int * n)(*[g.numel() // g.shape[0] for g, _, _ in part])
                c = lambda a: ctypes.cast(a, ctypes.c_void_p)  # noqa: E731
                L._check(L.lib().rtdetr_fold_scale_batch(n, c(arr[0]), c(arr[1]), c(arr[2]), c(rows), c(inner),
                                                         L._stream()), "rtdetr_fold_scale_batch")
        return (None, *out)


# MOE_FOLD_BWD_BATCH=0: one torch.mul per folded weight's gradient (A/B switch)
_FOLD_BWD_BATCH = os.environ.get("MOE_FOLD_BWD_BATCH", "1") != "0"
# the frozen stem on libmoe_hip: 1 = the direct 3 -> 32 kernel, 2 = also the
# 32 -> 32 / 32 -> 64 layers on the implicit GEMM; 0: modules (MIOpen)
_STEM_HIP = int(os.environ.get("MOE_STEM_HIP", "2"))


def _fold_batch_ok(g, gw):
    """rtdetr_fold_scale_batch takes the gradient (bf16, dense in the weight's
    layout: output channel outermost, 16-B aligned, whole 8-element groups)."""
    return (g.is_cuda and g.dtype == torch.bfloat16 and gw.stride() == g.stride() and g.data_ptr() % 16 == 0
            and gw.data_ptr() % 16 == 0 and (g.numel() // g.shape[0]) % 8 == 0 and g.numel() > 0
            and (g.is_contiguous() or g.is_contiguous(memory_format=torch.channels_last)))


class FoldPlan:
    """Device table of the backbone's folds (see _FoldAll)."""

    def __init__(self, layers):
        self.layers = layers
        self.outs = None
        self.key = None

    def _build(self):
        import numpy as np

        from ..moe import _lib as L

        ws = [l.conv.weight for l in self.layers]
        self.scales = [l.norm.scale_shift()[0].float().contiguous() for l in self.layers]
        self.outs = [torch.empty_like(w) for w in ws]
        rec = np.zeros(len(ws), dtype=[("w", "<u8"), ("s", "<u8"), ("o", "<u8"), ("rows", "<i4"), ("inner", "<i4")])
        chunks = []
        for i, (w, sc, o) in enumerate(zip(ws, self.scales, self.outs)):
            rec[i] = (w.data_ptr(), sc.data_ptr(), o.data_ptr(), w.shape[0], w.numel() // w.shape[0])
            chunks += [(i, c) for c in range((w.numel() + 2047) // 2048)]
        dev = ws[0].device
        self.table = torch.from_numpy(rec.view(np.uint8).copy()).to(dev)
        self.chunks = torch.tensor(chunks, dtype=torch.int32, device=dev)
        self.n_chunks = len(chunks)
        self.lib = L

    def usable(self):
        ws = [l.conv.weight for l in self.layers]
        return (len(ws) > 0 and all(w.is_cuda and w.dtype == torch.bfloat16 and (w.numel() // w.shape[0]) % 8 == 0
                                    and w.data_ptr() % 16 == 0 and
                                    (w.is_contiguous() or w.is_contiguous(memory_format=torch.channels_last))
                                    for w in ws))

    def run(self):
        key = tuple((l.conv.weight.data_ptr(), l.conv.weight.dtype, l.norm.scale_shift()[0].data_ptr())
                    for l in self.layers)
        if key != self.key:
            if torch.cuda.is_current_stream_capturing():
                raise RuntimeError("FoldPlan: first use inside a graph capture (run one eager step first)")
            self._build()
            self.key = key
        L = self.lib
        L._check(L.lib().rtdetr_fold_scale_multi(self.table.data_ptr(), self.chunks.data_ptr(), self.n_chunks,
                                                 L._stream()), "rtdetr_fold_scale_multi")


class ConvNormLayer(nn.Module):
    """Conv + BN + act.  With a frozen BN the BN folds into the convolution
    (scaled weights) and its shift is applied with the activation by one fused
    kernel (fused.BiasReLU); ``conv_shift`` leaves the shift to the caller
    (the block output adds it together with the shortcut, fused.AddBiasReLU)."""

    def __init__(self, cin, cout, k, s, act=None, frozen=False):
        super().__init__()
        self.conv = nn.Conv2d(cin, cout, k, s, (k - 1) // 2, bias=False)
        self.norm = _norm(cout, frozen)
        self.act_name = act
        self.act = nn.ReLU(inplace=True) if act == "relu" else (nn.SiLU(inplace=True) if act == "silu" else nn.Identity())
        self.fold = frozen and act in (None, "relu")

    def folded(self):
        """Frozen BN: (W * scale, shift); the folded weight PResNet.forward made
        for this step (one launch for all layers) is consumed."""
        scale, shift = self.norm.scale_shift()
        w = getattr(self, "_w_folded", None)  # set by PResNet.forward (one launch for all)
        self._w_folded = None
        if w is None:
            w = _FoldScale.apply(self.conv.weight, scale)
        return w, shift

    def conv_shift(self, x, folded=None):
        """Frozen BN: (conv(x, W * scale), shift) -- the BN output minus its shift."""
        w, shift = folded if folded is not None else self.folded()
        return conv2d(x, w, self.conv.stride, self.conv.padding), shift

    def hip_ok(self, x_like, cin, w):
        """Whether this layer's convolution runs on the HIP kernels for an input
        like x_like with cin channels (the fused epilogues need it)."""
        return (_FUSED_EPI and self.fold and x_like.shape[0] > 0
                and hip_conv_ok_for(x_like.is_cuda, x_like.dtype, cin, w, self.conv.stride, self.conv.padding))

    def bias_relu(self, x, folded, mask_input=False, grad_premasked=False, link=None):
        """relu(BN(conv(x))) with the frozen BN folded: one HIP launch when
        fused (hip_ok), else conv + the BiasReLU kernel."""
        w, shift = folded
        if mask_input or grad_premasked or self.hip_ok(x, x.shape[1], w):
            return conv2d_bias_relu(x, w, shift, mask_input, grad_premasked, link, self.conv.stride)
        y, _ = self.conv_shift(x, folded)
        return BiasReLU.apply(y, shift)

    def forward(self, x):
        if self.fold:
            y, shift = self.conv_shift(x)
            if self.act_name == "relu":
                return BiasReLU.apply(y, shift)
            return y + shift.view(1, -1, 1, 1).to(y.dtype)
        if self.act_name in (None, "silu") and _FUSED_BN:
            if not self.norm.training and not torch.is_grad_enabled():  # inference: running statistics
                from . import evalfold

                y = evalfold.conv_folded(self, x)  # BN (+ SiLU) folded into the convolution
                if y is not None:
                    return y
                y = conv_module(self.conv, x)
                if bn_eval_ok([y], [self.norm]):
                    return bn_act_eval([y], [self.norm], self.act_name)  # BN + SiLU in one HIP pass
                return self.act(self.norm(y))
            y, part = conv_module_stats(self.conv, x)  # (the BN statistics from the conv epilogue)
            if bn_act_ok([y], [self.norm]):
                return bn_act([y], [self.norm], self.act_name, part)  # BN + SiLU in HIP (training statistics)
            return self.act(self.norm(y))
        y = conv_module(self.conv, x)
        return self.act(self.norm(y))


class _AvgPool2x2(torch.autograd.Function):
    """AvgPool2d(2, 2) on channels_last bf16 through rtdetr_avgpool2x2_nhwc_fwd
    / _bwd (one launch each way, 16-B channel vectors)."""

    @staticmethod
    def forward(ctx, x, link=None):
        from ..moe import _lib as L

        B, C, H, W = x.shape
        y = torch.empty((B, C, H // 2, W // 2), dtype=x.dtype, device=x.device, memory_format=torch.channels_last)
        L._check(L.lib().rtdetr_avgpool2x2_nhwc_fwd(x.data_ptr(), B, H, W, C, y.data_ptr(), L._stream()),
                 "rtdetr_avgpool2x2_nhwc_fwd")
        ctx.shape = (B, C, H, W)
        ctx.link = link  # x is a block output whose other consumer is branch2a (GradLink, downsampling shortcut)
        return y

    @staticmethod
    def backward(ctx, gy):
        from ..moe import _lib as L

        B, C, H, W = ctx.shape
        gy = gy.contiguous(memory_format=torch.channels_last)
        if gy.data_ptr() % 16:
            gy = gy.clone(memory_format=torch.channels_last)
        gx = torch.empty((B, C, H, W), dtype=gy.dtype, device=gy.device, memory_format=torch.channels_last)
        link = ctx.link
        ext = None
        if link is not None and link.g_ext is not None and not link.ext_used and _ext_ok(link.g_ext, gx):
            ext = link.g_ext  # the encoder's gradient of this stage output (stage_taps), added in the same pass
            link.ext_used = True
        L._check(L.lib().rtdetr_avgpool2x2_nhwc_bwd_add(gy.data_ptr(), None if ext is None else ext.data_ptr(),
                                                         B, H, W, C, gx.data_ptr(), L._stream()),
                 "rtdetr_avgpool2x2_nhwc_bwd")
        if link is not None:  # handed to branch2a's dgrad epilogue (which autograd runs after this)
            link.g_short = gx
        return gx, None


def _ext_ok(ext, like):
    return (ext.dtype == like.dtype and ext.shape == like.shape and ext.data_ptr() % 16 == 0
            and ext.is_contiguous(memory_format=torch.channels_last))


class _StageTap(torch.autograd.Function):
    """Identity on a returned stage output (C3 / C4 / C5) for its external
    consumer (the encoder).  The output's other consumer, the next stage's
    first block, finishes its gradient through a GradLink (branch2a's dgrad
    epilogue adds the shortcut gradient and applies the ReLU mask); the
    external gradient must be masked too.  Backward: the gradient is parked on
    the link (no gradient returned, so autograd issues no accumulation add);
    the shortcut's average-pool backward adds it in the same pass, or the
    producing fork adds it (rtdetr_relu_grad2 / a masked add) when the link
    path does not run.  Autograd runs this right after the consumer's own
    backward (a node created after the whole backbone), before any node of
    the next stage -- when the consumer taps again (HybridEncoder.forward);
    PResNet's own tap on its outputs runs just before the producing fork."""

    @staticmethod
    def forward(ctx, x, link):
        ctx.link = link
        ctx.set_materialize_grads(False)
        return x.view_as(x)

    @staticmethod
    def backward(ctx, g):
        if g is not None:
            g = g.contiguous(memory_format=torch.channels_last)
            if g.data_ptr() % 16:
                g = g.clone(memory_format=torch.channels_last)
            link = ctx.link
            link.g_ext = g if link.g_ext is None else link.g_ext + g
            link.ext_used = False
        return None, None


# MOE_STAGE_TAP=0: no taps (A/B: the round-4 behaviour, where an external
# consumer's gradient of C3 / C4 was summed by autograd and, on the GradLink
# path, never masked -- tests/test_gpu_backbone.py::test_stage_outputs_with_external_consumer)
_STAGE_TAP = os.environ.get("MOE_STAGE_TAP", "1") != "0"


def stage_taps(feats):
    """The backbone outputs as the encoder should consume them: a block output
    that carries a GradLink goes through _StageTap (gradient handed over on the
    link); anything else as is."""
    if not (_STAGE_TAP and torch.is_grad_enabled()):
        return list(feats)
    out = []
    for f in feats:
        link = getattr(f, "grad_link", None)
        if link is not None and f.requires_grad:
            t = _StageTap.apply(f, link)
            t.grad_link = link  # (a consumer may tap again: the later tap hands over first)
            f = t
        out.append(f)
    return out


def stem_max_pool(x, pool: nn.MaxPool2d):
    """The stem's MaxPool2d(3, 2, 1): channels_last bf16 GPU activations that
    take no gradient (the frozen stem) go through rtdetr_maxpool3x3s2_nhwc_fwd
    (one 16-B-vector launch; torch's NHWC kernel took 157 us at C2)."""
    if (x.is_cuda and x.dtype == torch.bfloat16 and not (torch.is_grad_enabled() and x.requires_grad)
            and pool.kernel_size in (3, (3, 3)) and pool.stride in (2, (2, 2)) and pool.padding in (1, (1, 1))
            and pool.dilation in (1, (1, 1)) and not pool.ceil_mode and x.shape[1] % 8 == 0
            and x.is_contiguous(memory_format=torch.channels_last) and x.data_ptr() % 16 == 0):
        from ..moe import _lib as L

        B, C, H, W = x.shape
        y = torch.empty((B, C, (H - 1) // 2 + 1, (W - 1) // 2 + 1), dtype=x.dtype, device=x.device,
                        memory_format=torch.channels_last)
        L._check(L.lib().rtdetr_maxpool3x3s2_nhwc_fwd(x.data_ptr(), B, H, W, C, y.data_ptr(), L._stream()),
                 "rtdetr_maxpool3x3s2_nhwc_fwd")
        return y
    return pool(x)


def avg_pool_2x2(x, link=None):
    """AvgPool2d(2, 2, ceil_mode=True).  Even H and W (every RT-DETR input padded
    to a multiple of 32) take a reshape-mean over the channels_last layout, whose
    backward is one broadcast kernel (ROCm's NHWC avg_pool2d backward took
    ~400 us per call at 1280x736, batch 8); bf16 GPU activations take the
    HIP kernel pair (_AvgPool2x2), one 16-B-vector launch each way."""
    B, C, H, W = x.shape
    if H % 2 or W % 2 or not x.is_contiguous(memory_format=torch.channels_last):
        return F.avg_pool2d(x, 2, 2, 0, ceil_mode=True)
    if x.is_cuda and x.dtype == torch.bfloat16 and C % 8 == 0 and x.data_ptr() % 16 == 0:
        return _AvgPool2x2.apply(x, link)
    y = x.permute(0, 2, 3, 1).reshape(B, H // 2, 2, W // 2, 2, C).mean(dim=(2, 4))
    return y.permute(0, 3, 1, 2)


class _Shortcut(nn.Module):
    """ResNet-D shortcut: AvgPool(2) then 1x1 conv when downsampling."""

    def __init__(self, cin, cout, stride, frozen):
        super().__init__()
        self.down = stride == 2
        self.conv = ConvNormLayer(cin, cout, 1, 1, frozen=frozen)

    def forward(self, x):
        return self.conv(avg_pool_2x2(x) if self.down else x)

    def conv_shift(self, x, link=None):
        return self.conv.conv_shift(avg_pool_2x2(x, link) if self.down else x)


_NO_FORK = os.environ.get("MOE_BACKBONE_FORK", "1") == "0"
_NO_FOLD_ALL = os.environ.get("MOE_FOLD_ALL", "1") == "0"


def _fork_ok(short):
    """Whether _block_out takes its fused fork path for a block with this
    shortcut (given a folded, HIP-eligible last convolution).  Only then does
    the last convolution's dgrad apply the ReLU mask of its input, so the
    producer may skip its own ReLU backward (grad_premasked) only then."""
    return not _NO_FORK and (short is None or short.conv.fold)


def _block_out(last, short, h, x, folded_last=None, mask_input=False, link_in=None, short_link=None):
    """relu(last(h) + shortcut(x)) as a (main, shortcut) pair of handles on the
    same activation (see fused.AddBiasReLUFork).  With frozen BNs the two BN
    shifts join the residual add and the ReLU in one fused kernel -- the
    epilogue of last's HIP convolution when it has one (folded_last given and
    hip_ok; mask_input: h is a ReLU output only last consumes)."""
    if last.fold and _fork_ok(short) and folded_last is not None:
        wl, sl = folded_last
        if mask_input or last.hip_ok(h, h.shape[1], wl):
            b, bias = (x, sl) if short is None else short.conv_shift(x, short_link)
            if short is not None:
                bias = sl + bias
            return conv2d_add_bias_relu_fork(h, wl, b, bias, mask_input, link_in if short is None else None)
    if mask_input:  # the producer skipped its ReLU backward for the fork path's dgrad mask
        raise RuntimeError("_block_out: mask_input set but the fused fork path does not run")
    if last.fold and (short is None or short.conv.fold):
        a, sa = last.conv_shift(h, folded_last)
        b, bias = (x, sa) if short is None else short.conv_shift(x)
        if short is not None:
            bias = sa + bias
        if _NO_FORK:  # A/B switch (MOE_BACKBONE_FORK=0): autograd accumulate + mask
            y = AddBiasReLU.apply(a, b, bias)
            return y, y
        return AddBiasReLUFork.apply(a, b, bias)
    y = F.relu(last(h) + (x if short is None else short(x)))
    return y, y


_GRAD_LINK = os.environ.get("MOE_GRAD_LINK", "1") != "0"  # A/B switch for the GradLink hand-off


_DOWN_LINK = os.environ.get("MOE_DOWN_LINK", "1") != "0"  # A/B switch: GradLink through downsampling shortcuts


def _link_for(short, x, fused):
    """The previous block's GradLink when this block's shortcut is the
    identity -- or (round 4) the ResNet-D downsampling shortcut, whose
    average-pool backward hands its gradient over -- and both its first
    convolution and its output are fused (both ends of the hand-off run:
    branch2a's dgrad epilogue, this block's fork / shortcut)."""
    if not fused or not _GRAD_LINK:
        return None
    if short is not None and not (_DOWN_LINK and short.down and short.conv.fold):
        return None
    return getattr(x, "grad_link", None)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, cout, stride, shortcut, frozen):
        super().__init__()
        self.short = None if shortcut else _Shortcut(cin, cout, stride, frozen)
        self.branch2a = ConvNormLayer(cin, cout, 3, stride, "relu", frozen)
        self.branch2b = ConvNormLayer(cout, cout, 3, 1, None, frozen)

    def forward(self, x, x_short=None):
        """x feeds branch2a, x_short (default x) the shortcut; returns the
        (main, shortcut) handles of the output."""
        xs = x if x_short is None else x_short
        a, b = self.branch2a, self.branch2b
        if _FUSED_EPI and a.fold and b.fold and a.act_name == "relu" and x.is_cuda:
            fa, fb = a.folded(), b.folded()
            ok_a = a.hip_ok(x, x.shape[1], fa[0])
            ok_b = b.hip_ok(x, fa[0].shape[0], fb[0]) and _fork_ok(self.short)
            pre_ab = ok_a and ok_b  # branch2b's dgrad (the fork path of _block_out) masks branch2a's ReLU
            link = _link_for(self.short, x, ok_a and ok_b)
            h = a.bias_relu(x, fa, grad_premasked=pre_ab, link=link) if ok_a else a.bias_relu(x, fa)
            return _block_out(b, self.short, h, xs, fb, mask_input=pre_ab, link_in=link)
        return _block_out(self.branch2b, self.short, self.branch2a(x), xs)


class BottleNeck(nn.Module):
    expansion = 4

    def __init__(self, cin, cout, stride, shortcut, frozen):
        super().__init__()
        width = cout
        self.branch2a = ConvNormLayer(cin, width, 1, 1, "relu", frozen)
        self.branch2b = ConvNormLayer(width, width, 3, stride, "relu", frozen)
        self.branch2c = ConvNormLayer(width, cout * 4, 1, 1, None, frozen)
        self.short = None if shortcut else _Shortcut(cin, cout * 4, stride, frozen)

    def forward(self, x, x_short=None):
        """x feeds branch2a, x_short (default x) the shortcut; returns the
        (main, shortcut) handles of the output.  Fused (frozen BNs, HIP
        convolutions): each branch's shift + ReLU is its convolution's
        epilogue, the block output's residual add + ReLU is branch2c's, and
        branch2a's / branch2b's ReLU backwards run in the dgrad epilogue of the
        next convolution (their only consumer) where that one is HIP too."""
        xs = x if x_short is None else x_short
        a, b, c = self.branch2a, self.branch2b, self.branch2c
        if _FUSED_EPI and a.fold and b.fold and c.fold and x.is_cuda:
            fa, fb, fc = a.folded(), b.folded(), c.folded()
            ok_a = a.hip_ok(x, x.shape[1], fa[0])
            ok_b = b.hip_ok(x, fa[0].shape[0], fb[0])
            ok_c = c.hip_ok(x, fb[0].shape[0], fc[0]) and _fork_ok(self.short)
            pre_ab, pre_bc = ok_a and ok_b, ok_b and ok_c  # pre_bc: only when _block_out takes its fork path
            link = _link_for(self.short, x, ok_a and ok_c)
            h1 = a.bias_relu(x, fa, grad_premasked=pre_ab, link=link)
            h2 = b.bias_relu(h1, fb, mask_input=pre_ab, grad_premasked=pre_bc)
            return _block_out(c, self.short, h2, xs, fc, mask_input=pre_bc, link_in=link,
                              short_link=link if self.short is not None else None)
        return _block_out(self.branch2c, self.short, self.branch2b(self.branch2a(x)), xs)


class PResNet(nn.Module):
    def __init__(self, depth=50, return_idx=(1, 2, 3), freeze_norm=True, freeze_at=0):
        """freeze_norm / freeze_at follow the rtdetrv2_r50vd configuration named
        by the reference (scripts/train_rtdetr_thirdparty.py:30-35): frozen
        BatchNorm statistics in the backbone and a frozen stem (freeze_at=0),
        so neither the stem's weight gradient nor its input gradient is
        computed."""
        super().__init__()
        block = BottleNeck if depth >= 50 else BasicBlock
        c = 64
        self.stem = nn.Sequential(
            ConvNormLayer(3, c // 2, 3, 2, "relu", freeze_norm),
            ConvNormLayer(c // 2, c // 2, 3, 1, "relu", freeze_norm),
            ConvNormLayer(c // 2, c, 3, 1, "relu", freeze_norm),
        )
        self.pool = nn.MaxPool2d(3, 2, 1)
        ch_in = c
        self.stages = nn.ModuleList()
        self.out_channels = []
        for i, (n, cout) in enumerate(zip(_DEPTHS[depth], [64, 128, 256, 512])):
            stride = 1 if i == 0 else 2
            blocks = []
            for b in range(n):
                shortcut = b > 0 or (i == 0 and block is BasicBlock)
                blocks.append(block(ch_in, cout, stride if b == 0 else 1, shortcut, freeze_norm))
                ch_in = cout * block.expansion
            self.stages.append(nn.Sequential(*blocks))
            self.out_channels.append(ch_in)
        if freeze_at >= 0:
            for prm in self.stem.parameters():
                prm.requires_grad_(False)
            for st in self.stages[:freeze_at]:
                for prm in st.parameters():
                    prm.requires_grad_(False)
        self.return_idx = list(return_idx)
        self.out_channels = [self.out_channels[i] for i in self.return_idx]
        self.out_strides = [[4, 8, 16, 32][i] for i in self.return_idx]

    def _fold_all(self):
        """Fold every frozen BN of the stages (and stem) in one launch when all
        the folded weights are GPU bf16 (TrainStep precision "bf16")."""
        plan = getattr(self, "_fold_plan", None)
        if plan is None:  # the 16-B vector kernel needs whole 8-element groups per output channel
            layers = [m for m in self.modules() if isinstance(m, ConvNormLayer) and m.fold
                      and (m.conv.weight.numel() // m.conv.weight.shape[0]) % 8 == 0]
            plan = self._fold_plan = FoldPlan(layers)
        if _NO_FOLD_ALL or not plan.usable():  # A/B switch MOE_FOLD_ALL=0: one fold kernel per layer
            return
        need = torch.is_grad_enabled() and any(l.conv.weight.requires_grad for l in plan.layers)
        ws = [l.conv.weight for l in plan.layers]
        outs = _FoldAll.apply(plan, *ws) if need else (plan.run() or tuple(plan.outs))
        for l, w in zip(plan.layers, outs):
            l._w_folded = w

    @staticmethod
    def _stem_amp():
        return torch.is_autocast_enabled("cuda") and torch.get_autocast_dtype("cuda") == torch.bfloat16

    def _stem_hip_ok(self, x):
        """bf16 input and weights -- or fp32 ones under bf16 autocast (the
        evaluation forward, precision "amp"), cast as autocast would for the
        convolutions."""
        amp = self._stem_amp()
        ok_dt = (torch.bfloat16, torch.float32) if amp else (torch.bfloat16,)
        return (_STEM_HIP and x.is_cuda and x.dtype in ok_dt and x.dim() == 4 and x.shape[0] > 0
                and x.shape[1] == 3 and not x.requires_grad and x.is_contiguous(memory_format=torch.channels_last)
                and len(self.stem) == 3 and all(isinstance(l, ConvNormLayer) and l.fold and l.act_name == "relu"
                                                and l.conv.kernel_size == (3, 3) for l in self.stem)
                and [l.conv.out_channels for l in self.stem] == [32, 32, 64]
                and not any(p.requires_grad for p in self.stem.parameters())
                and all(l.conv.weight.dtype in ok_dt for l in self.stem))

    def _stem(self, x):
        """The frozen ResNet-D stem (three 3x3 conv + folded BN + ReLU).  GPU
        bf16 without gradients: the 3 -> 32 layer on the direct kernel
        (rtdetr_conv3x3_direct_fwd, bias + ReLU fused); with MOE_STEM_HIP=2
        also the 32 -> 32 / 32 -> 64 layers on the implicit-GEMM forward
        (32-deep K-tiles, bias + ReLU in its epilogue).  Elsewhere the
        modules."""
        if not self._stem_hip_ok(x):
            return self.stem(x)
        from ..moe import _lib as L
        from .conv import _fwd, _nhwc

        l1, l2, l3 = self.stem
        if x.dtype != torch.bfloat16:  # bf16 autocast: the convolution's own input cast
            x = x.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        w, shift = l1.folded()
        y = L.conv3x3_direct_fwd(x, w.to(torch.bfloat16), shift.float().contiguous(), l1.conv.stride[0], True)
        for l in (l2, l3):
            if _STEM_HIP >= 2:
                w, shift = l.folded()
                y = _fwd(y, _nhwc(w.to(torch.bfloat16)), shift.float().contiguous(), None, True, l.conv.stride[0])
            else:
                y = l(y)
        return y

    def forward(self, x):
        self._fold_all()
        x = stem_max_pool(self._stem(x), self.pool)
        xs = None
        outs = []
        for i, stage in enumerate(self.stages):
            for blk in stage:
                x, xs = blk(x, xs)
            if i in self.return_idx:
                outs.append(x)
        # returned outputs whose gradient the next stage finishes through a
        # GradLink: any external consumer's gradient reaches the link (masked
        # there), never an unmasked autograd sum (stage_taps)
        return stage_taps(outs)


@torch.no_grad()
def calibrate_frozen_bn(model: nn.Module, images: torch.Tensor, residual_gain: float | None = 0.1) -> int:
    """Data-dependent initialisation of every frozen BatchNorm: its running
    mean / variance become the per-channel statistics of its convolution's
    output on ``images`` (one forward pass, layer by layer).  A randomly
    initialised backbone with the default frozen statistics (mean 0, var 1)
    lets activations grow through ~50 layers, so bf16 rounding differences are
    amplified far beyond what a pretrained backbone (rtdetrv2_r50vd loads
    ImageNet weights + statistics) shows; the parity tests calibrate first so
    they measure the implementation, not a badly conditioned init.  With
    unit-variance branches a random ResNet is chaotic (a 0.2 % input
    perturbation grows to ~40 % at stage 5 in fp32 alone; 1 % with this gain), so the last BN of
    every residual branch also gets gamma = ``residual_gain`` (the
    small-residual init of trained ResNets; None keeps gamma).  Returns the
    number of layers calibrated (CPU or GPU, any dtype)."""
    layers = [m for m in model.modules() if isinstance(m, ConvNormLayer) and isinstance(m.norm, FrozenBatchNorm2d)]
    if residual_gain is not None:
        for blk in model.modules():
            last = getattr(blk, "branch2c", None) if isinstance(blk, BottleNeck) else \
                (getattr(blk, "branch2b", None) if isinstance(blk, BasicBlock) else None)
            if last is not None and isinstance(last.norm, FrozenBatchNorm2d):
                last.norm.weight.fill_(residual_gain)

    def pre(mod, args):
        x = args[0]
        y = F.conv2d(x, mod.conv.weight.to(x.dtype), None, mod.conv.stride, mod.conv.padding).float()
        mod.norm.running_mean.copy_(y.mean((0, 2, 3)))
        mod.norm.running_var.copy_(y.var((0, 2, 3), unbiased=False))
        mod._w_folded = None  # refold with the new statistics

    global _FUSED_EPI
    fused_was, _FUSED_EPI = _FUSED_EPI, False  # the fused blocks bypass ConvNormLayer.forward (no hook would fire)
    hooks = [m.register_forward_pre_hook(pre) for m in layers]
    for m in layers:  # block outputs call conv_shift directly (no forward hook fires there)
        m.conv_shift = (lambda x, folded=None, _m=m, _f=m.conv_shift: (pre(_m, (x,)), _f(x))[1])
    for m in model.modules():
        if isinstance(m, PResNet):
            m._fold_plan = None  # the one-launch fold caches the scales: rebuilt on next use
    was = model.training
    try:
        model.eval()
        (model.backbone if hasattr(model, "backbone") else model)(images)
    finally:
        model.train(was)
        for h in hooks:
            h.remove()
        for m in layers:
            del m.conv_shift
            m._w_folded = None
        _FUSED_EPI = fused_was
    return len(layers)
