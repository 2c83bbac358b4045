"""Inference-mode re-parameterisation of the HybridEncoder and the decoder's
input projections (round 6): every trainable BatchNorm that runs on its
running statistics in evaluation is folded into the convolution in front of
it, and each RepVgg block's two branches become ONE 3x3 convolution:

  ConvNormLayer / input projection   act(BN(conv(x, W)))
      = act(conv(x, s W) + t)          s = gamma / sqrt(var + eps), t = beta - mean s
  RepVggBlock                        silu(BN1(conv3x3(x, W3)) + BN2(conv1x1(x, W1))) [+ r]
      = silu(conv3x3(x, s1 W3 + center(s2 W1)) + t1 + t2) [+ r]

(the RepVGG deployment identity: a 1x1 convolution is a 3x3 one whose only
non-zero tap is the centre).  The shift, the SiLU and the CSPRep shortcut r
run in the convolution's epilogue (rtdetr_conv_fwd_act), so the evaluation
forward has no BatchNorm pass and no 1x1 branch convolution left: the engine's
scripts/eval_detector.py path (reference scripts/eval_detector.py:99-116,
src/models/vision/rtdetr.py:98-128 eval_rtdetr_detector).

The folded weights are computed in fp32 from the current parameters and
running statistics and rounded once to bf16, when the model enters eval mode
(``refresh``, called from RTDETRMoE.train(False)); they are written into
persistent buffers in place, so graphs captured by engine.EvalForward keep
reading valid addresses across validations.  Training (train(True)) marks
them stale; the training forward never reads them.
MOE_EVAL_FOLD=0 keeps the unfolded inference path (conv + one BatchNorm / SiLU
pass, fused.bn_act_eval) as the A/B switch.
"""
from __future__ import annotations

import os

import torch
from torch import nn

_ON = os.environ.get("MOE_EVAL_FOLD", "1") != "0"


def _scale_shift(bn: nn.BatchNorm2d):
    s = bn.weight.detach().float() / torch.sqrt(bn.running_var.detach().float() + bn.eps)
    t = bn.bias.detach().float() - bn.running_mean.detach().float() * s
    return s, t


def _foldable_bn(bn) -> bool:
    return (isinstance(bn, nn.BatchNorm2d) and bn.affine and bn.track_running_stats
            and bn.running_mean is not None and bn.running_var is not None)


def _store(mod: nn.Module, w: torch.Tensor, b: torch.Tensor, act: int, stride: int = 1):
    """Write (bf16 channels_last weight, fp32 bias) into mod's persistent fold
    buffers (same addresses on every refresh of the same shape and device);
    mod._eval_fold = (weight, bias, act, stride)."""
    w = w.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    b = b.float().contiguous()
    old = getattr(mod, "_eval_fold", None)
    if (old is not None and old[0].shape == w.shape and old[0].device == w.device
            and old[1].shape == b.shape):
        old[0].copy_(w)
        old[1].copy_(b)
        mod._eval_fold = (old[0], old[1], act, stride)
    else:
        mod._eval_fold = (w, b, act, stride)


def fold_conv_bn(mod: nn.Module, conv: nn.Conv2d, bn: nn.BatchNorm2d, act: int):
    s, t = _scale_shift(bn)
    _store(mod, conv.weight.detach().float() * s.view(-1, 1, 1, 1), t, act, conv.stride[0])


def fold_repvgg(block: nn.Module):
    c3, c1 = block.conv1, block.conv2
    s3, t3 = _scale_shift(c3.norm)
    s1, t1 = _scale_shift(c1.norm)
    w = c3.conv.weight.detach().float() * s3.view(-1, 1, 1, 1)
    w[:, :, 1, 1] += c1.conv.weight.detach().float()[:, :, 0, 0] * s1.view(-1, 1)
    _store(block, w, t3 + t1, 2)


def refresh(model: nn.Module):
    """Fold every eligible layer of ``model`` (called when it enters eval mode)."""
    from .backbone import ConvNormLayer
    from .encoder import HybridEncoder, RepVggBlock

    if not _ON:
        return
    with torch.no_grad():
        # a RepVgg block's own two ConvNormLayers are folded into the block's weight, not on their own
        inner = {id(c) for b in model.modules() if isinstance(b, RepVggBlock) for c in (b.conv1, b.conv2)}
        for m in model.modules():
            if id(m) in inner:
                continue
            if isinstance(m, RepVggBlock):
                c3, c1 = m.conv1, m.conv2
                if (_foldable_bn(c3.norm) and _foldable_bn(c1.norm) and c3.conv.kernel_size == (3, 3)
                        and c1.conv.kernel_size == (1, 1) and c3.conv.stride == (1, 1) and c1.conv.stride == (1, 1)
                        and c3.conv.bias is None and c1.conv.bias is None):
                    fold_repvgg(m)
            elif isinstance(m, ConvNormLayer):
                if (not m.fold and _foldable_bn(m.norm) and m.conv.bias is None and m.act_name in (None, "silu")
                        and m.conv.stride[0] == m.conv.stride[1] and m.conv.groups == 1):
                    fold_conv_bn(m, m.conv, m.norm, 2 if m.act_name == "silu" else 0)
            elif isinstance(m, nn.Sequential) and len(m) == 2 and isinstance(m[0], nn.Conv2d) \
                    and m[0].bias is None and _foldable_bn(m[1]) and _is_input_proj(model, m):
                fold_conv_bn(m, m[0], m[1], 0)
        for m in model.modules():
            if isinstance(m, HybridEncoder) or hasattr(m, "_eval_fold"):
                m._eval_fold_ready = True


def invalidate(model: nn.Module):
    for m in model.modules():
        if hasattr(m, "_eval_fold_ready"):
            m._eval_fold_ready = False


def _is_input_proj(model, seq) -> bool:
    """The encoder's and the decoder's input projections (1x1 conv + BN)."""
    from .decoder import RTDETRDecoder
    from .encoder import HybridEncoder

    for owner in model.modules():
        if isinstance(owner, (HybridEncoder, RTDETRDecoder)) and any(seq is p for p in owner.input_proj):
            return True
    return False


def folded(mod: nn.Module, x: torch.Tensor):
    """mod's (weight, bias, act) when the folded inference path applies to
    input x: eval mode, no autograd, refreshed folds, a bf16 channels_last GPU
    input the HIP convolution takes; else None."""
    ef = getattr(mod, "_eval_fold", None)
    if (ef is None or not _ON or mod.training or torch.is_grad_enabled()
            or not getattr(mod, "_eval_fold_ready", False)):
        return None
    from .conv import hip_conv_ok

    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.device == ef[0].device
            and hip_conv_ok(x, ef[0], ef[3], (ef[0].shape[-1] - 1) // 2)):
        return None
    return ef


def conv_folded(mod: nn.Module, x: torch.Tensor, resid=None, out=None, out_row=0):
    """act(conv(x, W') + b') [+ resid after the activation] in one launch, or
    None when the folded path does not apply (out / out_row: conv.conv_act_eval)."""
    ef = folded(mod, x)
    if ef is None:
        return None
    w, b, act, st = ef
    from .conv import conv_act_eval

    if resid is not None and not (resid.is_cuda and resid.dtype == torch.bfloat16):
        return None
    return conv_act_eval(x, w, b, act, resid=resid, st=st, out=out, out_row=out_row)
