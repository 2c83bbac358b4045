"""AddLayerNorm (src/rtdetr_moe/norm.py) on the CPU: the torch path equals
nn.LayerNorm(a + b) (same parameters and state-dict keys, forward and
gradients), and the encoder / decoder layers load an nn.LayerNorm state dict."""
from __future__ import annotations

import torch
from torch import nn


def test_add_layer_norm_cpu_matches_layernorm():
    from src.rtdetr_moe.norm import AddLayerNorm

    torch.manual_seed(0)
    ref = nn.LayerNorm(256)
    ref.weight.data.normal_(1.0, 0.1)
    ref.bias.data.normal_(0.0, 0.1)
    m = AddLayerNorm(256)
    m.load_state_dict(ref.state_dict())
    assert set(m.state_dict()) == {"weight", "bias"}
    a = torch.randn(2, 7, 256, requires_grad=True)
    b = torch.randn(2, 7, 256, requires_grad=True)
    a2, b2 = a.detach().clone().requires_grad_(True), b.detach().clone().requires_grad_(True)
    g = torch.randn(2, 7, 256)
    out = m(a, b)
    out.backward(g)
    exp = ref(a2 + b2)
    exp.backward(g)
    torch.testing.assert_close(out, exp)
    torch.testing.assert_close(a.grad, a2.grad)
    torch.testing.assert_close(b.grad, b2.grad)
    torch.testing.assert_close(m.weight.grad, ref.weight.grad)
    torch.testing.assert_close(m.bias.grad, ref.bias.grad)
    torch.testing.assert_close(m(a), ref(a))  # b = None: a plain LayerNorm


def test_layers_use_add_layer_norm():
    from src.moe.config import MoEConfig
    from src.rtdetr_moe.decoder import TransformerDecoderLayer
    from src.rtdetr_moe.encoder import TransformerEncoderLayer
    from src.rtdetr_moe.norm import AddLayerNorm

    enc = TransformerEncoderLayer(256, 8, 1024, MoEConfig(num_experts=4, top_k=1))
    dec = TransformerDecoderLayer(256, 8, 1024, 3, 4, MoEConfig(num_experts=4, top_k=1))
    for mod in (enc.norm1, enc.norm2, dec.norm1, dec.norm2, dec.norm3):
        assert isinstance(mod, AddLayerNorm) and isinstance(mod, nn.LayerNorm)
    # residual=True on the CPU (eager MoE path): x + FFN(x)
    x = torch.randn(2, 5, 256)
    ctx = torch.zeros(2, dtype=torch.int32)
    torch.testing.assert_close(enc.ffn(x, ctx, residual=True), x + enc.ffn(x, ctx))
