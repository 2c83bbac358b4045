"""The decoder's query selection runs the encoder-output heads with autograd on
the selected rows only (decoder.py RTDETRDecoder.forward).  Check it against
the straightforward formulation (heads over every token, then gather), values
and gradients, on CPU."""
from __future__ import annotations

import torch

from src.rtdetr_moe.decoder import RTDETRDecoder


def _full_heads(dec, memory, shapes):
    anchors, valid = dec._anchors(shapes, memory.device, torch.float32)
    out_mem = dec.enc_output(valid.to(memory.dtype) * memory)
    enc_logits = dec.enc_score_head(out_mem)
    enc_coord = dec.enc_bbox_head(out_mem).float() + anchors
    topk = torch.topk(enc_logits.detach().float().max(-1).values, dec.num_queries, dim=1).indices
    boxes = enc_coord.gather(1, topk[..., None].expand(-1, -1, 4)).sigmoid()
    logits = enc_logits.gather(1, topk[..., None].expand(-1, -1, enc_logits.shape[-1]))
    return logits, boxes


def test_selected_rows_heads_match_full_heads():
    torch.manual_seed(0)
    dec = RTDETRDecoder(num_classes=3, hidden=32, feat_channels=(16, 16, 16), num_queries=20, num_layers=1,
                        nhead=4, dim_feedforward=64)
    for m in [dec.enc_bbox_head]:  # non-zero last layer so box gradients are exercised
        torch.nn.init.normal_(m.layers[-1].weight, std=0.1)
    feats = [torch.randn(2, 16, 8, 10), torch.randn(2, 16, 4, 5), torch.randn(2, 16, 2, 3)]
    out = dec(feats, None)
    proj = [p(f) for p, f in zip(dec.input_proj, feats)]
    shapes = [tuple(f.shape[-2:]) for f in proj]
    memory = torch.cat([f.flatten(2).permute(0, 2, 1) for f in proj], 1).contiguous()
    ref_logits, ref_boxes = _full_heads(dec, memory, shapes)
    got = out["enc_outputs"]
    torch.testing.assert_close(got["pred_logits"], ref_logits, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(got["pred_boxes"], ref_boxes, rtol=1e-5, atol=1e-6)

    params = [dec.enc_output[0].weight, dec.enc_score_head.weight, dec.enc_bbox_head.layers[0].weight]
    w = torch.randn_like(ref_logits)
    g_new = torch.autograd.grad((got["pred_logits"] * w).sum() + got["pred_boxes"].sum(), params, retain_graph=True)
    g_ref = torch.autograd.grad((ref_logits * w).sum() + ref_boxes.sum(), params)
    for a, b in zip(g_new, g_ref):
        torch.testing.assert_close(a, b, rtol=1e-4, atol=1e-6)


def test_token_linear_chunked_weight_grad():
    from src.rtdetr_moe.linear import _TokenLinear, chunked_wgrad

    torch.manual_seed(1)
    x = torch.randn(3, 2601, 24, dtype=torch.float64, requires_grad=True)  # rows not a multiple of the chunk
    w = torch.randn(16, 24, dtype=torch.float64, requires_grad=True)
    b = torch.randn(16, dtype=torch.float64, requires_grad=True)
    gy = torch.randn(3, 2601, 16, dtype=torch.float64)
    y = _TokenLinear.apply(x, w, b, torch.float64)
    torch.testing.assert_close(y, torch.nn.functional.linear(x, w, b))
    g = torch.autograd.grad((y * gy).sum(), (x, w, b))
    r = torch.autograd.grad((torch.nn.functional.linear(x, w, b) * gy).sum(), (x, w, b))
    for a, c in zip(g, r):  # dW is summed over chunks in fp32
        torch.testing.assert_close(a.to(c.dtype), c, rtol=1e-5, atol=1e-4)
    k = chunked_wgrad(gy.reshape(-1, 16), x.detach().reshape(-1, 24), target_chunk=1000)
    torch.testing.assert_close(k.double(), gy.reshape(-1, 16).t() @ x.detach().reshape(-1, 24), rtol=1e-5, atol=1e-4)
