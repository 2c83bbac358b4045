"""FlatAdamW (csrc/optim.hip: grad-norm clip + AdamW + bf16 weight refresh)
against torch.nn.utils.clip_grad_norm_ + torch.optim.AdamW on fp32 masters
(the semantics it restates; the reference trains through Ultralytics' AdamW,
src/models/vision/rtdetr.py:82-94).  Tolerance: fp32 masters within
rtol 2e-5 / atol 1e-7 of torch's (different fp32 operation order); bf16
weights exactly the RNE of FlatAdamW's own masters."""
from __future__ import annotations

import pytest
import torch

DEV = "cuda"


def _params(seed):
    g = torch.Generator().manual_seed(seed)
    shapes = [((37, 13, 3, 3), torch.bfloat16, True), ((37,), torch.bfloat16, False), ((5,), torch.float32, False),
              ((1000, 3), torch.float32, False), ((4096 + 7,), torch.bfloat16, False), ((2, 2049), torch.float32, False),
              ((64, 16, 1, 1), torch.bfloat16, True)]
    out = []
    for shp, dt, cl in shapes:
        t = (torch.randn(shp, generator=g) * 0.1).to(DEV)
        if cl:
            t = t.contiguous(memory_format=torch.channels_last)
        out.append(torch.nn.Parameter(t.to(dt)))
    return out


@pytest.mark.gpu
@pytest.mark.parametrize("clip", [0.0, 0.05, 100.0])
@pytest.mark.parametrize("inv_world", [1.0, 0.5])
def test_flat_adamw_matches_torch(hip_lib, clip, inv_world):
    from src.rtdetr_moe.optim import FlatAdamW, _storage_flat

    ps = _params(0)
    ref = [torch.nn.Parameter(p.detach().float().clone()) for p in ps]  # torch's fp32 masters (same strides)
    groups = [(ps[:3], 1e-3), (ps[3:], 3e-4)]
    opt = FlatAdamW(groups, weight_decay=1e-2, clip_norm=clip)
    topt = torch.optim.AdamW([{"params": ref[:3], "lr": 1e-3}, {"params": ref[3:], "lr": 3e-4}], lr=1e-3,
                             weight_decay=1e-2, foreach=False)
    g = torch.Generator().manual_seed(1)
    for step in range(4):
        grads = []
        for i, p in enumerate(ps):
            if step == 2 and i == 4:  # no gradient this step: skipped by both
                grads.append(None)
                continue
            gr = (torch.randn(p.shape, generator=g) * (0.3 + i)).to(DEV).to(p.dtype)
            if p.dim() == 4:
                gr = gr.contiguous(memory_format=torch.channels_last if step % 2 == 0 else torch.contiguous_format)
            grads.append(gr)
        for r, gr in zip(ref, grads):
            r.grad = None if gr is None else gr.float() * inv_world
        opt.step(grads, inv_world=inv_world)
        if clip > 0:
            torch.nn.utils.clip_grad_norm_([r for r in ref if r.grad is not None], clip, foreach=False)
        topt.step()
        torch.cuda.synchronize()
        for p, r in zip(ps, ref):
            m = opt.master_of(p)
            torch.testing.assert_close(m, _storage_flat(r.detach()), rtol=2e-5, atol=1e-7)
            if p.dtype == torch.bfloat16:
                assert torch.equal(_storage_flat(p.detach()), m.to(torch.bfloat16))
            else:
                assert torch.equal(_storage_flat(p.detach()), m)
        tn = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(r.grad) for r in ref if r.grad is not None]))
        if clip == 0.0:
            tn = torch.linalg.vector_norm(torch.stack([torch.linalg.vector_norm(gr.float() * inv_world)
                                                       for gr in grads if gr is not None]))
        assert abs(float(opt.grad_norm()) - float(tn)) <= 1e-4 * float(tn) or clip > 0
