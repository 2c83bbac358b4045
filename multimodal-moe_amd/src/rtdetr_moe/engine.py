"""Training / validation engine (filled in below the DDP helpers)."""
from __future__ import annotations

import torch
from torch.nn.parallel import DistributedDataParallel as DDP


def wrap_ddp(model: torch.nn.Module, local_rank: int, bucket_cap_mb: int = 64) -> DDP:
    """Data-parallel wrapper over RCCL.  Expert weights
    that are sharded over an expert-parallel group (C4) are excluded from the
    gradient all-reduce."""
    ignore = [n for n, p in model.named_parameters() if getattr(p, "expert_parallel", False)]
    if ignore:
        DDP._set_params_and_buffers_to_ignore_for_model(model, ignore)
    return DDP(model, device_ids=[local_rank], output_device=local_rank, broadcast_buffers=False,
               gradient_as_bucket_view=True, bucket_cap_mb=bucket_cap_mb)
