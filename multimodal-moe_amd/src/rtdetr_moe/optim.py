"""Flat mixed-precision AdamW on the GPU (libmoe_hip ``train_*`` kernels).

The training step's optimizer.  Semantics are torch's: the gradient clip of
``torch.nn.utils.clip_grad_norm_`` (global 2-norm, scale min(1, max/(norm+1e-6)))
followed by ``torch.optim.AdamW`` (decoupled weight decay, bias-corrected
moments) with fp32 master weights -- the reference trains through Ultralytics'
AdamW inside ``RTDETR.train`` (``src/models/vision/rtdetr.py:82-94``).

Layout: one flat fp32 buffer each for the master weights, exp_avg and
exp_avg_sq; every parameter owns a segment starting at a multiple of 8
elements.  fp32 parameters (norms, router, ...) ARE their master segment
(``p.data`` is a view of it), so the update writes them in place; bf16
parameters (GEMM / convolution operands, TrainStep precision "bf16") keep
their own storage, which the kernel refreshes with the RNE of the new master.
Gradients are read where autograd (or the backward hipGraph) left them,
through a device table rebuilt only when a gradient address changes -- three
launches per step instead of ~400 per-tensor casts, norms and scales.
"""
from __future__ import annotations

import ctypes

import numpy as np
import torch
import torch.distributed as dist

from ..moe import _lib as L

CHUNK = 2048  # elements per workgroup (csrc/optim.hip OPT_CHUNK)
_REC = np.dtype([("grad", "<u8"), ("lowp", "<u8"), ("numel", "<i8"), ("moff", "<i8"),
                 ("gdtype", "<i4"), ("group", "<i4"), ("pad0", "<i4"), ("pad1", "<i4")])
assert _REC.itemsize == 48


def _storage_flat(t: torch.Tensor) -> torch.Tensor:
    """1-D view of a dense tensor in STORAGE order (e.g. channels_last conv
    weights), so masters, gradients and bf16 weights line up element by element."""
    dims = sorted(range(t.dim()), key=lambda i: -t.stride(i))
    expect = 1
    for i in reversed(dims):
        if t.size(i) != 1 and t.stride(i) != expect:
            raise ValueError(f"FlatAdamW: tensor with strides {t.stride()} is not dense")
        expect *= t.size(i)
    return t.as_strided((t.numel(),), (1,))


class FlatAdamW:
    """``groups``: list of (params, lr).  Parameters must be CUDA tensors of
    dtype fp32 or bf16 on one device."""

    def __init__(self, groups, *, weight_decay=1e-4, betas=(0.9, 0.999), eps=1e-8, clip_norm=0.0, sharded=(),
                 shard_group=None):
        """``sharded``: parameters each rank holds a different shard of (the
        expert-parallel experts).  The clip norm is global:
        their squared-norm partial is summed over ``shard_group`` (one fp32
        all-reduce) before the norm is finalised, so every rank computes the
        same clip coefficient (torch's clip_grad_norm_ over the whole model)."""
        if not 1 <= len(groups) <= 4:
            raise ValueError("FlatAdamW: 1..4 parameter groups")
        self.lrs = [float(lr) for _, lr in groups]
        self.wd = float(weight_decay)
        self.beta1, self.beta2 = (float(b) for b in betas)
        self.eps = float(eps)
        self.clip_norm = float(clip_norm)
        self.params, self.group_of, self.offsets = [], [], []
        off = 0
        for gi, (ps, _) in enumerate(groups):
            for p in ps:
                if p.dtype not in (torch.float32, torch.bfloat16) or not p.is_cuda:
                    raise ValueError("FlatAdamW: CUDA fp32/bf16 parameters only")
                self.params.append(p)
                self.group_of.append(gi)
                self.offsets.append(off)
                off += (p.numel() + 7) // 8 * 8
        dev = self.params[0].device
        self.device = dev
        self.total = off
        self.master = torch.zeros(off, dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        for p, o in zip(self.params, self.offsets):
            if p.dtype == torch.bfloat16 and p.data_ptr() % 16:
                raise ValueError("FlatAdamW: bf16 parameters must be 16-B aligned (vector stores)")
            seg = self.master[o:o + p.numel()]
            seg.copy_(_storage_flat(p.detach()).float())
            if p.dtype == torch.float32:  # the parameter is its master (same strides)
                p.data = seg.as_strided(p.shape, p.stride())
        shard_ids = {id(p) for p in sharded}
        self.shard_group = shard_group
        # chunks of replicated tensors first, then the sharded ones: the norm's
        # partials of the latter are the tail [n_rep_chunks, n_chunks)
        order = [i for i, p in enumerate(self.params) if id(p) not in shard_ids] + \
                [i for i, p in enumerate(self.params) if id(p) in shard_ids]
        chunks = [(i, c) for i in order for c in range((self.params[i].numel() + CHUNK - 1) // CHUNK)]
        self.n_rep_chunks = sum((self.params[i].numel() + CHUNK - 1) // CHUNK for i in order
                                if id(self.params[i]) not in shard_ids)
        self.chunks = torch.tensor(chunks, dtype=torch.int32, device=dev).reshape(-1, 2)
        self.n_chunks = len(chunks)
        self.partials = torch.empty(max(self.n_chunks, 1), dtype=torch.float32, device=dev)
        self.coef = torch.zeros(2, dtype=torch.float32, device=dev)  # [grad norm, applied grad scale]
        self.tsteps = torch.zeros(len(self.params), dtype=torch.int32, device=dev)  # per-tensor AdamW step
        self._staged = {}  # param index -> buffer with the parameter's strides (gradient in another layout)
        self._ptrs = None
        self._table = None
        self.steps = 0

    # -- gradient table ---------------------------------------------------
    def _grad_source(self, i, p, g):
        if g is None:  # skipped this step (torch.optim semantics): gdtype 2
            return None
        if g.shape != p.shape or g.dtype not in (p.dtype, torch.float32):
            raise ValueError("FlatAdamW: gradient must have the parameter's shape and dtype (or fp32)")
        if g.stride() != p.stride() or g.data_ptr() % 16:  # stage in the parameter's layout, 16-B aligned
            buf = self._staged.get(i)
            if buf is None or buf.dtype != g.dtype:
                buf = self._staged[i] = torch.empty_strided(p.shape, p.stride(), dtype=g.dtype, device=p.device)
            buf.copy_(g)
            return buf
        return g

    def _build_table(self, srcs):
        rec = np.zeros(len(self.params), dtype=_REC)
        for i, (p, g) in enumerate(zip(self.params, srcs)):
            rec[i]["grad"] = g.data_ptr() if g is not None else 0
            rec[i]["lowp"] = p.data_ptr() if p.dtype == torch.bfloat16 else 0
            rec[i]["numel"] = p.numel()
            rec[i]["moff"] = self.offsets[i]
            rec[i]["gdtype"] = 2 if g is None else (0 if g.dtype == torch.bfloat16 else 1)
            rec[i]["group"] = self.group_of[i]
        self._table = torch.from_numpy(rec.view(np.uint8).copy()).to(self.device)

    # -- step --------------------------------------------------------------
    @torch.no_grad()
    def step(self, grads=None, inv_world=1.0):
        """One clipped AdamW update from ``grads`` (aligned with the parameters;
        default: each parameter's ``.grad``).  ``inv_world`` scales gradients
        that hold a sum over data-parallel ranks."""
        if grads is None:
            grads = [p.grad for p in self.params]
        srcs = [self._grad_source(i, p, g) for i, (p, g) in enumerate(zip(self.params, grads))]
        ptrs = tuple(s.data_ptr() if s is not None else 0 for s in srcs)
        if ptrs != self._ptrs:
            self._build_table(srcs)
            self._ptrs = ptrs
        self.steps += 1
        lib, s = L.lib(), L._stream()
        tab = self._table.data_ptr()
        L._check(lib.train_grad_sqnorm(tab, self.chunks.data_ptr(), self.n_chunks, self.partials.data_ptr(), s),
                 "train_grad_sqnorm")
        self._reduce_sharded_partials()
        L._check(lib.train_grad_norm_finalize(self.partials.data_ptr(), self.n_chunks, self.clip_norm,
                                              float(inv_world), self.coef.data_ptr(), tab, len(self.params),
                                              self.tsteps.data_ptr(), s), "train_grad_norm_finalize")
        lrs = (ctypes.c_float * len(self.lrs))(*self.lrs)
        L._check(lib.train_adamw_step(tab, self.chunks.data_ptr(), self.n_chunks, self.coef.data_ptr(),
                                      self.master.data_ptr(), self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                                      self.tsteps.data_ptr(), lrs, len(self.lrs), self.wd, self.beta1, self.beta2,
                                      self.eps, s), "train_adamw_step")

    def _reduce_sharded_partials(self):
        """Sum the sharded tensors' squared-norm partials over the shard group:
        their total (identical on every rank after the all-reduce) replaces the
        first tail partial, the rest of the tail is zeroed; the finalize kernel
        then sums replicated + all shards in a fixed order."""
        n_rep, n = self.n_rep_chunks, self.n_chunks
        if n_rep == n or not (dist.is_available() and dist.is_initialized()):
            return
        if dist.get_world_size(self.shard_group) == 1:
            return
        tail = self.partials[n_rep:n]
        tot = tail.sum().reshape(1)
        dist.all_reduce(tot, group=self.shard_group)
        tail.zero_()
        tail[:1].copy_(tot)

    def master_of(self, p) -> torch.Tensor:
        """The fp32 master of parameter ``p`` (storage order, 1-D view)."""
        for q, o in zip(self.params, self.offsets):
            if q is p:
                return self.master[o:o + p.numel()]
        raise KeyError("not a parameter of this optimizer")

    def grad_norm(self) -> torch.Tensor:
        """Total gradient norm of the last step (device scalar, no sync)."""
        return self.coef[0]

    def state_dict(self):
        return {"steps": self.steps, "lrs": list(self.lrs), "master": self.master, "exp_avg": self.exp_avg,
                "exp_avg_sq": self.exp_avg_sq, "tensor_steps": self.tsteps}

    def load_state_dict(self, sd):
        self.steps = int(sd["steps"])
        self.lrs = [float(x) for x in sd["lrs"]]
        self.master.copy_(sd["master"])
        self.exp_avg.copy_(sd["exp_avg"])
        self.exp_avg_sq.copy_(sd["exp_avg_sq"])
        self.tsteps.copy_(sd["tensor_steps"])
        with torch.no_grad():
            for p, o in zip(self.params, self.offsets):
                if p.dtype == torch.bfloat16:
                    _storage_flat(p).copy_(self.master[o:o + p.numel()])



class DPGradReducer:
    """Data-parallel gradient sum in fp32.

    The replicated parameters' gradients (bf16 for GEMM / convolution
    operands, fp32 otherwise) are widened into ONE flat fp32 buffer by one HIP
    launch (``train_grad_pack``; a tensor without a gradient contributes
    zeros) and summed over the ranks with ONE all-reduce, so no ring hop
    rounds a partial sum to bf16.  ``__call__`` returns fp32 views of the
    summed gradients in the parameters' own layouts; FlatAdamW reads them in
    place and applies the 1/world mean (``inv_world``) inside its kernels."""

    def __init__(self, params, group=None):
        self.params = list(params)
        self.group = group
        self.offsets, off = [], 0
        for p in self.params:
            self.offsets.append(off)
            off += (p.numel() + 7) // 8 * 8
        dev = self.params[0].device
        self.flat = torch.zeros(max(off, 8), dtype=torch.float32, device=dev)
        self.views = [self.flat[o:o + p.numel()].as_strided(p.shape, p.stride())
                      for p, o in zip(self.params, self.offsets)]
        chunks = [(i, c) for i, p in enumerate(self.params) for c in range((p.numel() + CHUNK - 1) // CHUNK)]
        self.chunks = torch.tensor(chunks, dtype=torch.int32, device=dev).reshape(-1, 2)
        self.n_chunks = len(chunks)
        self._staged = {}
        self._ptrs = None
        self._table = None

    def _source(self, i, p, g):
        if g is None:
            return None
        if g.shape != p.shape or g.dtype != p.dtype:
            raise ValueError("DPGradReducer: gradient must have the parameter's shape and dtype")
        if g.stride() != p.stride() or g.data_ptr() % 16:
            buf = self._staged.get(i)
            if buf is None:
                buf = self._staged[i] = torch.empty_strided(p.shape, p.stride(), dtype=p.dtype, device=p.device)
            buf.copy_(g)
            return buf
        return g

    @torch.no_grad()
    def __call__(self, grads):
        srcs = [self._source(i, p, g) for i, (p, g) in enumerate(zip(self.params, grads))]
        ptrs = tuple(s.data_ptr() if s is not None else 0 for s in srcs)
        if ptrs != self._ptrs:
            rec = np.zeros(len(self.params), dtype=_REC)
            for i, (p, g) in enumerate(zip(self.params, srcs)):
                rec[i]["grad"] = g.data_ptr() if g is not None else 0
                rec[i]["numel"] = p.numel()
                rec[i]["moff"] = self.offsets[i]
                rec[i]["gdtype"] = 2 if g is None else (0 if g.dtype == torch.bfloat16 else 1)
            self._table = torch.from_numpy(rec.view(np.uint8).copy()).to(self.flat.device)
            self._ptrs = ptrs
        L._check(L.lib().train_grad_pack(self._table.data_ptr(), self.chunks.data_ptr(), self.n_chunks,
                                         self.flat.data_ptr(), L._stream()), "train_grad_pack")
        if dist.is_available() and dist.is_initialized() and dist.get_world_size(self.group) > 1:
            dist.all_reduce(self.flat, group=self.group)
        return self.views
