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
                 ("gdtype", "<i4"), ("group", "<i4"), ("hi_out", "<u8")])
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
    place and applies the 1/world mean (``inv_world``) inside its kernels.
    A parameter without a gradient on EVERY rank comes back as None (agreed
    over the group on the first call; torch.optim then skips it: no decay, no
    moment update), and ``broadcast_params`` gives every replica rank 0's
    weights at the start, as DDP does."""

    def __init__(self, params, group=None):
        self.params = list(params)
        self.group = group
        self._has_grad = None
        self._local_pattern = None
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

    def _world(self):
        return dist.get_world_size(self.group) if dist.is_available() and dist.is_initialized() else 1

    @torch.no_grad()
    def broadcast_params(self):
        """Rank 0's values of every replicated parameter on every rank (staged
        through the host on gloo); call before the optimizer copies its masters."""
        if self._world() <= 1:
            return
        gloo = dist.get_backend(self.group) == "gloo"
        for p in self.params:
            if gloo:
                h = p.detach().cpu()
                dist.broadcast(h, 0, group=self.group)
                p.copy_(h.to(p.device))
            else:
                dist.broadcast(p.data, 0, group=self.group)

    def _agree_has_grad(self, srcs):
        local = [0 if s is None else 1 for s in srcs]
        if self._has_grad is None:
            agg = torch.tensor(local, dtype=torch.int32)
            if self._world() > 1:
                if dist.get_backend(self.group) == "gloo":
                    dist.all_reduce(agg, group=self.group)
                else:
                    d = agg.to(self.flat.device)
                    dist.all_reduce(d, group=self.group)
                    agg = d.cpu()
            self._has_grad = (agg > 0).tolist()
            self._local_pattern = local
        elif local != self._local_pattern:
            raise RuntimeError("DPGradReducer: the set of parameters with a gradient changed after the first step")

    @torch.no_grad()
    def __call__(self, grads):
        srcs = [self._source(i, p, g) for i, (p, g) in enumerate(zip(self.params, grads))]
        self._agree_has_grad(srcs)
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
        if self._world() > 1:
            dist.all_reduce(self.flat, group=self.group)
        return [v if h else None for v, h in zip(self.views, self._has_grad)]


def _collective(kind, out, inp, group):
    """reduce_scatter_tensor (sum) / all_gather_into_tensor; device tensors on a
    gloo group (several ranks sharing one GPU in the tests) are staged through
    the host, which gloo needs."""
    fn = dist.reduce_scatter_tensor if kind == "rs" else dist.all_gather_into_tensor
    if out.is_cuda and dist.get_backend(group) == "gloo":
        o = torch.empty(out.shape, dtype=out.dtype)
        fn(o, inp.detach().cpu(), group=group)
        out.copy_(o.to(out.device))
    else:
        fn(out, inp, group=group)


class ShardedDPAdamW:
    """Data-parallel AdamW with the optimizer state sharded over the ranks
    (ZeRO-1; SURVEY.md 8(e) C3, the DP exchange redesigned for point-to-point
    xGMI).  Per step, on the ``group`` of W ranks:

      1. ONE ``train_grad_pack`` launch widens every replicated gradient (bf16
         GEMM / conv operands, fp32 otherwise) to fp32 into a flat buffer laid
         out rank-block-major: block r = rank r's slice of the bf16-parameter
         space, then its slice of the fp32-parameter space (a tensor that
         straddles a slice boundary is packed as pieces);
      2. ONE reduce-scatter (fp32 sums, no bf16 rounding per ring hop) leaves
         each rank the summed gradient of its 1/W slice;
      3. clip norm: the squared norms of the local slice and of the rank-local
         expert-parallel shards (``sharded``), one fp32 scalar all-reduce, so
         every rank computes the global norm of the rank-mean gradient
         (torch's clip_grad_norm_ over the whole model);
      4. AdamW on the local slice only (fp32 masters / moments of 1/W of the
         replicated parameters + the local expert shards), writing the new
         bf16 (fp32) weights into this rank's slice of the flat parameter
         spaces;
      5. ONE all-gather per parameter space (bf16, and the small fp32 one)
         refreshes every rank's replicated weights in place.

    Per rank the collectives move (W-1)/W (4 B x replicated params + 2 B x
    bf16 params + 4 B x fp32 params) -- at C2's 68 M parameters ~357 MB at W = 8
    instead of the flat all-reduce's ~476 MB -- and the optimizer does 1/W of
    the work.  The replicated parameters become views of the two flat spaces
    (before any graph capture), broadcast from rank 0 once at construction so
    every replica starts identical.  A parameter whose gradient is None on
    every rank is skipped (torch.optim semantics: no decay, no moment update,
    no step count); the pattern is agreed over the group on the first step and
    must not change afterwards."""

    ALIGN = 8  # elements: every tensor / piece starts at a multiple (16-B / 32-B vectors)

    def __init__(self, groups, *, weight_decay=1e-4, betas=(0.9, 0.999), eps=1e-8, clip_norm=0.0, sharded=(),
                 group=None):
        if not 1 <= len(groups) <= 4:
            raise ValueError("ShardedDPAdamW: 1..4 parameter groups")
        if not (dist.is_available() and dist.is_initialized()):
            raise RuntimeError("ShardedDPAdamW needs torch.distributed initialised")
        self.group = group
        self.W = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.lrs = [float(lr) for _, lr in groups]
        self.wd = float(weight_decay)
        self.beta1, self.beta2 = (float(b) for b in betas)
        self.eps = float(eps)
        self.clip_norm = float(clip_norm)
        shard_ids = {id(p) for p in sharded}
        self.params, self.group_of = [], []
        for gi, (ps, _) in enumerate(groups):
            for p in ps:
                if p.dtype not in (torch.float32, torch.bfloat16) or not p.is_cuda:
                    raise ValueError("ShardedDPAdamW: CUDA fp32/bf16 parameters only")
                self.params.append(p)
                self.group_of.append(gi)
        dev = self.params[0].device
        self.device = dev
        A, W = self.ALIGN, self.W
        rep = [i for i, p in enumerate(self.params) if id(p) not in shard_ids]
        self.ep_idx = [i for i, p in enumerate(self.params) if id(p) in shard_ids]
        self.rep_idx = rep
        # ---- the two flat parameter spaces (bf16, fp32) of the replicated tensors ----
        self.space_of, self.poff, self.S, self.pieces = self.layout(
            {i: (0 if self.params[i].dtype == torch.bfloat16 else 1, self.params[i].numel()) for i in rep}, W, A)
        Sb, Sf = self.S
        self.PB = torch.zeros(Sb * W, dtype=torch.bfloat16, device=dev)
        self.PF = torch.zeros(Sf * W, dtype=torch.float32, device=dev)
        with torch.no_grad():
            for i in rep:
                p = self.params[i]
                sp = self.PB if self.space_of[i] == 0 else self.PF
                o = self.poff[i]
                sp[o:o + p.numel()].copy_(_storage_flat(p.detach()))
            self._bcast(self.PB)
            self._bcast(self.PF)
            for i in rep:
                p = self.params[i]
                sp = self.PB if self.space_of[i] == 0 else self.PF
                o = self.poff[i]
                if p.dtype == torch.bfloat16 and (sp.data_ptr() + 2 * o) % 16:
                    raise ValueError("ShardedDPAdamW: misaligned bf16 parameter view")
                p.data = sp[o:o + p.numel()].as_strided(p.shape, p.stride())
        # ---- gradient buffers: rank-block-major flat, and this rank's slice ----
        B = Sb + Sf
        self.G = torch.zeros(B * W, dtype=torch.float32, device=dev)
        self.Gs = torch.zeros(B, dtype=torch.float32, device=dev)
        # pack table (gradient pointers are filled per step when they change)
        self.pack_moff = np.array([r * B + (Sb if s else 0) + (i0 + self.poff[i] - r * self.S[s])
                                   for (i, i0, n, r, s) in self.pieces], dtype=np.int64)
        self.pack_chunks = self._chunks([n for (_, _, n, _, _) in self.pieces])
        # ---- optimizer state: this rank's slice (both spaces) + the expert shards ----
        mine = [(k, pc) for k, pc in enumerate(self.pieces) if pc[3] == self.rank]
        self.mine = mine
        ep_off, off = [], B
        for i in self.ep_idx:
            ep_off.append(off)
            off += (self.params[i].numel() + A - 1) // A * A
        self.ep_off = ep_off
        self.master = torch.zeros(max(off, A), dtype=torch.float32, device=dev)
        self.exp_avg = torch.zeros_like(self.master)
        self.exp_avg_sq = torch.zeros_like(self.master)
        with torch.no_grad():
            self.master[:Sb].copy_(self.PB[self.rank * Sb:(self.rank + 1) * Sb].float())
            self.master[Sb:B].copy_(self.PF[self.rank * Sf:(self.rank + 1) * Sf])
            for i, o in zip(self.ep_idx, ep_off):
                p = self.params[i]
                self.master[o:o + p.numel()].copy_(_storage_flat(p.detach()).float())
        n_ent = len(mine) + len(self.ep_idx)
        self.opt_chunks = self._chunks([pc[2] for _, pc in mine] + [self.params[i].numel() for i in self.ep_idx])
        self.partials = torch.empty(max(self.opt_chunks.shape[0], 1), dtype=torch.float32, device=dev)
        self.tot = torch.zeros(1, dtype=torch.float32, device=dev)
        self.coef = torch.zeros(2, dtype=torch.float32, device=dev)
        self.tsteps = torch.zeros(max(n_ent, 1), dtype=torch.int32, device=dev)
        self.steps = 0
        self._pack_ptrs = None
        self._pack_table = None
        self._opt_ptrs = None
        self._opt_table = None
        self._has_grad = None  # agreed (over the group) on the first step
        self._staged = {}

    @staticmethod
    def layout(tensors, W, A=8):
        """tensors {index: (space 0 bf16 / 1 fp32, numel)} -> (space_of,
        offset in the space (multiples of A), slice length per rank per space
        [Sb, Sf] (multiples of A), pieces): every tensor cut at the rank-slice
        boundaries of its space into pieces (index, start in the tensor,
        length, owning rank, space) -- the packing / optimizer units."""
        space_of, poff, tot = {}, {}, [0, 0]
        for i, (s, n) in tensors.items():
            space_of[i] = s
            poff[i] = tot[s]
            tot[s] += (n + A - 1) // A * A
        S = [max(A, (n + A * W - 1) // (A * W) * A) for n in tot]
        pieces = []
        for i, (s, n) in tensors.items():
            a, o = poff[i], poff[i]
            while a < o + n:
                r = a // S[s]
                b = min(o + n, (r + 1) * S[s])
                pieces.append((i, a - o, b - a, r, s))
                a = b
        return space_of, poff, S, pieces

    def _bcast(self, t):
        """Rank 0's values on every rank (staged through the host on gloo)."""
        if dist.get_backend(self.group) == "gloo":
            h = t.detach().cpu()
            dist.broadcast(h, 0, group=self.group)
            t.copy_(h.to(t.device))
        else:
            dist.broadcast(t, 0, group=self.group)

    def _chunks(self, lengths):
        ch = [(k, c) for k, n in enumerate(lengths) for c in range((n + CHUNK - 1) // CHUNK)]
        return torch.tensor(ch if ch else [(0, 0)], dtype=torch.int32, device=self.device).reshape(-1, 2)

    def _source(self, i, g):
        p = self.params[i]
        if g is None:
            return None
        if g.shape != p.shape or g.dtype not in (p.dtype, torch.float32):
            raise ValueError("ShardedDPAdamW: gradient must have the parameter's shape and dtype (or fp32)")
        if g.stride() != p.stride() or g.data_ptr() % 16:
            buf = self._staged.get(i)
            if buf is None or buf.dtype != g.dtype:
                buf = self._staged[i] = torch.empty_strided(p.shape, p.stride(), dtype=g.dtype, device=p.device)
            buf.copy_(g)
            return buf
        return g

    def _agree_has_grad(self, srcs):
        local = torch.tensor([0 if s is None else 1 for s in srcs], dtype=torch.int32)
        if self._has_grad is None:
            agg = local.clone()
            if self.W > 1:
                if dist.get_backend(self.group) == "gloo":
                    dist.all_reduce(agg, group=self.group)
                else:
                    d = agg.to(self.device)
                    dist.all_reduce(d, group=self.group)
                    agg = d.cpu()
            self._has_grad = (agg > 0).tolist()
            self._local_pattern = local.tolist()
        elif local.tolist() != self._local_pattern:
            raise RuntimeError("ShardedDPAdamW: the set of parameters with a gradient changed after the first step")

    def _build_pack(self, srcs):
        rec = np.zeros(len(self.pieces), dtype=_REC)
        for k, (i, i0, n, r, s) in enumerate(self.pieces):
            g = srcs[i]
            rec[k]["grad"] = (g.data_ptr() + i0 * g.element_size()) if g is not None else 0
            rec[k]["numel"] = n
            rec[k]["moff"] = self.pack_moff[k]
            rec[k]["gdtype"] = 2 if g is None else (0 if g.dtype == torch.bfloat16 else 1)
        self._pack_table = torch.from_numpy(rec.view(np.uint8).copy()).to(self.device)

    def _build_opt(self, srcs):
        Sb, Sf = self.S
        rec = np.zeros(len(self.mine) + len(self.ep_idx), dtype=_REC)
        for k, (_, (i, i0, n, r, s)) in enumerate(self.mine):
            a = self.poff[i] + i0                    # element offset in the parameter space
            loc = a - r * self.S[s] + (Sb if s else 0)  # offset in this rank's slice / master
            rec[k]["grad"] = self.Gs.data_ptr() + 4 * loc
            rec[k]["numel"] = n
            rec[k]["moff"] = loc
            rec[k]["gdtype"] = 1 if self._has_grad[i] else 2
            rec[k]["group"] = self.group_of[i]
            if s == 0:
                rec[k]["lowp"] = self.PB.data_ptr() + 2 * a
            else:
                rec[k]["hi_out"] = self.PF.data_ptr() + 4 * a
        base = len(self.mine)
        for j, (i, o) in enumerate(zip(self.ep_idx, self.ep_off)):
            p, g = self.params[i], srcs[i]
            rec[base + j]["grad"] = g.data_ptr() if g is not None else 0
            rec[base + j]["numel"] = p.numel()
            rec[base + j]["moff"] = o
            rec[base + j]["gdtype"] = 2 if g is None else (0 if g.dtype == torch.bfloat16 else 1)
            rec[base + j]["group"] = self.group_of[i]
            if p.dtype == torch.bfloat16:
                rec[base + j]["lowp"] = p.data_ptr()
            else:
                rec[base + j]["hi_out"] = p.data_ptr()
        self._opt_table = torch.from_numpy(rec.view(np.uint8).copy()).to(self.device)

    @torch.no_grad()
    def step(self, grads=None, inv_world=None):
        """One clipped AdamW update of the rank-mean gradient from ``grads``
        (aligned with the parameters; default: each parameter's ``.grad``,
        the rank-local gradients -- the reduction happens here)."""
        if grads is None:
            grads = [p.grad for p in self.params]
        inv = 1.0 / self.W if inv_world is None else float(inv_world)
        srcs = [self._source(i, g) for i, g in enumerate(grads)]
        self._agree_has_grad(srcs)
        ptrs = tuple(s.data_ptr() if s is not None else 0 for s in srcs)
        if ptrs != self._pack_ptrs:
            self._build_pack(srcs)
            self._pack_ptrs = ptrs
        if ptrs != self._opt_ptrs:
            self._build_opt(srcs)
            self._opt_ptrs = ptrs
        self.steps += 1
        lib, s = L.lib(), L._stream()
        L._check(lib.train_grad_pack(self._pack_table.data_ptr(), self.pack_chunks.data_ptr(),
                                     self.pack_chunks.shape[0], self.G.data_ptr(), s), "train_grad_pack")
        _collective("rs", self.Gs, self.G, self.group)
        tab, nch = self._opt_table.data_ptr(), self.opt_chunks.shape[0]
        L._check(lib.train_grad_sqnorm(tab, self.opt_chunks.data_ptr(), nch, self.partials.data_ptr(), s),
                 "train_grad_sqnorm")
        torch.sum(self.partials[:nch], 0, keepdim=True, out=self.tot)
        if self.W > 1:
            if dist.get_backend(self.group) == "gloo":
                h = self.tot.cpu()
                dist.all_reduce(h, group=self.group)
                self.tot.copy_(h.to(self.device))
            else:
                dist.all_reduce(self.tot, group=self.group)
        n_ent = len(self.mine) + len(self.ep_idx)
        L._check(lib.train_grad_norm_finalize(self.tot.data_ptr(), 1, self.clip_norm, inv, self.coef.data_ptr(),
                                              tab, n_ent, self.tsteps.data_ptr(), s), "train_grad_norm_finalize")
        lrs = (ctypes.c_float * len(self.lrs))(*self.lrs)
        L._check(lib.train_adamw_step(tab, self.opt_chunks.data_ptr(), nch, self.coef.data_ptr(),
                                      self.master.data_ptr(), self.exp_avg.data_ptr(), self.exp_avg_sq.data_ptr(),
                                      self.tsteps.data_ptr(), lrs, len(self.lrs), self.wd, self.beta1, self.beta2,
                                      self.eps, s), "train_adamw_step")
        Sb, Sf = self.S
        _collective("ag", self.PB, self.PB[self.rank * Sb:(self.rank + 1) * Sb], self.group)
        _collective("ag", self.PF, self.PF[self.rank * Sf:(self.rank + 1) * Sf], self.group)

    def grad_norm(self) -> torch.Tensor:
        return self.coef[0]

    def reduced_grads(self):
        """Test / debug helper (one extra all-gather): the summed fp32
        gradient of every replicated parameter, {param index: tensor in the
        parameter's layout}, from the slices of the last step."""
        full = torch.empty_like(self.G)
        _collective("ag", full, self.Gs, self.group)
        Sb, Sf = self.S
        B = Sb + Sf
        out = {}
        for i in self.rep_idx:
            p = self.params[i]
            flat = torch.empty(p.numel(), dtype=torch.float32, device=self.device)
            s = self.space_of[i]
            for (j, i0, n, r, sp) in self.pieces:
                if j == i:
                    src = r * B + (Sb if sp else 0) + (i0 + self.poff[i] - r * self.S[sp])
                    flat[i0:i0 + n].copy_(full[src:src + n])
            out[i] = flat.as_strided(p.shape, p.stride())
        return out

    def master_of(self, p) -> torch.Tensor:
        """The fp32 master of parameter ``p`` (storage order, 1-D): gathered
        from the owning ranks for replicated parameters (a collective: call on
        every rank), local for expert shards."""
        for i, q in enumerate(self.params):
            if q is p:
                break
        else:
            raise KeyError("not a parameter of this optimizer")
        if i in self.ep_idx:
            o = self.ep_off[self.ep_idx.index(i)]
            return self.master[o:o + p.numel()]
        Sb, Sf = self.S
        B = Sb + Sf
        allm = torch.empty(B * self.W, dtype=torch.float32, device=self.device)
        _collective("ag", allm, self.master[:B], self.group)
        flat = torch.empty(p.numel(), dtype=torch.float32, device=self.device)
        for (j, i0, n, r, sp) in self.pieces:
            if j == i:
                src = r * B + (Sb if sp else 0) + (i0 + self.poff[i] - r * self.S[sp])
                flat[i0:i0 + n].copy_(allm[src:src + n])
        return flat
