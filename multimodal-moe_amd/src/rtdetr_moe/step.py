"""One RT-DETR-MoE training step, optionally with the model's forward and
backward captured as hipGraphs.

Why graphs: the model's forward + backward launch ~4,000 kernels (MIOpen
convolutions + BatchNorm, element-wise ops, 13 MoE launches x 7 layers);
issued eagerly from Python and the autograd engine, the host takes longer to
enqueue the backward than the GPU takes to run it.  Captured (GraphedModel),
the forward and the backward are one hipGraph replay each.  The backward graph
computes torch.autograd.grad of the forward outputs w.r.t. every trainable
parameter into static gradient buffers that the optimizer reads directly (no
per-parameter AccumulateGrad copies).  What stays eager: the Hungarian
matching (host linear_sum_assignment, one device->host copy of all cost
matrices), the batched set criterion, and the optimizer: when world > 1
the data-parallel reduction (one fp32 reduce-scatter over RCCL, AdamW on this
rank's slice, one all-gather of the weights: optim.ShardedDPAdamW), gradient
clipping and the fused AdamW update.

The captured forward keeps the MoE aux losses as an explicit graph output so
their gradients reach the router through the captured backward.
"""
from __future__ import annotations

import os
import time

import torch
import torch.distributed as dist
from torch import nn

from .conv import check_grad_slots
from .linear import TokenSelfAttention, deferred_weight_grads, merge_deferred
from .model import RTDETRMoE

_FUSED_CRIT = os.environ.get("MOE_FUSED_CRITERION", "1") != "0"  # A/B switch
# MOE_ZERO=0: GPU data parallelism through the flat fp32 all-reduce + replicated
# FlatAdamW (optim.DPGradReducer) instead of the sharded optimizer (A/B switch)
_ZERO = os.environ.get("MOE_ZERO", "1") != "0"

# Stream-capture mode of every hipGraph capture (step graphs, the evaluation
# forward): "thread_local", so that only the capturing thread is restricted.
# It is NOT what keeps a capture that holds RCCL collectives (the C4
# expert-parallel all-to-alls) alive -- quiesce_collectives is: the process
# group's watchdog thread polls the end events of recent eager collectives,
# and a poll that lands while the capture is open, with the RCCL stream joined
# into it, fails with hipErrorCapturedEvent and terminates the process (in
# either mode: tools/rccl_capture_probe.py, gpurun_out/r6b global, r6p
# thread_local; with the drain: r6c).
CAPTURE_MODE = "thread_local"
# Seconds to let the RCCL watchdog retire the warm-up's eager collectives
# before a capture opens (quiesce_collectives; its poll period is ~100 ms).
_DRAIN_S = float(os.environ.get("MOE_CAPTURE_DRAIN_S", "0.5"))


def rccl_env():
    """Call before every ``init_process_group("nccl")``: one CUDA event per
    collective instead of torch's recycled event cache, so that no event a
    capture recorded (captured collectives' end events) is ever handed to an
    eager collective that the watchdog then polls.  Together with
    quiesce_collectives this leaves the watchdog only eagerly recorded,
    completed events to look at."""
    os.environ.setdefault("TORCH_NCCL_CUDA_EVENT_CACHE", "0")


def quiesce_collectives():
    """Before opening a capture while an RCCL group is live: drain the device,
    then give the group's watchdog time to retire every completed eager
    collective, so that none of their events is polled while the capture is
    open (see CAPTURE_MODE).  No eager collective may be issued between this
    call and the end of the capture."""
    if not (dist.is_available() and dist.is_initialized()):
        return
    if "nccl" not in str(dist.get_backend()).lower():
        return
    torch.cuda.synchronize()
    if _DRAIN_S > 0:
        time.sleep(_DRAIN_S)


def _drop_autograd_graphs(model=None):
    """Release the autograd graphs of the warm-up / capture passes now.  Two
    things keep such a graph -- and the parameters' AccumulateGrad nodes in
    it, which remember the side stream they were created on -- alive past the
    capture: the MoE layers' cached aux-loss tensors (``last_aux``,
    ``last_aux_weighted``: differentiable, they reach every parameter upstream
    of the router) and the custom Functions' ctx reference cycles.  A later
    pass on another stream (the re-capture's new side stream, bench.py's eager
    profile steps) would then re-use the stale nodes and synchronise across
    streams in every step (torch's "AccumulateGrad node's stream does not
    match" warning).  The cached tensors are detached (same storage: their
    values still follow graph replays) and the cycles collected."""
    import gc

    from ..moe.layer import MoEFFN

    if model is not None:
        for m in model.modules():
            if isinstance(m, MoEFFN):
                if m.last_aux is not None:
                    m.last_aux = tuple(t.detach() if torch.is_tensor(t) else t for t in m.last_aux)
                for name in ("last_aux_weighted", "ep_aux_weighted"):
                    t = getattr(m, name, None)
                    if torch.is_tensor(t):
                        setattr(m, name, t.detach())
    gc.collect()


def release_graphs():
    """Before ``dist.destroy_process_group()``: free every unreachable captured
    graph (their captured RCCL kernels keep the communicator busy: the destroy
    then hangs, gpurun_out/r6c) and drain the device."""
    import gc

    gc.collect()
    if torch.cuda.is_available() and torch.cuda.is_initialized():
        torch.cuda.synchronize()


class FlatOutputs(nn.Module):
    """Model wrapper whose forward returns a flat tuple of tensors (a graph
    output signature): final, auxiliary and encoder logits/boxes + MoE aux loss."""

    def __init__(self, model: RTDETRMoE):
        super().__init__()
        self.model = model

    def forward(self, images, ctx):
        out = self.model(images, ctx)
        sets = [out] + list(out["aux_outputs"]) + [out["enc_outputs"]]
        flat = []
        for s in sets:
            flat += [s["pred_logits"], s["pred_boxes"]]
        aux = self.model.moe_aux_loss()
        flat.append(aux if aux is not None else out["pred_boxes"].sum() * 0.0)
        return tuple(flat)

    @staticmethod
    def unflatten(flat):
        pairs = [{"pred_logits": flat[i], "pred_boxes": flat[i + 1]} for i in range(0, len(flat) - 1, 2)]
        out = dict(pairs[0])
        out["aux_outputs"] = pairs[1:-1]
        out["enc_outputs"] = pairs[-1]
        return out, flat[-1]


class _ReplayFn(torch.autograd.Function):
    """Forward = replay of the captured forward graph; backward = copy the
    incoming output gradients into the static buffers and replay the captured
    backward graph (parameter grads land in the runner's static buffers)."""

    @staticmethod
    def forward(ctx, runner, anchor):
        runner.g_fwd.replay()
        ctx.runner = runner
        return tuple(o.detach() for o in runner.static_out)

    @staticmethod
    def backward(ctx, *grads):
        r = ctx.runner
        for buf, g in zip(r.static_gout, grads):
            if g is None:
                buf.zero_()
            else:
                buf.copy_(g)
        r.g_bwd.replay()
        return None, None


class GraphedModel:
    """Capture ``fn(images, ctx) -> tuple of tensors`` forward and backward as
    two hipGraphs (see the module docstring).  After ``loss.backward()`` the
    parameter gradients are in ``static_grads`` (one per ``params`` entry)."""

    def __init__(self, fn, params, images, ctx, warmup=3, autocast=False):
        self.fn = fn
        self.params = params
        self.autocast = autocast
        self.static_images = images.clone()
        self.static_ctx = ctx.clone()
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up: convolution search, library attributes, allocator
            for _ in range(warmup):
                out = self._run()
                grads = torch.autograd.grad([o for o in out if o.requires_grad],
                                            params, [torch.ones_like(o) for o in out if o.requires_grad],
                                            allow_unused=True)
                check_grad_slots()
                del out, grads
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        quiesce_collectives()
        self.pool = torch.cuda.graph_pool_handle()
        self.g_fwd = torch.cuda.CUDAGraph()
        # captured on the warm-up stream: the autograd nodes the warm-up created
        # (AccumulateGrad keeps the stream it was made on) then match the capture
        # stream, so the backward needs no cross-stream syncs -- a single chain,
        # no fork/join branches for the HIP runtime to spread over parallel streams
        with torch.cuda.graph(self.g_fwd, pool=self.pool, stream=side, capture_error_mode=CAPTURE_MODE):
            out = self._run()
        self.static_out = out
        self.diff = [i for i, o in enumerate(out) if o.requires_grad]
        self.static_gout = [torch.zeros_like(o) for o in out]
        self.g_bwd = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.g_bwd, pool=self.pool, stream=side, capture_error_mode=CAPTURE_MODE):
            grads = torch.autograd.grad([out[i] for i in self.diff], params,
                                        [self.static_gout[i] for i in self.diff], allow_unused=True)
            check_grad_slots()
        self.static_grads = [g if g is not None else torch.zeros_like(p) for g, p in zip(grads, params)]
        self.anchor = torch.zeros((), device=images.device, requires_grad=True)
        del grads
        _drop_autograd_graphs(self.fn if isinstance(self.fn, nn.Module) else None)
        torch.cuda.synchronize()

    def _run(self):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.autocast, cache_enabled=False):
            return self.fn(self.static_images, self.static_ctx)

    def __call__(self, images, ctx):
        if images.data_ptr() != self.static_images.data_ptr():
            self.static_images.copy_(images)
        if ctx.data_ptr() != self.static_ctx.data_ptr():
            self.static_ctx.copy_(ctx)
        return _ReplayFn.apply(self, self.anchor)


class GraphedStep:
    """The whole differentiable step -- model forward, set criterion with the
    GPU Hungarian matcher (``SetCriterion.forward_padded``), backward to every
    parameter -- captured as ONE hipGraph.  Inputs (images, context ids,
    padded targets, box count) live in static buffers refreshed by device
    copies before each replay; gradients land in ``static_grads``.  No host
    round trip inside the step: the host only refreshes inputs, replays, and
    launches the optimizer.  Targets are padded to ``max_boxes`` per image;
    a batch with more boxes re-captures at the next multiple of 16; the new
    capture allocates new gradient buffers, announced through ``on_capture``
    (TrainStep re-points ``p.grad`` and drops its flat all-reduce views)."""

    def __init__(self, fn, criterion, params, images, ctx, targets, num_boxes, *, warmup=3, autocast=False,
                 max_boxes=None, on_capture=None):
        from .criterion import pad_targets

        self.fn, self.criterion, self.params, self.autocast = fn, criterion, params, autocast
        self.on_capture = on_capture  # called with static_grads after every (re-)capture
        self.captures = 0
        dev = images.device
        self.static_images = images.clone()
        self.static_ctx = ctx.clone()
        need = max((len(t["boxes"]) for t in targets), default=0)
        self.M = max_boxes or max(16, (need + 15) // 16 * 16)
        self.tb, self.tl, self.nv = pad_targets(targets, self.M)
        self.nb = torch.full((), float(num_boxes), dtype=torch.float32, device=dev)
        self.status = torch.zeros(1, dtype=torch.int32, device=dev)
        self.warmup = warmup
        self._capture()

    def _loss(self):
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=self.autocast, cache_enabled=False):
            flat = self.fn(self.static_images, self.static_ctx)
        out, aux = FlatOutputs.unflatten(flat)
        if _FUSED_CRIT and self.criterion.fused_ok(out, self.M):  # matching + losses in 3 HIP launches
            total, losses = self.criterion.loss_padded(out, self.tb, self.tl, self.nv, self.nb, self.status)
            return total + aux, losses
        losses = self.criterion.forward_padded(out, self.tb, self.tl, self.nv, self.nb, self.status)
        return sum(losses.values()) + aux, losses

    def _grads(self, loss):
        """Gradients of every parameter: autograd for most, the conforming dense
        layers' weight + bias gradients batched after it (linear.DeferredWgrad)."""
        from .conv import batched_flips, deferred_wgrads
        from contextlib import nullcontext

        # bf16 weights live at fixed addresses: the convolutions' flipped weights in one launch
        # (conv.batched_flips); autocast's per-step weight casts would not.  The convolutions'
        # weight-gradient slice sums batched at the end of the backward (conv.deferred_wgrads;
        # under autocast the weight casts' backward reads each gradient at once)
        flips = nullcontext() if self.autocast else batched_flips(loss.device)
        with deferred_weight_grads() as deferred, flips, deferred_wgrads(enabled=not self.autocast):
            grads = torch.autograd.grad(loss, self.params, allow_unused=True)
        check_grad_slots()
        self.deferred_layers = 0 if deferred is None else len(deferred.items)
        return merge_deferred(self.params, grads, deferred)

    def _capture(self):
        side = torch.cuda.Stream()
        side.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(side):  # warm-up: convolution search, library attributes, allocator
            for _ in range(self.warmup):
                loss, _ = self._loss()
                grads = self._grads(loss)
                del loss, grads
        torch.cuda.current_stream().wait_stream(side)
        torch.cuda.synchronize()
        quiesce_collectives()
        self.pool = torch.cuda.graph_pool_handle()
        self.graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(self.graph, pool=self.pool, stream=side,
                              capture_error_mode=CAPTURE_MODE):  # warm-up stream: see GraphedModel
            loss, losses = self._loss()
            grads = self._grads(loss)
            self.static_loss = loss.detach()
            self.static_losses = {k: v.detach() for k, v in losses.items()}
        self.static_grads = [g if g is not None else torch.zeros_like(p) for g, p in zip(grads, self.params)]
        del loss, losses, grads
        _drop_autograd_graphs(self.fn if isinstance(self.fn, nn.Module) else None)
        torch.cuda.synchronize()
        self.captures += 1
        if self.on_capture is not None:
            self.on_capture(self.static_grads)

    def __call__(self, images, ctx, targets, num_boxes):
        from .criterion import pad_targets

        need = max((len(t["boxes"]) for t in targets), default=0)
        if need > self.M:  # larger than the captured padding: re-capture (rare)
            self.M = (need + 15) // 16 * 16
            self.tb, self.tl, self.nv = pad_targets(targets, self.M)
            self.graph = None
            self._capture()
        if images.data_ptr() != self.static_images.data_ptr():
            self.static_images.copy_(images)
        if ctx.data_ptr() != self.static_ctx.data_ptr():
            self.static_ctx.copy_(ctx)
        pad_targets(targets, self.M, self.tb, self.tl, self.nv)
        if torch.is_tensor(num_boxes):  # device scalar (e.g. all-reduced box count): no host sync
            self.nb.copy_(num_boxes.reshape(()))
        else:
            self.nb.fill_(float(num_boxes))
        self.graph.replay()
        return self.static_loss


def _ep_group(model: nn.Module):
    """The process group the expert-parallel layers shard their experts over
    (None = the default group; every EP layer uses the same one)."""
    from ..moe.layer import MoEFFN

    groups = {id(m.ep_group): m.ep_group for m in model.modules() if isinstance(m, MoEFFN) and m.ep_size > 1}
    if len(groups) > 1:
        raise ValueError("expert-parallel layers over different process groups are not supported")
    return next(iter(groups.values()), None)


@torch.no_grad()
def clip_grad_norm_sharded(rep_params, shard_params, max_norm, shard_group=None):
    """torch.nn.utils.clip_grad_norm_ over a model whose ``shard_params`` are
    sharded across ``shard_group`` (expert parallelism): the global norm is
    sqrt(|g_rep|^2 + sum over ranks |g_shard|^2), identical on every rank, so
    the clip coefficient -- and hence the replicated weights -- stay in lockstep.
    Returns the total norm."""
    rep = [p.grad for p in rep_params if p.grad is not None]
    shard = [p.grad for p in shard_params if p.grad is not None]
    dev = (rep or shard)[0].device if (rep or shard) else torch.device("cpu")
    sq_rep = torch.stack([g.float().pow(2).sum() for g in rep]).sum() if rep else torch.zeros((), device=dev)
    sq_sh = torch.stack([g.float().pow(2).sum() for g in shard]).sum() if shard else torch.zeros((), device=dev)
    if shard_params and dist.is_available() and dist.is_initialized() and dist.get_world_size(shard_group) > 1:
        sq_sh = sq_sh.reshape(1)
        dist.all_reduce(sq_sh, group=shard_group)
        sq_sh = sq_sh.reshape(())
    total = (sq_rep + sq_sh).sqrt()
    coef = (max_norm / (total + 1e-6)).clamp(max=1.0)
    for g in rep + shard:
        g.mul_(coef.to(g.dtype))
    return total


def gemm_params(model: nn.Module):
    """Parameters that are GEMM / convolution operands: weights and biases of
    Linear, Conv2d and MultiheadAttention layers and the MoE expert weights,
    plus LayerNorm affines (the HIP layer_norm kernel wants them in the input
    dtype).  These are held in bf16 (TrainStep precision "bf16"); BatchNorm
    (mixed bf16-input / fp32-affine kernels), the MoE router and everything
    else stay fp32."""
    from ..moe.layer import MoEFFN

    out, seen = [], set()
    for mod in model.modules():
        if isinstance(mod, (nn.Linear, nn.Conv2d, nn.LayerNorm)):  # layer_norm on HIP needs weight dtype == input
            ps = [mod.weight, mod.bias]
        elif isinstance(mod, (nn.MultiheadAttention, TokenSelfAttention)):
            ps = [mod.in_proj_weight, mod.in_proj_bias]
        elif isinstance(mod, MoEFFN):
            ps = [mod.w1, mod.b1, mod.w2, mod.b2]
        else:
            continue
        for p in ps:
            if p is not None and id(p) not in seen:
                seen.add(id(p))
                out.append(p)
    return out


class TrainStep:
    """precision (GPU):
      "bf16" (default) -- GEMM/conv operands (gemm_params) held in bf16, fp32
             master copies in the optimizer, no autocast: no per-layer weight
             casts in the forward nor grad casts in the backward (about 1,700
             cast ops per C2 step under autocast, most of the host time of an
             eager step); the optimizer (optim.FlatAdamW: gradient clip +
             AdamW in three HIP launches) reads the bf16 grads, updates the
             flat fp32 masters and rewrites the bf16 weights;
      "amp"  -- fp32 parameters under bf16 autocast (same optimizer).
    On CPU the model runs in fp32 with torch.optim.AdamW and
    clip_grad_norm_ (the semantics FlatAdamW restates)."""

    def __init__(self, model: RTDETRMoE, criterion, images, ctx, *, lr=1e-4, lr_backbone=1e-5,
                 weight_decay=1e-4, clip_norm=0.1, graphs=True, ddp_local=None, world=1, precision="bf16",
                 targets=None, num_boxes=1.0, zero=None):
        """zero: the ZeRO-1 optimizer (optim.ShardedDPAdamW) -- default: at
        world > 1 unless MOE_ZERO=0; True also at world 1 (a world-1 process
        group: the RCCL reduce-scatter / all-gather branch on one GPU, tests)."""
        self.model = model
        self.criterion = criterion
        self.clip_norm = clip_norm
        self.phases = None  # list to enable per-phase event marks (phase_summary)
        self.world = world
        self.graphs = graphs
        self.precision = precision if images.is_cuda else "fp32"
        named = [(n, p) for n, p in model.named_parameters() if p.requires_grad]
        self.params = [p for _, p in named]
        if self.precision == "bf16":
            for p in gemm_params(model):
                p.data = p.data.to(torch.bfloat16)
        bb = [p for n, p in named if n.startswith("backbone.")]
        rest = [p for n, p in named if not n.startswith("backbone.")]
        self.ep_params = [p for p in self.params if getattr(p, "expert_parallel", False)]
        self.dp_params = [p for p in self.params if not getattr(p, "expert_parallel", False)]
        self.ep_group = _ep_group(model)
        if images.is_cuda:
            # flat fp32 masters + moments, clip + AdamW + bf16 weight refresh in
            # three HIP launches (optim.py); fp32 parameters become views of
            # their master segment -- before any graph capture bakes addresses.
            # Expert-parallel shards enter the clip norm through a sum over the
            # EP group (the same global norm on every rank)
            from .optim import FlatAdamW, ShardedDPAdamW

            use_zero = (world > 1 and _ZERO) if zero is None else bool(zero)
            if world > 1 and not use_zero:
                # (A/B flat path) every replica starts from rank 0's weights, as DDP
                # does, before FlatAdamW copies its masters
                from .optim import DPGradReducer

                self.reducer = DPGradReducer(self.dp_params)
                self.reducer.broadcast_params()
            if use_zero:
                # C3 data parallelism: reduce-scatter of the fp32 gradients,
                # AdamW on this rank's 1/world slice, all-gather of the weights
                # (optim.ShardedDPAdamW); the replicated parameters become views
                # of its flat spaces here, before any graph capture
                self.opt = ShardedDPAdamW([(bb, lr_backbone), (rest, lr)], weight_decay=weight_decay,
                                          clip_norm=clip_norm, sharded=self.ep_params)
            else:
                self.opt = FlatAdamW([(bb, lr_backbone), (rest, lr)], weight_decay=weight_decay,
                                     clip_norm=clip_norm, sharded=self.ep_params, shard_group=self.ep_group)
            self.opt_params = None
        else:
            self.opt_params = bb + rest
            self.opt = torch.optim.AdamW([{"params": bb, "lr": lr_backbone}, {"params": rest, "lr": lr}], lr=lr,
                                         weight_decay=weight_decay)
        self.flat = FlatOutputs(model)
        self.reducer = getattr(self, "reducer", None)
        if world > 1 and images.is_cuda:
            from ..moe.layer import MoEFFN

            # expert-parallel weights are not reduced (their gradients already
            # hold every rank's tokens), so their layers must not pre-scale by
            # 1/world: the optimizer applies 1/world to every gradient
            for m in model.modules():
                if isinstance(m, MoEFFN) and m.ep_size > 1:
                    m.ep_grad_scale = 1.0
        images = self._cast_in(images)
        self.runner = None
        self.stepper = None
        if graphs and targets is not None:  # whole step as one graph (GPU matcher)
            self.stepper = GraphedStep(self.flat, criterion, self.params, images, ctx, targets, num_boxes,
                                       autocast=self.precision == "amp", on_capture=self._bind_grads)
            self.fn = None
            self.ddp = None
        elif graphs:
            self.runner = GraphedModel(self.flat, self.params, images, ctx, autocast=self.precision == "amp")
            self.fn = self.runner
            self.ddp = None
            # the optimizer reads the static gradient buffers of the backward graph
            for p, g in zip(self.params, self.runner.static_grads):
                p.grad = g
        elif world > 1 and not images.is_cuda:  # CPU (gloo): DDP buckets overlapped with the backward
            from .engine import wrap_ddp

            self.ddp = wrap_ddp(self.flat, ddp_local)
            self.fn = self.ddp
        else:
            self.fn = self.flat
            self.ddp = None

    def _bind_grads(self, static_grads):
        """Point every parameter's .grad at the (new) static gradient buffers of
        a capture (the reducer rebuilds its table when the addresses change)."""
        for p, g in zip(self.params, static_grads):
            p.grad = g

    def _cast_in(self, images):
        return images.to(torch.bfloat16) if self.precision == "bf16" else images

    def use_eager(self):
        """Leave graph mode (bench.py's kernel-profiling steps): later steps run
        the model eagerly; parameter grads go back to autograd allocation."""
        if self.runner is not None or self.stepper is not None:
            self.runner = None
            self.stepper = None
            self.fn = self.flat
            self.graphs = False
            for p in self.params:
                p.grad = None
            _drop_autograd_graphs(self.model)  # the captures' AccumulateGrad nodes (side stream) go too

    def _allreduce_grads(self):
        """Data-parallel gradient sum (GPU, world > 1): the replicated
        parameters' gradients summed in fp32 by one all-reduce
        (optim.DPGradReducer).  Returns the gradient list in the optimizer's
        parameter order: the summed fp32 views for replicated parameters, the
        local gradients for expert-parallel ones; the optimizer divides by the
        world size inside its kernels."""
        red = {id(p): v for p, v in zip(self.dp_params, self.reducer([p.grad for p in self.dp_params]))}
        return [red.get(id(p), p.grad) for p in self.opt.params]

    def _mark(self, name):
        if self.phases is not None:
            e = torch.cuda.Event(enable_timing=True)
            e.record()
            self.phases.append((name, e, time.perf_counter()))

    def __call__(self, images, ctx, targets, num_boxes):
        self._mark("start")
        if self.stepper is not None:
            loss = self.stepper(self._cast_in(images), ctx, targets, num_boxes)
            self._mark("step_graph")
            self._optimizer_step()
            self._mark("optimizer")
            return loss
        if self.runner is None:
            for p in self.params:
                p.grad = None
        with torch.autocast(images.device.type, dtype=torch.bfloat16, enabled=self.precision == "amp"):
            flat = self.fn(self._cast_in(images), ctx)
        self._mark("forward")
        out, aux = FlatOutputs.unflatten(flat)
        losses = self.criterion(out, targets, num_boxes)
        loss = sum(losses.values()) + aux
        self._mark("criterion")
        if self.ddp is None and self.runner is None and images.is_cuda:
            # dense weight gradients batched after the backward (DDP's reducer
            # needs every gradient during the backward, so not under DDP)
            with deferred_weight_grads() as deferred:
                loss.backward()
            if deferred is not None:
                grads = merge_deferred(self.params, [p.grad for p in self.params], deferred)
                for p, g in zip(self.params, grads):
                    p.grad = g
        else:
            loss.backward()
        check_grad_slots()
        self._mark("backward")
        self._optimizer_step()
        self._mark("optimizer")
        return loss.detach()

    def _optimizer_step(self):
        if self.opt_params is None:  # GPU: FlatAdamW / ShardedDPAdamW (reduction + clip inside)
            if self.reducer is not None:
                self.opt.step(self._allreduce_grads(), inv_world=1.0 / self.world)
            else:
                self.opt.step()
        else:
            if self.clip_norm > 0:
                clip_grad_norm_sharded(self.dp_params, self.ep_params, self.clip_norm, self.ep_group)
            self.opt.step()

    def phase_summary(self):
        """{phase: (gpu ms, host ms)} averaged over the marked steps (syncs)."""
        torch.cuda.synchronize()
        acc, n = {}, 0
        ph = self.phases or []
        for i in range(1, len(ph)):
            name, e, t = ph[i]
            if name == "start":
                n += 1
                continue
            pe, pt = ph[i - 1][1], ph[i - 1][2]
            g, h = acc.get(name, (0.0, 0.0))
            acc[name] = (g + pe.elapsed_time(e), h + 1e3 * (t - pt))
        n = max(n + 1, 1)
        return {k: (round(g / n, 3), round(h / n, 3)) for k, (g, h) in acc.items()}
