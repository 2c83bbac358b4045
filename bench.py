#!/usr/bin/env python
"""Benchmark: images/sec (fwd+bwd) of RT-DETR-MoE at 1280x720, bs=8/GPU, MI355X.

Metric and configs come from BASELINE.json.  One "step" = one full training
step of the C2 workload on one batch: RT-DETR-R50 + 8-expert top-2 MoE FFN in
the AIFI encoder layer and all 6 decoder layers, bf16 weights with fp32
master copies (``--precision amp``: fp32 weights under bf16 autocast),
forward, Hungarian-matched VFL/L1/GIoU losses + MoE aux losses, backward,
grad clip, AdamW step; by default forward + criterion + backward replay as
ONE hipGraph.  Synthetic ZOD-shaped batches generated once
and kept resident in HBM; random-init weights.

  python bench.py                               # N=1, defaults
  python bench.py --gpus N                      # starts N ranks itself (launch_ranks)
  python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 \
      --master-port P bench.py --gpus N         # DP over RCCL (C3), weak scaling

Rank 0 prints ONE JSON line.  Besides the contract keys it carries
``roofline`` for the dominant HIP kernel (the grouped expert GEMM: kernel
times from dispatch-stamped HIP events recorded by libmoe_hip itself -- in
graph mode over eager steps right after the timed region, since ROCm 7.2
stamps no events inside a hipGraph -- next to the rocprofv3-derived average
of the committed kernel summary; algorithmic bytes and flops per launch;
bound = HBM, since at d=256, F=1024 every expert GEMM has ~200 flop/B, below
the MI355X balance of ~312), ``roofline_dispatch`` for the row movers, and
``cpu_baseline``: the same model and step in fp32 on the host cores at the
workload's batch (MoE layers through the package's CPU device path,
src/moe/eager.py, in fp32 torch ops; kind "port"), timed on a bounded sample
(rank 0, N=1 only), and ``roofline_e2e``: images/s x measured model FLOP per
image (FlopCounterMode over one fp32 CPU fwd+bwd at the workload's resolution)
/ the bf16 MFMA peak.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import subprocess
import sys
import time
from datetime import timedelta
from pathlib import Path

ROOT = Path(__file__).resolve().parent


def _free_port():
    import socket

    with socket.socket(socket.AF_INET, socket.SOCK_STREAM) as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def launch_ranks(n, argv, script=None, poll_s=0.5):
    """Start ``n`` worker ranks of ``script`` (default: this file) as fresh
    child processes, one per GPU, and wait for them (the multi-GPU analogue of
    the reference's ``device="0,1,..."`` string, rtdetr.py:89).  The parent
    never touches the GPU: it runs before ``import torch`` and execs nothing,
    so each child initialises HIP itself.  Each child gets RANK / LOCAL_RANK /
    WORLD_SIZE / LOCAL_WORLD_SIZE and a 127.0.0.1 rendezvous.  Returns the
    first non-zero child exit code (the other ranks are then terminated by
    PID, so a dead rank ends the job instead of hanging it), else 0."""
    port = os.environ.get("MASTER_PORT") or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", MASTER_PORT=port)
        procs.append(subprocess.Popen([sys.executable, str(script or Path(__file__).resolve())] + list(argv),
                                      env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            c = p.poll()
            if c is None:
                continue
            live.remove(p)
            if c != 0 and rc == 0:
                rc = c if c > 0 else 128 - c
                print(f"[bench] rank {procs.index(p)} exited with {c}; stopping the other ranks", file=sys.stderr,
                      flush=True)
                for q in live:
                    q.terminate()
        if live:
            time.sleep(poll_s)
    for p in procs:
        p.wait()
    return rc


def _requested_gpus(argv):
    ap = argparse.ArgumentParser(add_help=False)
    ap.add_argument("--gpus", type=int, default=1)
    return ap.parse_known_args(argv)[0].gpus


if __name__ == "__main__" and "WORLD_SIZE" not in os.environ and _requested_gpus(sys.argv[1:]) > 1:
    # `python bench.py --gpus N` without a launcher: start the N ranks here,
    # before anything imports torch or touches a GPU
    sys.exit(launch_ranks(_requested_gpus(sys.argv[1:]), sys.argv[1:]))

for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT)):
    if p not in sys.path:
        sys.path.insert(0, p)
os.environ.setdefault("HSA_ENABLE_IPC_MODE_LEGACY", "0")
# MIOpen convolution search (torch.backends.cudnn.benchmark, --conv-search) in
# its fast mode: find-db lookups + quick heuristics, seconds instead of minutes
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
# ...starting from the find/perf databases measured on MI355X and shipped with
# the package (multimodal-moe_amd/miopen_db/README.md): same algorithm choices
# on every fresh box
os.environ.setdefault("MIOPEN_USER_DB_PATH", str(ROOT / "multimodal-moe_amd" / "miopen_db"))

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

METRIC = "images/sec (fwd+bwd) RT-DETR-MoE 1280×720 bs=8/GPU at 1/2/4/8 MI355X"
PEAK_BF16_TFLOPS = 2500.0   # MI355X dense bf16 MFMA (MI355X_MICROARCH.md, chip-level parameters)
PEAK_FP8_TFLOPS = 5000.0    # MI355X dense fp8 MFMA (the MXFP8 expert GEMMs of C5)
PEAK_HBM_GBS = 8000.0       # MI355X HBM3E spec peak

WORKLOADS = {
    "c2": dict(spec="rtdetr-r50-moe8-top2", batch=8, desc="C2: RT-DETR-R50 + 8-expert top-2 MoE, bs=8/GPU, bf16",
               dtype="bf16"),
    "c4": dict(spec="rtdetr-r50-moe16-top2-ep{N}", batch=8, single_ctx=True,
               desc="C4: 16-expert top-2, expert-parallel all-to-all, solar-context-binned batches"),
    "c5": dict(spec="rtdetr-r50-moe32-top4-cf1.25-fp8", batch=16, dtype="bf16 + MXFP8 (e4m3) expert GEMMs",
               desc="C5: 32-expert top-4 fp8 experts, capacity factor 1.25, bs=16/GPU"),
}


def load_pmc_traffic(workload):
    """HBM bytes per launch per kernel group from the committed PMC summary of
    the same workload (tools/gpu_round.sh + tools/profile_summary.py:
    rocprofv3 --pmc FETCH_SIZE / WRITE_SIZE passes, gfx950-corrected)."""
    # the newest round's summary (profiles/rNN/pmc_traffic_<wl>.json), else the top-level one
    cands = sorted((ROOT / "profiles").glob(f"r[0-9][0-9]/pmc_traffic_{workload}.json"))
    p = cands[-1] if cands else ROOT / "profiles" / f"pmc_traffic_{workload}.json"
    if not p.exists():
        return {}
    try:
        data = json.loads(p.read_text())
    except ValueError:
        return {}
    out = {}
    for g, e in data.get("groups", {}).items():
        if "hbm_bytes_per_launch" in e:
            out[g] = {"bytes": e["hbm_bytes_per_launch"], "source": f"{p.relative_to(ROOT)} ({data.get('source')})"}
            if "mfma_counter_frac" in e:  # rocprofv3 SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE/8 x 1024 SIMDs)
                out[g]["mfma_counter_frac"] = e["mfma_counter_frac"]
    return out


def lib_build_id():
    """sha256 (first 16 hex digits) of the libmoe_hip.so this process loaded:
    ties a committed rocprof summary to the build it was taken of."""
    import hashlib

    from src.moe import _lib as L

    return hashlib.sha256(Path(L.LIB_PATH).read_bytes()).hexdigest()[:16]


def load_rocprof_summary(workload):
    """(groups, source, meta) of the newest committed rocprofv3 kernel-trace
    summary of the same workload (profiles/rNN/<wl>/kernel_summary.json,
    tools/profile_summary.py over `rocprofv3 --kernel-trace --stats` of this
    bench command, graph replay included); meta holds the build id and the
    bench configuration of the profiled run (tools/profile_summary.py copies
    them from that run's own bench line)."""
    cands = sorted((ROOT / "profiles").glob(f"r[0-9][0-9]/{workload}/kernel_summary.json"))
    if not cands:
        return {}, None, {}
    try:
        data = json.loads(cands[-1].read_text())
    except ValueError:
        return {}, None, {}
    return data.get("groups", {}), f"{cands[-1].relative_to(ROOT)} ({data.get('source')})", data.get("bench", {})


def merge_groups(*ds):
    """Sum the profiler totals of several kinds (e.g. the bf16 and fp8 launches
    of the grouped GEMM) into one group."""
    ds = [d for d in ds if d]
    if not ds:
        return None
    out = {k: sum(d[k] for d in ds) for k in ("launches", "total_ms", "flops", "bytes", "t_mfma_ms", "t_hbm_ms",
                                               "t_roof_ms")}
    out["avg_us"] = 1e3 * out["total_ms"] / max(out["launches"], 1)
    return out


def roofline_entry(d, pmc, elapsed, kernel):
    """Roofline of one kernel group over the timed region.  Every launch is
    bounded by max(flops / MFMA peak of its dtype, algorithmic bytes / HBM
    peak); the group's bound is the resource with the larger summed time.
    achieved = algorithmic work / measured kernel time (dispatch-stamped HIP
    events).  The MFMA fraction is sum(flops_i / peak_i) / time, i.e. bf16
    launches priced at the bf16 peak and MXFP8 launches at the fp8 peak; the
    reported MFMA ``peak`` is the effective (flop-weighted) one."""
    if not d or d["total_ms"] <= 0:
        return None
    sec = d["total_ms"] * 1e-3
    hbm = d["t_hbm_ms"] >= d["t_mfma_ms"]
    ach_gbs = d["bytes"] / sec / 1e9
    ach_tf = d["flops"] / sec / 1e12
    peak_tf = d["flops"] / (d["t_mfma_ms"] * 1e-3) / 1e12 if d["t_mfma_ms"] > 0 else PEAK_BF16_TFLOPS
    mfma_frac = d["t_mfma_ms"] / d["total_ms"]
    e = {"bound": "hbm" if hbm else "mfma",
         "achieved": round(ach_gbs if hbm else ach_tf, 2),
         "peak": PEAK_HBM_GBS if hbm else round(peak_tf, 1),
         "unit": "GB/s" if hbm else "TFLOP/s",
         "frac": round((ach_gbs / PEAK_HBM_GBS) if hbm else mfma_frac, 4),
         "traffic": pmc["bytes"] if pmc else None,
         "kernel": kernel, "launches": d["launches"], "avg_us": round(d["avg_us"], 2),
         "algorithmic_bytes_per_launch": round(d["bytes"] / d["launches"]),
         "roofline_time_frac": round(d["t_roof_ms"] / d["total_ms"], 4),
         "share_of_step": round(d["total_ms"] / (elapsed * 1e3), 4)}
    if d["flops"]:
        e["flop_per_launch"] = round(d["flops"] / d["launches"])
        e["mfma"] = {"achieved": round(ach_tf, 2), "peak": round(peak_tf, 1), "unit": "TFLOP/s",
                     "frac": round(mfma_frac, 4)}
        if pmc and "mfma_counter_frac" in pmc:
            # matrix-core busy fraction from PMC counters over the same kernels
            # (SQ_VALU_MFMA_BUSY_CYCLES / SIMD-cycles of the kernels' lifetime)
            e["mfma"]["counter_frac"] = pmc["mfma_counter_frac"]
            e["mfma"]["counter_source"] = pmc["source"]
    if pmc:
        e["traffic_source"] = pmc["source"]
        e["traffic_over_algorithmic"] = round(pmc["bytes"] / (d["bytes"] / d["launches"]), 3)
    return e


def rocprof_headline(e, g, src, match):
    """Put the graph-replay timing of a kernel group on the headline.

    ``e`` is the live roofline entry (dispatch-stamped HIP events of eager
    steps right after the timed region: hipGraphs carry no events on ROCm
    7.2); ``g`` the group in the committed rocprofv3 summary of this bench
    command, whose average launch duration covers the replayed step graph.
    When that summary belongs to this build (``match``), achieved / frac /
    avg_us become the rocprof figures -- algorithmic bytes per launch (this
    run's library profiler) / rocprof's average duration / peak -- and the
    live event figures move to ``eager_events``; otherwise the headline stays
    live and the summary is reported as ``rocprof`` with ``matches_build``
    false."""
    if not e or not g or not g.get("avg_us"):
        return e
    bpl = e["algorithmic_bytes_per_launch"]
    sec = g["avg_us"] * 1e-6
    ach = bpl / sec / 1e9
    rp = {"avg_us": g["avg_us"], "launches": g.get("launches"), "achieved": round(ach, 2), "unit": "GB/s",
          "frac": round(ach / PEAK_HBM_GBS, 4), "source": src, "matches_build": bool(match)}
    if e.get("flop_per_launch"):
        rp["mfma_tflops"] = round(e["flop_per_launch"] / sec / 1e12, 1)
    if not match or e["bound"] != "hbm":
        e["rocprof"] = rp
        e["timing_source"] = "libmoe_hip dispatch-stamped HIP events (eager steps after the timed region)"
        return e
    live = {k: e[k] for k in ("avg_us", "launches", "achieved", "frac")}
    if "mfma" in e:
        live["mfma_tflops"] = e["mfma"]["achieved"]
    live["source"] = "libmoe_hip dispatch-stamped HIP events over the eager steps after the timed region"
    e.update({"avg_us": g["avg_us"], "launches": g.get("launches"), "achieved": rp["achieved"], "frac": rp["frac"],
              "eager_events": live,
              "timing_source": f"rocprofv3 --kernel-trace of this build's bench command (graph replay): {src}"})
    if "mfma" in e and e.get("flop_per_launch"):
        e["mfma"]["achieved"] = rp["mfma_tflops"]
        e["mfma"]["frac"] = round(e["flop_per_launch"] / sec / 1e12 / e["mfma"]["peak"], 4)
    return e


def parse_args():
    ap = argparse.ArgumentParser(description=__doc__.split("\n")[0])
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=10)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--workload", choices=sorted(WORKLOADS), default="c2")
    ap.add_argument("--batch", type=int, default=None, help="images per GPU (default: the workload's)")
    ap.add_argument("--spec-extra", default="", help="model-spec tokens appended to the workload's spec (A/B, "
                                                      "e.g. -epmb0 or -epcf0 for C4)")
    ap.add_argument("--img-h", type=int, default=720)
    ap.add_argument("--img-w", type=int, default=1280)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-seconds", type=float, default=125.0,
                    help="target length of the CPU baseline's timed sample (at least 5 steps when a step takes "
                         "<= 20 s, BASELINE.md 2)")
    ap.add_argument("--no-e2e-roofline", action="store_true", help="skip the model-FLOP count (roofline_e2e)")
    ap.add_argument("--no-kernel-timing", action="store_true", help="skip per-launch HIP events")
    ap.add_argument("--dump-prof-records", default=None, metavar="PATH",
                    help="with --no-graphs: write the timed steps' per-launch library records (kind, ms, flops, "
                         "algorithmic bytes, in launch order) as JSON (tools/gemm_traffic.py joins them with PMC)")
    ap.add_argument("--precision", choices=["bf16", "amp"], default="bf16",
                    help="bf16: bf16 GEMM/conv weights + fp32 master weights; amp: fp32 weights under bf16 autocast")
    ap.add_argument("--phase-timing", action="store_true",
                    help="report per-phase GPU/host ms (forward, criterion, backward, optimizer)")
    ap.add_argument("--conv-search", action=argparse.BooleanOptionalAction, default=True,
                    help="let MIOpen benchmark convolution algorithms (torch.backends.cudnn.benchmark)")
    ap.add_argument("--deterministic", action=argparse.BooleanOptionalAction, default=False,
                    help="MIOpen deterministic convolution solvers only (torch.backends.cudnn.deterministic)")
    ap.add_argument("--graphs", action=argparse.BooleanOptionalAction, default=True,
                    help="capture the model forward/backward as hipGraphs (default; not with expert parallelism). "
                         "ROCm 7.2 does not stamp timing events inside a graph (tools/graph_event_probe.py), so "
                         "with graphs the per-kernel roofline comes from --profile-steps eager steps run right "
                         "after the timed region")
    ap.add_argument("--tune", action="append", default=[], metavar="KEY=VALUE",
                    help="libmoe_hip tuning override (moe_set_tuning), repeatable; for A/B runs")
    ap.add_argument("--step-graph", action=argparse.BooleanOptionalAction, default=True,
                    help="graph mode: capture forward + criterion (GPU Hungarian matcher) + backward as ONE "
                         "hipGraph (default); --no-step-graph: forward and backward graphs around a host-matched "
                         "criterion")
    ap.add_argument("--profile-steps", type=int, default=3,
                    help="graph mode: eager steps after the timed region that carry the kernel events")
    ap.add_argument("--eval-steps", type=int, default=10,
                    help="eval leg after the training measurement: timed inference forwards of the same batch "
                         "(engine._evaluate's forward: model.eval(), no_grad, bf16 autocast); 0 skips it")
    return ap.parse_args()


def setup_dist(n_gpus):
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        torch.cuda.set_device(local)
        from src.rtdetr_moe.step import rccl_env

        rccl_env()
        # a rank that never arrives fails the job instead of hanging it
        dist.init_process_group("nccl", device_id=torch.device("cuda", local),
                                timeout=timedelta(seconds=float(os.environ.get("MOE_DIST_TIMEOUT_S", "600"))))
    else:
        torch.cuda.set_device(0)
    if n_gpus != world:
        print(f"[bench] warning: --gpus {n_gpus} but WORLD_SIZE={world}; using {world}", file=sys.stderr)
    if world > 1:
        world = dist.get_world_size()  # the process group's (RCCL's) own count, not the env's
    return world, rank, local


def heartbeat(period=30.0):
    """A daemon thread that prints to stderr every `period` s, so a long MIOpen
    convolution search in the first steps is not mistaken for a hang."""
    import threading

    t0 = time.perf_counter()

    def run():
        while True:
            time.sleep(period)
            print(f"[bench] alive {time.perf_counter() - t0:.0f} s", file=sys.stderr, flush=True)

    threading.Thread(target=run, daemon=True).start()


def log(rank, msg):
    """Progress to stderr (rank 0): long warm-ups stay visibly alive."""
    if rank == 0:
        print(f"[bench] {msg}", file=sys.stderr, flush=True)


def build_model(spec, device, world):
    from src.rtdetr_moe.model import RTDETRMoE

    torch.manual_seed(1)
    model = RTDETRMoE(spec).to(device).to(memory_format=torch.channels_last)
    if world > 1:  # identical initial weights on every rank (DDP would broadcast them)
        for t in list(model.parameters()) + list(model.buffers()):
            dist.broadcast(t.data, 0)
    return model


def expert_parallel_stats(model, spec, world):
    """C4 exchange accounting of the last step (rank-local): the slot rows S
    per (source, expert), the bytes of one all-to-all per MoE layer (E S d bf16
    rows: the fixed-capacity buffer; (W-1)/W of it leaves the rank), and the
    assignments the fixed-capacity exchange dropped (ep_overflow), against
    SURVEY 8(e)'s lossless-exchange budget A (W-1)/W 512 B per direction."""
    layers = [m for m in model.moe_layers() if getattr(m, "last_tokens", 0)]
    if not layers:
        return None
    cfg = layers[0].cfg
    per_layer, over, assign, a2a = [], 0, 0, 0.0
    for m in layers:
        T = m.last_tokens
        S = cfg.ep_slot_rows(T, m.d_model)
        b = cfg.num_experts * S * m.d_model * 2
        ov = int(m.last_ep_overflow) if m.last_ep_overflow is not None else 0
        over += ov
        assign += T * cfg.top_k
        a2a += 4 * b  # forward dispatch + combine, backward both transposes
        per_layer.append({"T": T, "slots": S, "lossless": S >= T,
                          "slot_factor": round(S * cfg.num_experts / (T * cfg.top_k), 3), "bytes_per_a2a": b,
                          "survey_bytes_per_a2a": round(T * cfg.top_k * 512 * (max(world, 8) - 1) / max(world, 8)),
                          "overflow": ov, "overflow_frac": round(ov / max(T * cfg.top_k, 1), 5)})
    return {"slot_factor": cfg.ep_capacity_factor if cfg.ep_capacity_factor > 0 else "lossless",
            "lossless_budget_mb": cfg.ep_lossless_mb,
            "max_layer_overflow_frac": max(p["overflow_frac"] for p in per_layer),
            "ep_overflow": over, "assignments": assign, "overflow_frac": round(over / max(assign, 1), 5),
            "a2a_bytes_per_step_per_rank": round(a2a), "layers": per_layer,
            "note": "survey_bytes_per_a2a: SURVEY 8(e)'s off-rank bytes of a lossless exchange at W=8; "
                    "bytes_per_a2a: this build's fixed-capacity buffer (its (W-1)/W leaves the rank)"}


def dp_exchange_bytes(model, world):
    """C3's gradient / weight exchange per rank per step for this
    model's replicated parameters (expert-parallel shards excluded), as ZeRO-1
    (optim.ShardedDPAdamW: fp32 reduce-scatter + bf16 / fp32 all-gather) and
    as the flat fp32 all-reduce (MOE_ZERO=0), ring algorithm, at this run's
    world size and at W = 8 (the driver's scaling run)."""
    nb = sum(p.numel() for p in model.parameters()
             if p.requires_grad and not getattr(p, "expert_parallel", False) and p.dtype == torch.bfloat16)
    nf = sum(p.numel() for p in model.parameters()
             if p.requires_grad and not getattr(p, "expert_parallel", False) and p.dtype != torch.bfloat16)

    def at(w):
        f = (w - 1) / w
        return {"zero1_reduce_scatter": round(f * 4 * (nb + nf)), "zero1_all_gather": round(f * (2 * nb + 4 * nf)),
                "zero1_total": round(f * (4 * (nb + nf) + 2 * nb + 4 * nf)),
                "flat_all_reduce": round(2 * f * 4 * (nb + nf))}

    return {"replicated_bf16_params": nb, "replicated_fp32_params": nf, "world": world, "bytes_per_rank": at(world),
            "bytes_per_rank_at_w8": at(8),
            "note": "ring collectives: each rank sends (W-1)/W of the buffer per reduce-scatter / all-gather, "
                    "2 (W-1)/W per all-reduce; issued after the step graph's replay (not overlapped)"}


def host_threads():
    """(threads used, CPUs in this process's affinity set): the affinity set,
    capped by OMP_NUM_THREADS when the box sets it (the GPU box exports the
    process's CPU share there; its affinity set is the whole machine)."""
    aff = len(os.sched_getaffinity(0))
    omp = os.environ.get("OMP_NUM_THREADS", "")
    n = min(aff, int(omp)) if omp.isdigit() and int(omp) > 0 else aff
    return max(1, n), aff


def _cpu_step_fn(spec, batch_img, img_h, img_w):
    """The workload's training step on the host, fp32: same model (MoE layers
    through src/moe/eager.py), same Hungarian-matched criterion, backward,
    clip_grad_norm_ + torch.optim.AdamW (what TrainStep runs on CPU)."""
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.data import SyntheticZOD
    from src.rtdetr_moe.model import RTDETRMoE

    torch.manual_seed(1)
    model = RTDETRMoE(spec)
    opt = torch.optim.AdamW(model.parameters(), lr=1e-4, weight_decay=1e-4)
    crit = SetCriterion(num_classes=1)
    data = SyntheticZOD(batch=batch_img, img_h=img_h, img_w=img_w, seed=0)
    images, targets, ctx = data.sample()
    nb = max(1.0, float(sum(len(t["boxes"]) for t in targets)))

    def step():
        opt.zero_grad(set_to_none=True)
        out = model(images, ctx)
        loss = sum(crit(out, targets, nb).values()) + model.moe_aux_loss()
        loss.backward()
        torch.nn.utils.clip_grad_norm_(model.parameters(), 0.1)
        opt.step()

    return step, len(model.moe_layers())


def model_flop_per_image(spec, img_h, img_w):
    """Measured FLOP of one fwd+bwd per image: torch.utils.flop_counter over
    one fp32 CPU training step of the same model at batch 1 (GEMMs, convolutions
    and attention; the deformable-attention sampling and element-wise work are
    not counted -- they are not MFMA work)."""
    from torch.utils.flop_counter import FlopCounterMode

    step, _ = _cpu_step_fn(spec, 1, img_h, img_w)
    with FlopCounterMode(display=False) as fc:
        step()
    return float(fc.get_total_flops())


def cpu_baseline(spec, batch_img, img_h, img_w, target_s):
    """The same training step in fp32 on the host cores at the workload's batch."""
    threads, aff = host_threads()
    torch.set_num_threads(threads)
    step, n_moe = _cpu_step_fn(spec, batch_img, img_h, img_w)
    t0 = time.perf_counter()
    step()  # warm-up: allocator and thread-pool start-up (no search or JIT on the CPU path)
    warm = time.perf_counter() - t0
    # BASELINE.md 2 plans 2 warm-up + 5 timed steps: one warm-up suffices here
    # (the per-step times below show no drift after it), and n = 5 timed steps
    # whenever a step takes <= target_s / 5
    n = max(1, min(5, int(target_s / max(warm, 1e-3))))
    times = []
    for _ in range(n):
        t1 = time.perf_counter()
        step()
        times.append(time.perf_counter() - t1)
    dt = sum(times)
    return {"value": round(batch_img * n / dt, 4), "unit": "images/sec", "cores": threads, "kind": "port",
            "affinity_cpus": aff, "step_s": [round(t, 2) for t in times], "warmup_s": round(warm, 2),
            "sample": f"{n} timed fwd+bwd+AdamW steps (+1 warm-up, {warm:.1f} s) of {spec} at batch {batch_img}, "
                      f"{img_w}x{img_h} padded to 32, fp32 torch on {threads} host threads "
                      f"(torch.set_num_threads; {aff} CPUs in the affinity set), {n_moe} MoE layers through "
                      f"src/moe/eager.py (fp32 torch ops{', MXFP8 expert GEMMs emulated' if 'fp8' in spec else ''})"}


def eval_leg(model, images, ctx, steps, warmup=3):
    """Inference speed of the trained model on the workload's batch: the
    forward engine._evaluate times for ``speed_inference_ms_per_img`` (reference
    scripts/eval_detector.py:99-116 derives fps_inference_only from it):
    engine.EvalForward -- model.eval(), no_grad, bf16 autocast, replayed as a
    hipGraph per input shape -- with the batch resident in HBM, timed between
    synchronizes; the same forward run eagerly is reported beside it.  Returns
    the eval block of the bench line."""
    from src.rtdetr_moe.engine import EvalForward

    def timed(fwd):
        for _ in range(warmup):
            fwd(images, ctx)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            fwd(images, ctx)
        torch.cuda.synchronize()
        return time.perf_counter() - t0

    was_training = model.training
    model.eval()
    try:
        graphed = EvalForward(model)
        graphed.prepare(images, ctx)
        dt = timed(graphed)
        eager = EvalForward(model)
        eager.enabled = False
        dt_eager = timed(eager)
        del graphed
    finally:
        model.train(was_training)
    n = steps * images.shape[0]
    return {"speed_inference_ms_per_img": round(1e3 * dt / n, 4), "fps_inference_only": round(n / dt, 2),
            "images_per_sec": round(n / dt, 2), "batch": int(images.shape[0]), "steps": steps, "warmup": warmup,
            "eager_images_per_sec": round(n / dt_eager, 2),
            "mode": "engine.EvalForward (engine._evaluate's forward): model.eval(), torch.no_grad, bf16 autocast, "
                    "hipGraph replay per input shape; batch resident in HBM, postprocess excluded"}


def main():
    args = parse_args()
    world, rank, local = setup_dist(args.gpus)
    if rank == 0:
        heartbeat()
    device = torch.device("cuda", local)
    wl = WORKLOADS[args.workload]
    spec = wl["spec"].format(N=world) + args.spec_extra
    torch.backends.cudnn.benchmark = bool(args.conv_search)
    torch.backends.cudnn.deterministic = bool(args.deterministic)
    batch = args.batch or wl["batch"]

    from src.moe import _lib as L
    from src.rtdetr_moe.data import SyntheticZOD

    L.lib()  # fail loudly if the HIP extension is missing
    build_id = lib_build_id()
    for kv in args.tune:
        key, val = kv.split("=", 1)
        L.set_tuning(key, int(val))
    from src.rtdetr_moe.criterion import SetCriterion
    from src.rtdetr_moe.step import TrainStep

    model = build_model(spec, device, world)
    data = SyntheticZOD(batch=batch, img_h=args.img_h, img_w=args.img_w, seed=1000 + rank,
                        single_context=(rank % 5) if wl.get("single_ctx") else None)
    images, targets, ctx = data.sample()
    images = images.to(device).contiguous(memory_format=torch.channels_last)
    ctx = ctx.to(device)
    targets = [{k: v.to(device) for k, v in t.items()} for t in targets]
    nb = torch.tensor([float(sum(len(t["boxes"]) for t in targets))], device=device)
    if world > 1:
        dist.all_reduce(nb)
    num_boxes = max(1.0, float(nb.item()) / world)

    graphs = args.graphs  # the EP layer's all-to-alls are fixed-capacity: capturable too
    # library-side kernel events around each MoE/MSDA launch: inside the timed
    # region when eager; in eager steps right after it when graphed
    timing = not args.no_kernel_timing
    ddp_local = local if (world > 1 and not graphs) else None
    step = TrainStep(model, SetCriterion(num_classes=1), images, ctx, graphs=graphs, world=world,
                     precision=args.precision, ddp_local=ddp_local,
                     targets=targets if args.step_graph else None, num_boxes=num_boxes)

    t_w = time.perf_counter()
    for i in range(args.warmup):  # the first steps run MIOpen's convolution search (can take minutes)
        step(images, ctx, targets, num_boxes)
        torch.cuda.synchronize()
        log(rank, f"warm-up step {i + 1}/{args.warmup} done ({time.perf_counter() - t_w:.1f} s)")
    if timing and not graphs:
        L.TIMER.start()
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(images, ctx, targets, num_boxes)
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    elapsed = time.perf_counter() - t0
    log(rank, f"timed {args.steps} steps: {1e3 * elapsed / args.steps:.2f} ms/step")
    phases = None
    if args.phase_timing:  # extra steps after the timed region, same execution mode
        step.phases = []
        for _ in range(3):
            step(images, ctx, targets, num_boxes)
        phases = step.phase_summary()
        step.phases = None
    prof_steps = args.steps
    if timing and not graphs:
        if args.dump_prof_records and rank == 0:
            recs = [(L.PROF_KINDS.get(k, str(k)), ms, fl, by) for k, ms, fl, by in L.profile_records(clear=False)]
            Path(args.dump_prof_records).write_text(json.dumps({"steps": args.steps, "records": recs}))
        L.TIMER.harvest()  # the K steps' launch records, read after the timed region
        L.TIMER.stop()
    elif timing:
        step.use_eager()
        step(images, ctx, targets, num_boxes)  # untimed: first eager step allocates
        torch.cuda.synchronize()
        L.TIMER.start()
        for _ in range(args.profile_steps):
            step(images, ctx, targets, num_boxes)
        L.TIMER.harvest()
        L.TIMER.stop()
        prof_steps = args.profile_steps
    # the exchange accounting of the last TRAINING step (the eval leg's
    # forwards below run eval-mode BatchNorm: different activations, routing)
    ep_stats = expert_parallel_stats(model, spec, world) if "-ep" in spec else None
    ev = None
    if args.eval_steps > 0:
        log(rank, f"eval leg: {args.eval_steps} inference forwards")
        ev = eval_leg(model, images, ctx, args.eval_steps)
    el = torch.tensor([elapsed], device=device, dtype=torch.float64)
    rccl_world = None
    if world > 1:
        dist.all_reduce(el, op=dist.ReduceOp.MAX)
        one = torch.ones(1, device=device)
        dist.all_reduce(one)  # the ranks that answer an RCCL all-reduce
        rccl_world = {"backend": dist.get_backend(), "world_size": dist.get_world_size(),
                      "all_reduce_ranks": int(one.item())}
        try:
            rccl_world["rccl_version"] = ".".join(map(str, torch.cuda.nccl.version()))
        except Exception:  # noqa: BLE001 (optional detail)
            pass
    elapsed = float(el.item())
    ksum = L.TIMER.summary() if timing else {}

    result = None
    if rank == 0:
        images_total = world * batch * args.steps
        value = images_total / elapsed
        pmc = load_pmc_traffic(args.workload)
        prof_elapsed = elapsed * prof_steps / args.steps  # share_of_step: per-step kernel time / step time
        roof = roofline_entry(merge_groups(ksum.get("grouped_gemm"), ksum.get("grouped_gemm_fp8")),
                              pmc.get("grouped_gemm"), prof_elapsed,
                              "grouped GEMM (gemm_v2_kernel: expert fwd, dgrad, wgrad)")
        rp, rp_src, rp_meta = load_rocprof_summary(args.workload)
        # the committed rocprof summary is THIS build's when its profiled bench
        # line carries the same library hash and configuration (else it is
        # reported, labelled stale, and the headline stays on the live events)
        rp_match = (rp_meta.get("libmoe_hip_sha16") == build_id and rp_meta.get("workload") == wl["desc"]
                    and rp_meta.get("precision") == args.precision and rp_meta.get("graphs") == bool(graphs)
                    and rp_meta.get("batch") == batch)
        roof = rocprof_headline(roof, rp.get("grouped_gemm"), rp_src, rp_match)
        rd = roofline_entry(ksum.get("dispatch"), pmc.get("dispatch"), prof_elapsed,
                            "dispatch kernels of this workload: combine_fwd (gate-weighted combine + residual) at "
                            "C2 / C5; permute_fwd + combine_fwd / _bwd where rows are copied (the EP send layout, "
                            "C4). The scatter half of the C2 dispatch has no kernel of its own: GEMM1 gathers the "
                            "token rows through the row map in its LDS-DMA loads (its bytes are in the grouped-GEMM "
                            "entry)")
        rd = rocprof_headline(rd, rp.get("dispatch"), rp_src, rp_match)
        kprof = {}
        for name, d in ksum.items():
            if d["total_ms"] <= 0:
                continue
            sec = d["total_ms"] * 1e-3
            kprof[name] = {"launches_per_step": round(d["launches"] / prof_steps, 1), "avg_us": round(d["avg_us"], 2),
                           "ms_per_step": round(d["total_ms"] / prof_steps, 3),
                           "GB_s": round(d["bytes"] / sec / 1e9, 1),
                           "roofline_time_frac": round(d["t_roof_ms"] / d["total_ms"], 4)}
            if d["flops"]:
                kprof[name]["TFLOP_s"] = round(d["flops"] / sec / 1e12, 1)
        result = {
            "metric": METRIC, "value": round(value, 3), "unit": "images/sec", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": round(1e3 * elapsed / args.steps, 3),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": wl.get("dtype", "bf16"),
            "data": "synthetic (ZOD-shaped batches resident in HBM, random-init weights)",
            "config": {"workload": wl["desc"], "arch": spec, "global_batch": world * batch,
                       "execution": ("hipGraph: forward + criterion (GPU matcher) + backward" if args.step_graph
                                     else "hipGraph fwd/bwd") if graphs else "eager",
                       "precision": "bf16 weights + fp32 master" if args.precision == "bf16" else "bf16 autocast",
                       "img": f"{args.img_w}x{args.img_h} (padded to {data.pad_w}x{data.pad_h})",
                       "parallelism": f"dp{world}" if "ep" not in spec else f"dp{world}+ep{world}",
                       "rccl_world": rccl_world, "batch": batch},
            "build": {"libmoe_hip_sha16": build_id, "precision": args.precision, "graphs": bool(graphs),
                      "tune": list(args.tune), "spec_extra": args.spec_extra},
            "roofline": roof, "roofline_dispatch": rd, "kernel_profile": kprof,
            "kernel_timing": None if not timing else (
                f"libmoe_hip dispatch-stamped events over the {args.steps} timed steps" if not graphs else
                f"libmoe_hip dispatch-stamped events over {args.profile_steps} eager steps right after the "
                f"timed region (same shapes; the timed steps replay hipGraphs, which carry no timing events)"),
            **({"eval": ev} if ev else {}),
            "dp_exchange": dp_exchange_bytes(model, world),
            **({"phases_gpu_host_ms": phases} if phases else {}),
            **({"expert_parallel": ep_stats} if ep_stats else {}),
        }
    if world > 1:
        from src.rtdetr_moe.step import release_graphs

        dist.barrier()
        step = None  # its captured graphs (C4: RCCL all-to-alls inside) go before the communicator
        release_graphs()
        dist.destroy_process_group()
    if rank == 0:
        if not args.no_e2e_roofline:
            log(rank, "counting model FLOP per image (fp32 CPU fwd+bwd under FlopCounterMode)")
            try:
                threads, _ = host_threads()
                torch.set_num_threads(threads)
                fpi = model_flop_per_image(spec, args.img_h, args.img_w)
                ach = result["value"] * fpi / 1e12
                result["roofline_e2e"] = {
                    "bound": "mfma", "achieved": round(ach, 2), "peak": PEAK_BF16_TFLOPS, "unit": "TFLOP/s",
                    "frac": round(ach / PEAK_BF16_TFLOPS, 4), "model_gflop_per_image": round(fpi / 1e9, 2),
                    "source": "images/s x FlopCounterMode FLOP of one fp32 CPU fwd+bwd per image (same model, "
                              f"{args.img_w}x{args.img_h}) / dense bf16 MFMA peak"}
            except Exception as e:  # report, never hide
                result["roofline_e2e"] = {"value": None, "error": f"{type(e).__name__}: {e}"}
        if world == 1 and not args.no_cpu_baseline:
            log(rank, "timing the CPU baseline")
            try:
                result["cpu_baseline"] = cpu_baseline(spec, batch, args.img_h, args.img_w, args.cpu_seconds)
            except Exception as e:  # report, never hide, a failed baseline
                result["cpu_baseline"] = {"value": None, "error": f"{type(e).__name__}: {e}"}
        else:
            result["cpu_baseline"] = None
        print(json.dumps(result), flush=True)


if __name__ == "__main__":
    main()
