"""Probe: RCCL all-to-alls in the BACKWARD of a captured step (the C4
expert-parallel transposes run on autograd's device thread), world-1
``nccl`` group.  Stages print as they finish; the flight recorder
(TORCH_NCCL_TRACE_BUFFER_SIZE) lists every collective the process group
tracked, with its state, after the capture and after the graph is freed.

    TORCH_NCCL_TRACE_BUFFER_SIZE=64 python tools/rccl_autograd_probe.py [--cache0] [--drain] > log 2>&1
"""
from __future__ import annotations

import faulthandler
import gc
import os
import pickle
import socket
import sys
import time

if "--cache0" in sys.argv:
    os.environ["TORCH_NCCL_CUDA_EVENT_CACHE"] = "0"
os.environ.setdefault("TORCH_NCCL_TRACE_BUFFER_SIZE", "64")

import torch  # noqa: E402
import torch.distributed as dist  # noqa: E402

faulthandler.dump_traceback_later(30, repeat=True)
T0 = time.time()


def say(msg):
    print(f"[{time.time() - T0:7.2f}s] {msg}", flush=True)


def trace(tag):
    try:
        raw = torch._C._distributed_c10d._dump_nccl_trace()
    except Exception as e:  # noqa: BLE001
        say(f"{tag}: no trace ({e})")
        return
    d = pickle.loads(raw)  # this process's own flight-recorder dump
    ents = d.get("entries", [])
    say(f"{tag}: {len(ents)} entries")
    for e in ents[-12:]:
        say("   " + ", ".join(f"{k}={e.get(k)}" for k in ("record_id", "profiling_name", "state", "is_p2p")
                                if k in e))


class A2A(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x):
        out = torch.empty_like(x)
        dist.all_to_all_single(out, x.contiguous())
        return out

    @staticmethod
    def backward(ctx, g):
        say(f"   backward a2a thread={__import__('threading').current_thread().name} "
            f"capturing={torch.cuda.is_current_stream_capturing()}")
        out = torch.empty_like(g)
        dist.all_to_all_single(out, g.contiguous())
        return out


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, device_id=dev)
    say(f"init ok cache={os.environ.get('TORCH_NCCL_CUDA_EVENT_CACHE', 'default')}")
    w = torch.randn(64, 64, device=dev, requires_grad=True)
    x = torch.randn(32, 64, device=dev)

    def step():
        y = A2A.apply(x @ w)
        (g,) = torch.autograd.grad((y * y).sum(), [w])
        return g

    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            ref = step()
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    say("eager warm-up ok")
    if "--drain" in sys.argv:
        time.sleep(0.5)
    trace("before capture")
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=side, capture_error_mode="thread_local"):
        out = step()
    say("capture ok")
    for _ in range(3):
        g.replay()
    torch.cuda.synchronize()
    say(f"replay ok equal={torch.equal(out, ref)}")
    time.sleep(1.0)
    say("slept 1 s with the graph alive")
    trace("after replay")
    del g
    gc.collect()
    torch.cuda.synchronize()
    say("graph freed")
    time.sleep(1.0)
    say("slept 1 s after the graph was freed")
    trace("after free")
    dist.destroy_process_group()
    say("destroyed")


if __name__ == "__main__":
    main()
    faulthandler.cancel_dump_traceback_later()
