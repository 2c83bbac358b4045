"""Stage-by-stage probe of RCCL (world-1 ``nccl`` group) inside a captured
hipGraph -- the C4 expert-parallel exchange path of bench.py --gpus N
(src/moe/ep.py ``_a2a``).  Each stage prints as it finishes; a stack dump
every 30 s names the stage that does not.

    python tools/rccl_capture_probe.py [--device-id] [--sleep=S] [--mode=global|thread_local|relaxed] [--release] > gpurun_out/rccl_probe.log 2>&1
"""
from __future__ import annotations

import faulthandler
import os
import socket
import sys
import time

import torch
import torch.distributed as dist

faulthandler.dump_traceback_later(30, repeat=True)
T0 = time.time()


def say(msg):
    print(f"[{time.time() - T0:7.2f}s] {msg}", flush=True)


def main():
    dev = torch.device("cuda", 0)
    torch.cuda.set_device(dev)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    kw = {"device_id": dev} if "--device-id" in sys.argv else {}
    dist.init_process_group("nccl", init_method=f"tcp://127.0.0.1:{port}", rank=0, world_size=1, **kw)
    say(f"init ok {kw}")
    x = torch.arange(4096, dtype=torch.float32, device=dev).reshape(64, 64)
    out = torch.empty_like(x)
    dist.all_to_all_single(out, x)
    torch.cuda.synchronize()
    say(f"eager a2a ok equal={torch.equal(out, x)}")
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(2):
            dist.all_to_all_single(out, x * 2)
    torch.cuda.current_stream().wait_stream(side)
    torch.cuda.synchronize()
    say("side-stream warm-up ok")
    sleep = float(next((a.split("=")[1] for a in sys.argv if a.startswith("--sleep=")), "0"))
    mode = next((a.split("=")[1] for a in sys.argv if a.startswith("--mode=")), "global")
    time.sleep(sleep)  # lets the watchdog retire the warm-up works (their events) before the capture
    g = torch.cuda.CUDAGraph()
    xs = x.clone()
    with torch.cuda.graph(g, stream=side, capture_error_mode=mode):
        y = xs * 3
        dist.all_to_all_single(out, y)
        z = out + 1
    say("capture ok")
    torch.cuda.synchronize()
    for i in range(3):
        xs.copy_(x + i)
        g.replay()
    torch.cuda.synchronize()
    say(f"replay ok equal={torch.equal(z, (x + 2) * 3 + 1)}")
    # bf16 and int64 as the EP layer exchanges them
    for dt in (torch.bfloat16, torch.int64):
        a = torch.ones(128, 256, dtype=dt, device=dev)
        b = torch.empty_like(a)
        g2 = torch.cuda.CUDAGraph()
        with torch.cuda.stream(side):
            dist.all_to_all_single(b, a)
        torch.cuda.synchronize()
        time.sleep(sleep)
        with torch.cuda.graph(g2, stream=side, capture_error_mode=mode):
            dist.all_to_all_single(b, a)
        g2.replay()
        torch.cuda.synchronize()
        say(f"{dt} capture+replay ok equal={torch.equal(a, b)}")
        dist.all_to_all_single(b, a)  # an eager collective after the captured ones (the nccl stream reused)
        torch.cuda.synchronize()
        time.sleep(0.5)
        say(f"{dt} eager after replay ok")
    if "--release" in sys.argv:  # drop the graphs (their captured RCCL kernels) before the communicator
        import gc

        del g, g2
        gc.collect()
        torch.cuda.synchronize()
        say("graphs released")
    dist.destroy_process_group()
    say("destroyed")


if __name__ == "__main__":
    main()
    faulthandler.cancel_dump_traceback_later()
