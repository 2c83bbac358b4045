"""Probe: is the C2 step host-bound, and does hipGraph replay remove it?
Times, for the bf16 model (bench.py defaults): eager forward (no grad), the
same forward captured in a hipGraph and replayed, and eager fwd+bwd; plus the
host enqueue time of each (no sync)."""
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
for p in (str(ROOT / "multimodal-moe_amd"), str(ROOT)):
    sys.path.insert(0, p)
import os  # noqa: E402
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
import torch  # noqa: E402


def main():
    import bench
    from src.moe import _lib as L
    from src.rtdetr_moe.data import SyntheticZOD
    from src.rtdetr_moe.step import FlatOutputs, gemm_params

    torch.backends.cudnn.benchmark = True
    L.lib()
    dev = torch.device("cuda", 0)
    model = bench.build_model("rtdetr-r50-moe8-top2", dev, 1)
    for p in gemm_params(model):
        p.data = p.data.to(torch.bfloat16)
    flat = FlatOutputs(model)
    images, targets, ctx = SyntheticZOD(batch=8, img_h=720, img_w=1280, seed=1).sample(dev)
    images = images.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)

    def timeit(fn, n=10):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        th = time.perf_counter() - t0
        torch.cuda.synchronize()
        tw = time.perf_counter() - t0
        return 1e3 * th / n, 1e3 * tw / n

    with torch.no_grad():
        h, w = timeit(lambda: flat(images, ctx))
        print(f"eager fwd (no grad): host {h:.2f} ms  wall {w:.2f} ms", flush=True)
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            for _ in range(2):
                flat(images, ctx)
        torch.cuda.current_stream().wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            out = flat(images, ctx)
        h, w = timeit(g.replay)
        print(f"graph fwd (no grad): host {h:.2f} ms  wall {w:.2f} ms", flush=True)

    def fb():
        for p in model.parameters():
            p.grad = None
        o = flat(images, ctx)
        sum(x.float().sum() for x in o).backward()
    h, w = timeit(fb, 5)
    print(f"eager fwd+bwd:      host {h:.2f} ms  wall {w:.2f} ms", flush=True)


if __name__ == "__main__":
    main()
