"""Probe: do timing events recorded inside a captured hipGraph report elapsed times after replay?"""
import torch

x = torch.randn(4096, 4096, device="cuda")
s = torch.cuda.Event(enable_timing=True)
e = torch.cuda.Event(enable_timing=True)
s.record(); y = x @ x; e.record(); torch.cuda.synchronize()
print("eager ms", s.elapsed_time(e))
g = torch.cuda.CUDAGraph()
st = torch.cuda.Stream()
with torch.cuda.stream(st):
    y = x @ x
    torch.cuda.synchronize()
    with torch.cuda.graph(g, stream=st):
        s.record(); y = x @ x; e.record()
for i in range(3):
    g.replay(); torch.cuda.synchronize()
    try:
        print("graph ms (pre-created events)", s.elapsed_time(e))
    except Exception as ex:
        print("graph elapsed failed:", type(ex).__name__, str(ex)[:100])
s2 = torch.cuda.Event(enable_timing=True); e2 = torch.cuda.Event(enable_timing=True)
g2 = torch.cuda.CUDAGraph()
with torch.cuda.stream(st):
    with torch.cuda.graph(g2, stream=st):
        s2.record(); y = x @ x; e2.record()
g2.replay(); torch.cuda.synchronize()
try:
    print("graph ms (fresh events)", s2.elapsed_time(e2))
except Exception as ex:
    print("fresh elapsed failed:", type(ex).__name__, str(ex)[:100])
