"""Launch-latency probe (measurement tool): one-block p4Dec256v32 batch call
+ synchronize, launched directly vs replayed from a captured hipGraph."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
import turbopfor_amd as tpf  # noqa: E402

dev = torch.device("cuda:0")
vals = torch.randint(0, 1 << 12, (1, 256), dtype=torch.int32, device=dev)
packed, offs = tpf.enc256v32(vals)
out = torch.empty_like(vals)
s = torch.cuda.Stream()
with torch.cuda.stream(s):
    for _ in range(20):
        tpf.dec256v32(packed, offs, 1, out=out)
    s.synchronize()
    n = 2000
    t0 = time.perf_counter()
    for _ in range(n):
        tpf.dec256v32(packed, offs, 1, out=out)
        s.synchronize()
    direct = (time.perf_counter() - t0) / n
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        tpf.dec256v32(packed, offs, 1, out=out)
    for _ in range(20):
        g.replay()
    s.synchronize()
    t0 = time.perf_counter()
    for _ in range(n):
        g.replay()
        s.synchronize()
    graph = (time.perf_counter() - t0) / n
print(f"direct launch + sync {direct * 1e6:.1f} us, graph replay + sync {graph * 1e6:.1f} us")
