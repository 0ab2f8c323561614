"""Encoder pass times vs working-set size (measurement tool, run under
rocprofv3 --kernel-trace --stats): does the write pass's second read of the
values come cheaper when the values are still in the 256 MiB Infinity Cache?

  mode full   : 10M-block C4-mix encode, `reps` times (values cold: 10 GB)
  mode chunkC : the same 10M blocks encoded as consecutive C-block chunks
                (plan(c), scan(c), write(c) back to back: write re-reads the
                chunk the plan pass just read)
usage: python scripts/enc_chunk_probe.py MODE [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, ROOT)
import turbopfor_amd as tpf  # noqa: E402
import bench  # noqa: E402

mode = sys.argv[1]
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 5
nb = 10_000_000
dev = torch.device("cuda:0")
vals, _ = bench.gen_c2(nb, 0, seed=11, dev=dev, pcts=[0, 5, 10, 25])
cap = int(tpf.lib().tpf_p4enc256v32_bound(nb))
out = torch.empty(cap, dtype=torch.uint8, device=dev)
if mode == "full":
    for _ in range(reps):
        tpf.enc256v32(vals, out=out)
else:
    c = int(mode[len("chunk"):])
    ccap = int(tpf.lib().tpf_p4enc256v32_bound(c))
    for _ in range(reps):
        for a in range(0, nb, c):
            m = min(c, nb - a)
            tpf.enc256v32(vals[a:a + m], out=out[: ccap if m == c else int(tpf.lib().tpf_p4enc256v32_bound(m))])
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
if mode == "full":
    tpf.enc256v32(vals, out=out)
else:
    for a in range(0, nb, c):
        m = min(c, nb - a)
        tpf.enc256v32(vals[a:a + m], out=out[: int(tpf.lib().tpf_p4enc256v32_bound(m))])
e1.record()
torch.cuda.synchronize()
print(mode, "one 10M-block pass (host loop incl.):", round(e0.elapsed_time(e1), 3), "ms")
