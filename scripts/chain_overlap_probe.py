"""Chained-D1 overlap probe (measurement tool): does phase A (block sums,
compute-bound) of one part of a list co-run with phase B (decode,
memory-bound) of another part on a second stream?  C3 list, 10M blocks."""
import os
import sys
import time

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, ROOT)
import turbopfor_amd as tpf  # noqa: E402
import bench  # noqa: E402

dev = torch.device("cuda:0")
nb = 10_000_000
vals, starts = bench.gen_c3(nb, seed=7, dev=dev)
packed, offs = tpf.enc256v32(vals, d1=True, starts=starts)
packed = packed.clone()
start0 = int(starts[0].item()) & 0xFFFFFFFF
out = torch.empty((nb, 256), dtype=torch.int32, device=dev)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e3


full = tpf.D1Chain(packed, offs, nb)
print(f"serial A+B (one list)           {timed(lambda: (full.sums(), full.decode(start0, out=out))):.3f} ms")
for K in (2, 4, 8):
    cuts = [nb * k // K for k in range(K + 1)]
    parts = [tpf.D1Chain(packed, offs[cuts[k]:], cuts[k + 1] - cuts[k]) for k in range(K)]
    # bases from one serial pass (the totals do not change between runs)
    bases, b = [], start0
    for k in range(K):
        bases.append(b)
        b = (b + int(parts[k].sums().item())) & 0xFFFFFFFF
    side = torch.cuda.Stream()
    main = torch.cuda.current_stream()
    evA = [torch.cuda.Event() for _ in range(K)]

    def overlapped():
        parts[0].sums()
        evA[0].record(main)
        side.wait_stream(main)
        with torch.cuda.stream(side):
            for k in range(1, K):
                parts[k].sums()
                evA[k].record(side)
        for k in range(K):
            if k:
                main.wait_event(evA[k])
            parts[k].decode(bases[k], out=out[cuts[k]:cuts[k + 1]])

    ms = timed(overlapped)
    ok = torch.equal(out, vals)
    print(f"K={K}: A(k+1..) on a side stream beside B(k)  {ms:.3f} ms  ok={ok}")
