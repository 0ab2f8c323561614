"""Measurement only: can phase A (compute-bound block sums) of one chunk of a
chained list overlap phase B (HBM-bound decode) of the previous chunk?
Splits the C3 list into K chunks; chunk c's sums run on stream A, its decode
on stream B after an event.  Decode bases are 0 (timing only: the values are
not the list's), so `verified` is reported only for K = 1.
usage: python scripts/chain_overlap_probe.py [nblocks] [K ...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, ROOT)
import turbopfor_amd as tpf  # noqa: E402
import bench_data  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
ks = [int(x) for x in sys.argv[2:]] or [1, 2, 4, 8, 16, 32]
dev = torch.device("cuda:0")
vals, starts = bench_data.gen_c3(nb, 7, dev)
packed, offs = tpf.enc256v32(vals, d1=True, starts=starts)
packed = packed.clone()
out = torch.empty((nb, 256), dtype=torch.int32, device=dev)
sA, sB = torch.cuda.Stream(), torch.cuda.Stream()


def plan(k):
    cuts = [nb * c // k // 64 * 64 for c in range(k)] + [nb]
    chains = [(tpf.D1Chain(packed, offs[cuts[c]:], cuts[c + 1] - cuts[c]), cuts[c], cuts[c + 1]) for c in range(k)]
    evs = [torch.cuda.Event() for _ in range(k)]
    return chains, evs


def run(chains, evs):
    cur = torch.cuda.current_stream()
    sA.wait_stream(cur)
    sB.wait_stream(cur)
    for (ch, s, e), ev in zip(chains, evs):
        with torch.cuda.stream(sA):
            ch.sums()
            ev.record(sA)
        with torch.cuda.stream(sB):
            sB.wait_event(ev)
            ch.decode(0, out=out[s:e])
    cur.wait_stream(sB)
    cur.wait_stream(sA)


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best


for k in ks:
    chains, evs = plan(k)
    t = timed(lambda: run(chains, evs))
    print(f"K={k}: {t:.4f} ms ({nb * 256 / t / 1e6:.1f} G int32/s)", flush=True)
