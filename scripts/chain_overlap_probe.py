"""Feasibility probe (measurement tool): does phase A of one part of a chained
list overlap with phase B of another when they run on two streams?

C3 posting list (10M blocks), p4D1Enc256v32-encoded as one chained list.
  seq   : tpf_p4d1dec256v32_chained over the whole list (phase A, scan, phase B)
  split : the list cut into K parts; part k's phase A runs on a second stream
          while part k-1's phase B runs on the first (bases precomputed on the
          host from a first run: timing only, the real pipeline would carry
          them on the device).
Prints ms per decode for both and checks the split output.
usage: python scripts/chain_overlap_probe.py [nblocks] [K] [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, ROOT)
import turbopfor_amd as tpf  # noqa: E402
import bench  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
K = int(sys.argv[2]) if len(sys.argv) > 2 else 4
reps = int(sys.argv[3]) if len(sys.argv) > 3 else 10
dev = torch.device("cuda:0")
vals, starts = bench.gen_c3(nb, seed=7, dev=dev)
start0 = int(starts[0].item()) & 0xFFFFFFFF
packed, offs = tpf.enc256v32(vals, d1=True, start0=start0)
offs_h = offs.cpu()
out = torch.empty((nb, 256), dtype=torch.int32, device=dev)

# whole list
ws_all = torch.empty(int(tpf.lib().tpf_p4d1dec256v32_chain_workspace_size(nb)), dtype=torch.uint8, device=dev)


def seq():
    tpf.dec256v32_chained(packed, offs, nb, start0=start0, out=out, ws=ws_all)


# parts: rebased bytes and offsets
cuts = [(nb * k) // K for k in range(K + 1)]
parts = []
for k in range(K):
    a, b = cuts[k], cuts[k + 1]
    o0 = int(offs_h[a])
    p = packed[o0:int(offs_h[b])]
    o = (offs[a:b + 1] - o0).contiguous()
    parts.append((tpf.D1Chain(p, o, b - a), out[a:b]))
# bases from a first pass
bases = []
base = start0
for ch, _ in parts:
    bases.append(base)
    base = (base + int(ch.sums().item())) & 0xFFFFFFFF
torch.cuda.synchronize()

s1 = torch.cuda.current_stream()
s2 = torch.cuda.Stream()


def split():
    ev = []
    # phase A of every part on s2, each signalling its own event
    s2.wait_stream(s1)
    with torch.cuda.stream(s2):
        for ch, _ in parts:
            ch.sums()
            e = torch.cuda.Event()
            e.record(s2)
            ev.append(e)
    # phase B of part k on s1 once its phase A is done
    for k, (ch, o) in enumerate(parts):
        s1.wait_event(ev[k])
        ch.decode(bases[k], out=o)
    s1.wait_stream(s2)


def timed(f):
    f()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


t_seq = timed(seq)
ref = out.clone()
out.zero_()
t_split = timed(split)
ok = bool(torch.equal(out, ref)) and bool(torch.equal(ref, vals))
g = lambda ms: round(nb * 256 / (ms * 1e-3) / 1e9, 1)
print(f"nblocks {nb} K {K}: seq {t_seq:.4f} ms ({g(t_seq)} G int32/s)  split {t_split:.4f} ms ({g(t_split)} G int32/s)  ok {ok}")
