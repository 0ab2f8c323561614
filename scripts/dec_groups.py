"""Grouped-load decode variants (scripts/dec_groups.hip, measurement tool)
against the product kernel, on full-size streams, A/B in one process.
Every variant's output is compared with the product decode's; times are HIP
events on torch's stream, best of `rounds` rounds of 10 launches, variants
alternating within each round.
usage: python scripts/dec_groups.py [nblocks] [rounds] [streams...]
streams: bwN (one bit width, 10% exceptions), c2, c3"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, ROOT)
import turbopfor_amd as tpf  # noqa: E402
import bench  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
names = sys.argv[3:] or ["bw1", "bw2", "bw4", "bw8", "bw12", "bw16", "bw17", "bw24", "bw32", "c2", "c3"]
dev = torch.device("cuda:0")
V = ctypes.CDLL(os.path.join(ROOT, "scripts", "libdecgrp.so"))
V.decgrp_launch.restype = ctypes.c_int
V.decgrp_launch.argtypes = [ctypes.c_int, ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                            ctypes.c_uint64, ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
DEALS = {0: "g16n6w7", 1: "g32n6w7", 2: "g64n6w7", 3: "g32n4w8", 4: "g64n8w6", 5: "g32n8w6"}
NOPROBE = set()
if os.environ.get("DEALS"):
    DEALS = {int(k): v for k, v in DEALS.items() if str(k) in os.environ["DEALS"].split(",")}


def stream_of(name):
    if name == "c2":
        vals, _ = bench.gen_c2(nb, 10.0, seed=7, dev=dev)
    elif name == "c3":
        vals, _ = bench.gen_c3(nb, seed=7, dev=dev)
        vals = vals.view(nb, 256)
    elif name == "c3d1":
        vals, starts = bench.gen_c3(nb, seed=7, dev=dev)
        packed, offs = tpf.enc256v32(vals.view(-1), d1=True, starts=starts)
        return (vals, starts), packed, offs
    else:
        vals = bench.gen_bw(nb, int(name[2:]), 10.0, seed=7, dev=dev)
    packed, offs = tpf.enc256v32(vals.view(-1))
    return vals, packed, offs


for name in names:
    vals, packed, offs = stream_of(name)
    starts = None
    if isinstance(vals, tuple):
        vals, starts = vals
        o1 = tpf.dec256v32(packed, offs, nb, starts=starts)
        assert torch.equal(o1, vals.view(nb, 256)), name
        del o1
    del vals
    ref = tpf.dec256v32(packed, offs, nb)
    out = torch.empty_like(ref)
    s = torch.cuda.current_stream().cuda_stream

    def run_var(deal, probe):
        rc = V.decgrp_launch(deal, probe, packed.data_ptr(), packed.numel(), offs.data_ptr(), nb, out.data_ptr(), None, s)
        assert rc == 0, rc

    cands = [("prod", lambda: tpf.dec256v32(packed, offs, nb, out=out)),
             ("prod-probe", lambda: tpf.probe256v32(packed, offs, nb, out))]
    if starts is not None:
        cands.append(("prod-d1", lambda: tpf.dec256v32(packed, offs, nb, out=out, starts=starts)))
    for d, dn in DEALS.items():
        cands.append((dn, (lambda d=d: run_var(d, 0))))
        if d not in NOPROBE:
            cands.append((dn + "-probe", (lambda d=d: run_var(d, 1))))
    for cn, fn in cands:
        if cn.endswith("probe") or cn == "prod-d1":  # prod-d1 verified against the values above
            continue
        out.zero_()
        fn()
        torch.cuda.synchronize()
        assert torch.equal(out, ref), (name, cn)
    best = {cn: 1e9 for cn, _ in cands}
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    for r in range(rounds):
        for cn, fn in cands:
            fn()
            e0.record()
            for _ in range(10):
                fn()
            e1.record()
            e1.synchronize()
            best[cn] = min(best[cn], e0.elapsed_time(e1) / 10)
    bpb = packed.numel() / nb
    line = " ".join(f"{cn}={best[cn]:.4f}" for cn, _ in cands)
    print(f"[{name}] B/blk={bpb:7.1f} {line}", flush=True)
    alg = packed.numel() + nb * 1032
    print(f"[{name}] GB/s: " + " ".join(f"{cn}={alg / best[cn] / 1e6:.0f}" for cn, _ in cands), flush=True)
    del packed, offs, ref, out
    torch.cuda.empty_cache()
print("ok")
