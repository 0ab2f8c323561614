"""Chained-D1 phase A (block delta sums) variants (scripts/dec_variants.hip
decvar_sums: pipeline depth NC, waves/SIMD, run length) against the
product's phase A (tpf_p4d1dec256v32_chain_sums), C3 postings, 10M blocks,
A/B in one process, every variant's sums compared with the product's.
usage: python scripts/chain_sum_variants.py [nblocks] [rounds]"""
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
dev = torch.device("cuda:0")
V = ctypes.CDLL(os.path.join(ROOT, "scripts", "libdecvar.so"))
V.decvar_sums.restype = ctypes.c_int
V.decvar_sums.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                          ctypes.c_void_p]
L = tpf.lib()
NAMES = {0: "nc6w7r16", 1: "nc4w8r16", 2: "nc3w8r16", 3: "nc8w6r16", 4: "nc6w7r32", 5: "nc4w8r32", 6: "nc2w8r16",
         7: "nc12w4r16", 8: "defer_nc4w8r32", 9: "defer_nc4w8r16", 10: "defer_nc6w7r16"}
vals, starts = bench.gen_c3(nb, seed=7, dev=dev)
packed, offs = tpf.enc256v32(vals.view(-1), d1=True, starts=starts)
del vals, starts
s = torch.cuda.current_stream().cuda_stream
wsb = int(L.tpf_p4d1dec256v32_chain_workspace_size(nb))
ws = torch.zeros(wsb, dtype=torch.uint8, device=dev)
tot = torch.zeros(1, dtype=torch.int32, device=dev)


def prod():
    assert L.tpf_p4d1dec256v32_chain_sums(packed.data_ptr(), packed.numel(), offs.data_ptr(), nb, ws.data_ptr(), wsb,
                                          tot.data_ptr(), None, ctypes.c_void_p(s)) == 0


prod()
torch.cuda.synchronize()
ref = ws[:nb * 4].view(torch.int32).clone()
out = torch.empty(nb, dtype=torch.int32, device=dev)
cands = [("prod", prod)]
for v, n in NAMES.items():
    def f(v=v):
        assert V.decvar_sums(v, packed.data_ptr(), packed.numel(), offs.data_ptr(), nb, out.data_ptr(), s) == 0
    cands.append((n, f))
    out.zero_()
    f()
    torch.cuda.synchronize()
    assert torch.equal(out, ref), n
best = {n: 1e9 for n, _ in cands}
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
for r in range(rounds):
    for n, fn in cands:
        fn()
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        e1.synchronize()
        best[n] = min(best[n], e0.elapsed_time(e1) / 10)
print(f"[c3 phase A] B/blk={packed.numel() / nb:.1f} " + " ".join(f"{n}={best[n]:.4f}" for n, _ in cands), flush=True)
print("ok")
