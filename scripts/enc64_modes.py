"""Block-mode mix of an encoded stream (measurement tool): the header byte of
the FIRST 128v64 block of every 256v64 unit of C4's 64-bit leg, and of every
256v32 block of the C3 D1 posting list, counted by mode (plain / bitmap /
vbyte / constant; a vbyte block with the 0xFF raw escape is not told apart).
usage: python scripts/enc64_modes.py [nunits]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, ROOT)
import turbopfor_amd as tpf  # noqa: E402
import bench  # noqa: E402
import bench_data  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
dev = torch.device("cuda:0")


def mix(packed, offs, n):
    h = packed[offs[:n].long()].to(torch.int32)
    kinds = {"plain": int(((h & 0xC0) == 0x00).sum()), "bitmap": int(((h & 0xC0) == 0x80).sum()),
             "vbyte": int(((h & 0xC0) == 0x40).sum()), "constant": int(((h & 0xC0) == 0xC0).sum())}
    return {k: round(v / n, 4) for k, v in kinds.items()}


v64 = bench_data.gen_v64(nb, seed=5, dev=dev)
p64, o64 = tpf.enc_batch("256v64", v64.view(-1), nb, 256)
print("C4 64-bit leg, first block of each unit:", mix(p64, o64, nb), "bytes/unit", round(int(o64[-1]) / nb, 1))
del v64, p64, o64
vals, starts = bench.gen_c3(nb, seed=7, dev=dev)
p32, o32 = tpf.enc256v32(vals, d1=True, start0=int(starts[0].item()) & 0xFFFFFFFF)
print("C3 D1 list, 256v32 blocks:", mix(p32, o32, nb), "bytes/block", round(int(o32[-1]) / nb, 1))
