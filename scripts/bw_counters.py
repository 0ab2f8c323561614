"""Per-bit-width decode counters (measurement tool, run under rocprofv3
--pmc): for each bit width, a 2M-block stream of that width alone (10%
exceptions for bw <= 28, the C2 generator), encoded, then decoded REPS times
with the product kernel.  Prints the order of the decode launches so that
scripts/bw_counters_report.py can map dispatches to widths.
usage: python scripts/bw_counters.py [nblocks] [bw ...]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, ROOT)
import turbopfor_amd as tpf  # noqa: E402
import bench  # noqa: E402

REPS = 3
nb = int(sys.argv[1]) if len(sys.argv) > 1 else 2_000_000
bws = [int(x) for x in sys.argv[2:]] or [2, 3, 4, 5, 6, 7, 8, 16, 24, 25, 32]
dev = torch.device("cuda:0")
order = []
for bw in bws:
    vals = bench.gen_bw(nb, bw, 10.0, seed=3, dev=dev)
    packed, offs = tpf.enc256v32(vals.view(-1))
    out = torch.empty_like(vals)
    for _ in range(REPS):
        tpf.dec256v32(packed, offs, nb, out=out)
    torch.cuda.synchronize()
    assert torch.equal(out, vals), bw
    order.append((bw, packed.numel() / nb))
    del vals, packed, offs, out
    torch.cuda.empty_cache()
print("ORDER", ";".join(f"{bw}:{b:.1f}" for bw, b in order), flush=True)
