"""256v64 encoder kernel timing / counters (measurement tool; run under
rocprofv3 --kernel-trace --stats or --pmc): `reps` launches of p4Enc256v64 on
C4's 64-bit leg (bench_data.gen_v64: bw 1..64, 0/5/10/25% exceptions).
usage: python scripts/enc64_kernel_times.py [nunits] [reps]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, ROOT)
import turbopfor_amd as tpf  # noqa: E402
import bench_data  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda:0")
v64 = bench_data.gen_v64(nb, seed=5, dev=dev)
L = tpf.lib()
out = torch.empty(int(L.tpf_enc_bound(tpf.FMT["256v64"], nb, 256)), dtype=torch.uint8, device=dev)
ws = torch.empty(max(1, int(L.tpf_enc_workspace_size(tpf.FMT["256v64"], nb, 256))), dtype=torch.uint8, device=dev)
offs = torch.empty(nb + 1, dtype=torch.int64, device=dev)


def once():
    tpf.enc_batch("256v64", v64.view(-1), nb, 256, out=out, offs=offs, ws=ws)


once()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    once()
e1.record()
torch.cuda.synchronize()
print("done 256v64 encode ms/launch", round(e0.elapsed_time(e1) / reps, 4), "G int64/s", round(nb * 256 / (e0.elapsed_time(e1) / reps) / 1e6, 1))
