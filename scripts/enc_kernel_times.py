"""Encoder kernel timing (measurement tool; run under rocprofv3 --kernel-trace
--stats for per-kernel times): C4-mix 256v32 encode, `reps` launches.
usage: python scripts/enc_kernel_times.py [nblocks] [reps] [probe]
probe 1/2: tpfm_enc256v32 modes 1/2 (the plan / write pass with the coding removed), 3 two-pass, 4 slot"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, ROOT)
import turbopfor_amd as tpf  # noqa: E402
import bench  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
probe = int(sys.argv[3]) if len(sys.argv) > 3 else 0
dev = torch.device("cuda:0")
vals, _ = bench.gen_c2(nb, 0, seed=11, dev=dev, pcts=[0, 5, 10, 25])
cap = int(tpf.lib().tpf_p4enc256v32_bound(nb))
out = torch.empty(cap, dtype=torch.uint8, device=dev)
for _ in range(reps):
    if probe:
        tpf.enc256v32_path(probe, vals, out)
    else:
        tpf.enc256v32(vals, out=out)
torch.cuda.synchronize()
print("done", probe)
