"""Encoder kernel timing (measurement tool; run under rocprofv3 --kernel-trace
--stats for per-kernel times, or --pmc for counters): `reps` launches of the
256v32 encoder on the C4 mix, or (data c3) p4D1Enc256v32 of the C3 posting
list chained from start0.
usage: python scripts/enc_kernel_times.py [nblocks] [reps] [mode] [c4|c3]
mode 0: the library's choice; 1/2: tpfm_enc256v32 pass probes (the plan /
write pass with the coding removed; 1 c4 only, 2 also c3: after the real D1
plan); 3 two-pass; 4 slot; 5 slot
without the fused scans.  Prints HIP-event ms per launch."""
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
data = sys.argv[4] if len(sys.argv) > 4 else "c4"
dev = torch.device("cuda:0")
if data == "c3":
    vals, starts = bench.gen_c3(nb, seed=7, dev=dev)
    start0 = int(starts[0].item()) & 0xFFFFFFFF
else:
    vals, _ = bench.gen_c2(nb, 0, seed=11, dev=dev, pcts=[0, 5, 10, 25])
    start0 = 0
d1 = data == "c3"
cap = int(tpf.lib().tpf_p4enc256v32_bound(nb))
out = torch.empty(cap, dtype=torch.uint8, device=dev)


def once():
    if probe:
        tpf.enc256v32_path(probe, vals, out, d1=d1, start0=start0)
    else:
        tpf.enc256v32(vals, d1=d1, start0=start0, out=out)


once()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record()
for _ in range(reps):
    once()
e1.record()
torch.cuda.synchronize()
print("done", data, "mode", probe, "ms/launch", round(e0.elapsed_time(e1) / reps, 4))
