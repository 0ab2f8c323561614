"""Per-width sweep of the plain 256v32 decode through both load paths
(measurement tool): for bw 1..32, nblocks blocks of that
width alone (10% exceptions for bw <= 28, bench.gen_bw), GPU-encoded; the
single-block pipeline and the grouped 1 KB loads (tpfm_dec256v32_path), and
the library's own per-launch choice (tpf.dec256v32), each timed with HIP
events over `reps` launches and verified.
usage: python scripts/dec_paths_sweep.py [nblocks] [reps]"""
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
dev = torch.device("cuda:0")
out = torch.empty((nb, 256), dtype=torch.int32, device=dev)


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


print("bw bytes_per_block single_ms grouped_ms library_ms library_path G_int32_per_s(single/grouped/library) verified", flush=True)
for bw in range(1, 33):
    vals = bench.gen_bw(nb, bw, 10.0, seed=42, dev=dev)
    p, o = tpf.enc256v32(vals)
    p = p.clone()
    res, ok = {}, True
    for name, f in (("single", lambda: tpf.dec256v32_path(0, p, o, nb, out)),
                    ("grouped", lambda: tpf.dec256v32_path(1, p, o, nb, out)),
                    ("library", lambda: tpf.dec256v32(p, o, nb, out=out))):
        out.zero_()
        res[name] = timed(f)
        ok = ok and bool(torch.equal(out, vals))
    choice = "grouped" if abs(res["library"] - res["grouped"]) < abs(res["library"] - res["single"]) else "single"
    g = lambda ms: round(nb * 256 / (ms * 1e-3) / 1e9, 1)
    print(bw, round(p.numel() / nb, 1), round(res["single"], 4), round(res["grouped"], 4), round(res["library"], 4), choice,
          f"{g(res['single'])}/{g(res['grouped'])}/{g(res['library'])}", ok, flush=True)
    del vals, p, o
