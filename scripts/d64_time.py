"""256v64 decode timing for library A/B runs (TPF_LIB selects the build):
C4's 64-bit leg (bench_data.gen_v64, 10M units by default), plain decode of
the whole stream `reps` times per round, best round; verified against the
values.  Prints one line: lib, ms, G int64/s, GB/s of algorithmic bytes.
usage: TPF_LIB=ablib/x.so python scripts/d64_time.py [nunits] [rounds]"""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, ROOT)
import bench_data  # noqa: E402
import turbopfor_amd as tpf  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
rounds = int(sys.argv[2]) if len(sys.argv) > 2 else 3
dev = torch.device("cuda:0")
v64 = bench_data.gen_v64(nb, seed=5, dev=dev)
packed, offs = tpf.enc_batch("256v64", v64.view(-1), nb, 256)
out = torch.empty(nb * 256, dtype=torch.int64, device=dev)
err = torch.zeros(1, dtype=torch.int64, device=dev)
tpf.dec_batch("256v64", packed, offs, nb, 256, out=out, err=err)
torch.cuda.synchronize()
ok = bool(torch.equal(out.view(nb, 256), v64)) and int(err.item()) == -1
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
best = 1e9
for _ in range(rounds):
    e0.record()
    for _ in range(10):
        tpf.dec_batch("256v64", packed, offs, nb, 256, out=out)
    e1.record()
    e1.synchronize()
    best = min(best, e0.elapsed_time(e1) / 10)
alg = packed.numel() + nb * (2048 + 8) + 8
print(f"{os.path.basename(os.environ.get('TPF_LIB', 'tree'))} dec256v64 ms={best:.4f} G_int64/s={nb * 256 / best / 1e6:.1f} "
      f"GB/s={alg / best / 1e6:.0f} frac={alg / best / 1e6 / 8000:.4f} B/unit={packed.numel() / nb:.1f} verified={ok}", flush=True)
