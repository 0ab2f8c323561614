"""Chained D1 decode split by phase (C3, 10M blocks): phase A (block sums +
run scan) alone, phase B alone, both; HIP events on torch's stream, best of
3 rounds of 10.  With a library built with -DTPF_DSUM_COUNT it also prints
how many blocks phase A sent to the wave decoder and its staging passes.
usage: TPF_LIB=ablib/x.so python scripts/chain_phase_probe.py [nblocks]"""
import ctypes
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, ROOT)
import turbopfor_amd as tpf  # noqa: E402
import bench_data  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 10_000_000
dev = torch.device("cuda:0")
vals, starts = bench_data.gen_c3(nb, 7, dev)
packed, offs = tpf.enc256v32(vals, d1=True, starts=starts)
packed = packed.clone()
chain = tpf.D1Chain(packed, offs, nb)
out = torch.empty((nb, 256), dtype=torch.int32, device=dev)
L = tpf.lib()
cnt = getattr(L, "tpf_dsum_counters", None) if hasattr(L, "tpf_dsum_counters") else None


def timed(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    best = 1e9
    for _ in range(3):
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(reps):
            fn()
        e1.record()
        torch.cuda.synchronize()
        best = min(best, e0.elapsed_time(e1) / reps)
    return best


a = timed(lambda: chain.sums())
chain.sums()
b = timed(lambda: chain.decode(0, out=out))
ab = timed(lambda: (chain.sums(), chain.decode(0, out=out)))
ok = bool(torch.equal(out, vals))
msg = f"{os.path.basename(os.environ.get('TPF_LIB', 'tree'))}: phaseA {a:.4f} ms  phaseB {b:.4f} ms  both {ab:.4f} ms " \
      f"({nb * 256 / ab / 1e6:.1f} G int32/s) verified {ok}"
if cnt is not None:
    c = (ctypes.c_ulonglong * 2)()
    cnt(c)
    msg += f"  [per phase-A call: fallback blocks {c[0] / 63:.0f}, passes {c[1] / 63:.0f}]"
print(msg, flush=True)
