"""Phase times of the chained 64-bit decode (measurement tool, round 6):
tpf_d1dec64_chain_sums (phase A: k_dsum128v64_lanes + u64 run scan) and
tpf_d1dec64_chain_decode (phase B: k_dec128v64w<2, Prefix>) timed separately
with HIP events on the C3-as-u64 chained list of bench.py --workload
c3chain64, plus the per-unit-starts decode of the same stream and the
decoder's data-movement probe on it (tpfm_probe256v64: its loads and stores,
no decoding).  With TPF_LIB=ablib/x.so (A/B and ablation builds) the sums may be wrong: nothing is
verified here.
usage: TPF_LIB=... python scripts/chain64_phase_probe.py [nunits] [reps]"""
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
reps = int(sys.argv[2]) if len(sys.argv) > 2 else 10
dev = torch.device("cuda:0")
vals, starts = bench_data.gen_c3_64(nb, seed=7, dev=dev, first_block=0, carry_fn=None)
packed, offs = tpf.enc_batch("256v64", vals.view(-1), nb, 256, d1=True, starts=starts)
L = tpf.lib()
fmt = tpf.FMT["256v64"]
ws = torch.empty(int(L.tpf_d1dec64_chain_workspace_size(nb)), dtype=torch.uint8, device=dev)
total = torch.zeros(1, dtype=torch.int64, device=dev)
out = torch.empty((nb, 256), dtype=torch.int64, device=dev)
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def a():
    assert L.tpf_d1dec64_chain_sums(fmt, packed.data_ptr(), packed.numel(), offs.data_ptr(), nb, ws.data_ptr(), ws.numel(),
                                    total.data_ptr(), None, s) == 0


def b():
    assert L.tpf_d1dec64_chain_decode(fmt, packed.data_ptr(), packed.numel(), offs.data_ptr(), nb, out.data_ptr(),
                                      ctypes.c_uint64(12345), ws.data_ptr(), None, s) == 0


def per_unit():
    tpf.dec_batch("256v64", packed, offs, nb, 256, starts=starts, out=out.view(-1))


def probe():
    tpf.probe256v64(packed, offs, nb, out.view(-1))


res = {}
for name, f in (("phaseA", a), ("phaseB", b), ("per_unit_starts", per_unit), ("probe", probe)):
    f()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        f()
    e1.record()
    torch.cuda.synchronize()
    res[name] = round(e0.elapsed_time(e1) / reps, 4)
print(os.path.basename(os.environ.get("TPF_LIB", "tree")), "ms", res, "packed_bytes", packed.numel())
