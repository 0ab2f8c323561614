"""A/B of the 256v32 encoders on one box (C4 mix, 10M blocks): the production
two-pass encoder (batch entry and tpf_probe_enc256v32 mode 3) vs the rejected
encoders of scripts/enc_variants.hip (scripts/libencvar.so, built by
scripts/build_variants.sh: look-back modes 4-12, load policies 13-15,
persistent grid 16/17), alternating, HIP events on the launch stream; every
output verified.  ENC_AB_PIPE=1 adds the pipelined encoder's variants."""
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
dev = torch.device("cuda:0")
vals, _ = bench.gen_c2(nb, 0, seed=11, dev=dev, pcts=[0, 5, 10, 25])
L = tpf.lib()
cap = int(L.tpf_p4enc256v32_bound(nb))
out = torch.empty(cap, dtype=torch.uint8, device=dev)
offs = torch.empty(nb + 1, dtype=torch.int64, device=dev)
V = ctypes.CDLL(os.path.join(ROOT, "scripts", "libencvar.so"))
V.encvar_workspace_size.restype = ctypes.c_size_t
V.encvar_workspace_size.argtypes = [ctypes.c_uint64]
V.encvar_launch.argtypes = [ctypes.c_int, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64,
                            ctypes.c_void_p, ctypes.c_void_p, ctypes.c_size_t, ctypes.c_void_p]
wsb = max(int(L.tpf_p4enc256v32_workspace_size(nb)), int(V.encvar_workspace_size(nb)))
ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)


def pipe():
    assert L.tpf_p4enc256v32_batch(vals.data_ptr(), nb, out.data_ptr(), cap, offs.data_ptr(), ws.data_ptr(), wsb, s) == 0


def probe(mode):
    def f():
        if mode <= 3:
            assert L.tpf_probe_enc256v32(mode, vals.data_ptr(), nb, out.data_ptr(), cap, offs.data_ptr(), ws.data_ptr(),
                                         wsb, s) == 0
        else:
            assert V.encvar_launch(mode, vals.data_ptr(), nb, out.data_ptr(), cap, offs.data_ptr(), ws.data_ptr(), wsb,
                                   s) == 0
    return f


twopass = probe(3)
# pipelined variants: 16 + chunk items + 1024 * lag + 65536 * minw + 2^20 * entries per ticket
def pv(ci, lag, minw, k):
    return probe(16 + ci + 1024 * lag + 65536 * minw + (1 << 20) * k)


VARIANTS = [("twopass", twopass), ("production", pipe), ("tp_nt", probe(13)), ("tp_sc1", probe(14)),
            ("tp_nt_write", probe(15)), ("tp_persist8", probe(16)), ("tp_persist4", probe(17)), ("lookback", probe(12)), ("lb_k4", probe(5)), ("lb_k6", probe(6)), ("lb_k8", probe(7)),
            ("lb_k8_a5120", probe(8)), ("lb_k8_a4096", probe(9)), ("lb_k6_a3840", probe(10)), ("lb_k12_a7680", probe(11)),
            ("lb_fallback", probe(4))]
if os.environ.get("ENC_AB_PIPE"):
    VARIANTS += [(f"ci{ci}_lag{lag}_w{w}_k{k}", pv(ci, lag, w, k))
                 for ci, lag, w, k in [(256, 2, 8, 8), (256, 2, 0, 8), (256, 2, 6, 8), (256, 2, 8, 16), (256, 4, 8, 8),
                                       (512, 2, 0, 8), (128, 4, 0, 8)]]


def timed(fn, reps=10):
    for _ in range(2):
        fn()
    e = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    e[0].record()
    for _ in range(reps):
        fn()
    e[1].record()
    torch.cuda.synchronize()
    return e[0].elapsed_time(e[1]) / reps


res = {}
for name, fn in VARIANTS:
    out.zero_()
    fn()
    torch.cuda.synchronize()
    tot = int(offs[-1].item())
    back = tpf.dec256v32(out[:tot], offs, nb)
    ok = bool(torch.equal(back, vals))
    res[name] = (tot, ok)
    print(name, "total", tot, "verified", ok, flush=True)
    assert ok and tot == res["twopass"][0], name
for rnd in range(2):
    for name, fn in VARIANTS:
        ms = timed(fn)
        print(f"round {rnd} {name:16s} {ms:.4f} ms  {nb * 256 / ms / 1e6:.1f} G int32/s", flush=True)
