"""Diagnostic (measurement tool): the 256v32 encode + decode batch pair on
random data, eager and captured into a hipGraph, with every buffer carved out
of ONE arena with 4 KB canary zones between them, with or without the
per-block block server running in another thread (or another thread launching
plain torch kernels).  After each call the
canaries must be intact and d_err must read -1.  Prints one line per mode.
usage: python scripts/graph_canary.py [nblocks] [iters]"""
import ctypes
import os
import sys
import threading
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
sys.path.insert(0, os.path.join(ROOT, "tests"))
import turbopfor_amd as tpf  # noqa: E402

nb = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
iters = int(sys.argv[2]) if len(sys.argv) > 2 else 20
DEV = "cuda:0"
L = tpf.lib()
G = 4096
CAN = 0xA5
cap = int(L.tpf_p4enc256v32_bound(nb))
wsb = int(L.tpf_p4enc256v32_workspace_size(nb))
sizes = {"vals": nb * 1024, "packed": cap, "offs": (nb + 1) * 8, "ws": wsb, "out": nb * 1024, "err": 8}
layout, pos = {}, G
for k, sz in sizes.items():
    layout[k] = (pos, sz)
    pos += (sz + 255) // 256 * 256 + G
arena = torch.full((pos,), CAN, dtype=torch.uint8, device=DEV)


def view(k, dt):
    a, sz = layout[k]
    return arena[a:a + sz].view(dt)


vals, packed, offs, ws, out, err = (view("vals", torch.int32), view("packed", torch.uint8), view("offs", torch.int64),
                                    view("ws", torch.uint8), view("out", torch.int32), view("err", torch.int64))
gen = torch.Generator(device=DEV)
gen.manual_seed(5)


def fresh():
    bw = torch.randint(1, 33, (nb, 1), device=DEV, generator=gen)
    raw = torch.randint(-(1 << 31), (1 << 31) - 1, (nb, 256), device=DEV, generator=gen, dtype=torch.int32)
    return torch.where(bw >= 32, raw, raw & ((torch.ones_like(bw) << bw) - 1).to(torch.int32)).view(-1)


def seq():
    s = ctypes.c_void_p(torch.cuda.current_stream().cuda_stream)
    assert L.tpf_p4enc256v32_batch(vals.data_ptr(), nb, packed.data_ptr(), cap, offs.data_ptr(), ws.data_ptr(), wsb, s) == 0
    assert L.tpf_p4dec256v32_batch(packed.data_ptr(), cap, offs.data_ptr(), nb, out.data_ptr(), err.data_ptr(), s) == 0


def check(tag):
    torch.cuda.synchronize()
    a = arena.cpu().numpy()
    bad = []
    regs = sorted(layout.values())
    gaps = [(0, regs[0][0])] + [(st + sz, nxt) for (st, sz), nxt in zip(regs, [r[0] for r in regs[1:]] + [len(a)])]
    for lo, hi in gaps:
        z = a[lo:hi]
        if (z != CAN).any():
            i = int(np.argmax(z != CAN))
            bad.append((lo + i, hi, z[i:i + 16].tobytes().hex()))
    e = int(err.cpu().item())
    ok_v = bool(torch.equal(out, vals))
    return bad, e, ok_v


srv_stop = threading.Event()


def per_block():
    L.tpf_p4Enc256v32.restype = ctypes.c_void_p
    L.tpf_p4Enc256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
    v = np.arange(256, dtype=np.uint32)
    buf = np.zeros(4096, np.uint8)
    while not srv_stop.is_set():
        L.tpf_p4Enc256v32(v.ctypes.data, 256, buf.ctypes.data)
        time.sleep(0.001)


def launcher():
    """another thread launching ordinary torch kernels on a stream of its own"""
    st = torch.cuda.Stream()
    y = torch.zeros(1 << 16, dtype=torch.int64, device=DEV)
    with torch.cuda.stream(st):
        while not srv_stop.is_set():
            y.add_(1)
            time.sleep(0.001)
    st.synchronize()


def run(mode, server):
    nbad, nerr, nval, first = 0, 0, 0, None
    g = None
    if mode == "graph":  # captured before the server thread starts (no other thread's HIP calls during capture)
        vals.copy_(fresh())
        seq()
        torch.cuda.synchronize()
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            seq()
    th = None
    if server:
        srv_stop.clear()
        th = threading.Thread(target=per_block if server == "perblock" else launcher)
        th.start()
    for it in range(iters):
        vals.copy_(fresh())
        out.zero_()
        if g is not None:
            g.replay()
        else:
            seq()
        bad, e, ok_v = check(it)
        nbad += bool(bad)
        nerr += e != -1
        nval += not ok_v
        if (bad or e != -1 or not ok_v) and first is None:
            first = (it, bad[:3], hex(e & ((1 << 64) - 1)), ok_v)
    if th is not None:
        srv_stop.set()
        th.join()
    print(f"mode={mode} server={server} iters={iters} canary_broken={nbad} err_wrong={nerr} values_wrong={nval} first={first}",
          flush=True)
    del g


print(f"nblocks={nb} layout={layout}", flush=True)
for mode, server in (("eager", None), ("eager", "perblock"), ("graph", None), ("graph", "perblock"), ("graph", "launcher")):
    run(mode, server)
print("done", flush=True)
