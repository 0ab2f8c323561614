"""Per-block drop-in API latency (measurement tool): turbopfor::p4Dec256v32 /
p4Enc256v32 (and the 32-bit p4Dec32 of configs[0]) through their extern "C"
mirrors, one block per call, as a reference caller relinked against
libturbopfor_amd.so would call them, for both per-block designs
(tpf_perblock_mode 0 = resident block server with request mailboxes in
device memory, 2 = the same with request mailboxes in host memory, 1 =
launch + synchronise).  The first line times a bare ctypes call (the
Python-side share of every number).
Prints the median, p99, p99.9 and maximum over `calls` calls.
usage: python scripts/perblock_latency.py [calls]"""
import ctypes
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "turbopfor-cpp_amd", "python"))
import turbopfor_amd as tpf  # noqa: E402

calls = int(sys.argv[1]) if len(sys.argv) > 1 else 2000
L = tpf.lib()
L.tpf_p4Enc256v32.restype = ctypes.c_void_p
L.tpf_p4Enc256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
L.tpf_p4Dec256v32.restype = ctypes.c_void_p
L.tpf_p4Dec256v32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
rng = np.random.default_rng(1)
vals = rng.integers(0, 1 << 12, 256, dtype=np.uint32)
buf = np.zeros(4096, np.uint8)
out = np.zeros(256, np.uint32)
end = L.tpf_p4Enc256v32(vals.ctypes.data, 256, buf.ctypes.data)
L.tpf_perblock_mode.restype = ctypes.c_int
L.tpf_perblock_mode.argtypes = [ctypes.c_int]
L.tpf_p4Dec32.restype = ctypes.c_void_p
L.tpf_p4Dec32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
L.tpf_p4Enc32.restype = ctypes.c_void_p
L.tpf_p4Enc32.argtypes = [ctypes.c_void_p, ctypes.c_uint, ctypes.c_void_p]
v127 = rng.integers(0, 256, 127, dtype=np.uint32)
b127 = np.zeros(1024, np.uint8)
o127 = np.zeros(256, np.uint32)
ts = np.empty(calls)
for i in range(calls):
    t0 = time.perf_counter()
    L.tpf_perblock_mode(-1)
    ts[i] = time.perf_counter() - t0
print(f"bare ctypes call (tpf_perblock_mode(-1)): median {np.median(ts) * 1e6:6.2f} us")
for mode, mname in ((1, "launch+sync"), (2, "server/hostmail"), (0, "block server")):
    L.tpf_perblock_mode(mode)
    L.tpf_p4Enc32(v127.ctypes.data, 127, b127.ctypes.data)
    for name, fn in (("p4Enc256v32", lambda: L.tpf_p4Enc256v32(vals.ctypes.data, 256, buf.ctypes.data)),
                     ("p4Dec256v32", lambda: L.tpf_p4Dec256v32(buf.ctypes.data, 256, out.ctypes.data)),
                     ("p4Dec32 n=127", lambda: L.tpf_p4Dec32(b127.ctypes.data, 127, o127.ctypes.data))):
        for _ in range(50):
            fn()
        ts = np.empty(calls)
        for i in range(calls):
            t0 = time.perf_counter()
            fn()
            ts[i] = time.perf_counter() - t0
        # p99.9 and max: a run of 20,000 calls crosses ~20 of the server's
        # 5 ms lifetimes, whose relaunch shows in the tail
        print(f"{mname:15s} {name:14s}: median {np.median(ts) * 1e6:6.1f} us, p99 {np.percentile(ts, 99) * 1e6:6.1f} us, "
              f"p99.9 {np.percentile(ts, 99.9) * 1e6:6.1f} us, max {ts.max() * 1e6:7.1f} us, mean {ts.mean() * 1e6:6.1f} us per call")
    assert np.array_equal(out, vals) and np.array_equal(o127[:127], v127)
L.tpf_perblock_mode(0)
print("ok")
