"""Per-block drop-in API latency (measurement tool): turbopfor::p4Dec256v32 /
p4Enc256v32 through their extern "C" mirrors, one block per call, as a
reference caller relinked against libturbopfor_amd.so would call them.
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
for name, fn in (("p4Enc256v32", lambda: L.tpf_p4Enc256v32(vals.ctypes.data, 256, buf.ctypes.data)),
                 ("p4Dec256v32", lambda: L.tpf_p4Dec256v32(buf.ctypes.data, 256, out.ctypes.data))):
    for _ in range(50):
        fn()
    t0 = time.perf_counter()
    for _ in range(calls):
        fn()
    dt = (time.perf_counter() - t0) / calls
    print(f"{name}: {dt * 1e6:.1f} us per call")
assert np.array_equal(out, vals)
print("ok")
