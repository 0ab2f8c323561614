"""ctypes binding of oracle/_ref/libtpref.so: the REFERENCE library compiled
from its own sources (oracle/Makefile `ref`).  Test/baseline infrastructure
only; absent unless built in the container that has /root/reference."""
import ctypes
import os

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
REF_SO = os.path.join(ROOT, "oracle", "_ref", "libtpref.so")
_lib = None
u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)


def available():
    return os.path.exists(REF_SO)


def lib():
    global _lib
    if _lib is None:
        L = ctypes.CDLL(REF_SO)
        for fam in ("tpref_s_", "tpref_d_"):
            for fmt, ip, vp in (("256v32", u32p, ctypes.c_uint32), ("128v32", u32p, ctypes.c_uint32),
                                ("32", u32p, ctypes.c_uint32), ("256v64", u64p, ctypes.c_uint64),
                                ("128v64", u64p, ctypes.c_uint64)):
                f = getattr(L, fam + "p4enc" + fmt)
                f.argtypes = [ip, ctypes.c_uint, u8p]
                f.restype = ctypes.c_void_p
                f = getattr(L, fam + "p4d1enc" + fmt)
                f.argtypes = [ip, ctypes.c_uint, u8p, vp]
                f.restype = ctypes.c_void_p
                f = getattr(L, fam + "p4dec" + fmt)
                f.argtypes = [u8p, ctypes.c_uint, ip]
                f.restype = ctypes.c_void_p
                f = getattr(L, fam + "p4d1dec" + fmt)
                f.argtypes = [u8p, ctypes.c_uint, ip, vp]
                f.restype = ctypes.c_void_p
        L.tpref_dec256v32_stream_mt.argtypes = [u8p, u64p, ctypes.c_uint64, u32p, ctypes.c_int, ctypes.c_int,
                                                ctypes.c_int]
        L.tpref_dec256v32_stream_mt.restype = ctypes.c_double
        L.tpref_abtest_dec256v32.argtypes = [u8p, ctypes.c_uint, ctypes.c_uint, ctypes.c_int]
        L.tpref_abtest_dec256v32.restype = ctypes.c_double
        _lib = L
    return _lib


def enc256v32_stream(vals2d, scalar=True):
    """Reference-encode (nb,256) uint32 blocks end to end -> (packed, offsets)."""
    L = lib()
    f = L.tpref_s_p4enc256v32 if scalar else L.tpref_d_p4enc256v32
    v = np.ascontiguousarray(vals2d, dtype=np.uint32)
    nb = v.shape[0]
    out = np.zeros(nb * 1100 + 4096, dtype=np.uint8)
    off = np.zeros(nb + 1, dtype=np.uint64)
    base = out.ctypes.data
    vp = v.ctypes.data
    pos = 0
    for i in range(nb):
        off[i] = pos
        end = f(ctypes.cast(vp + i * 1024, u32p), 256, ctypes.cast(base + pos, u8p))
        pos = end - base
    off[nb] = pos
    return out[:pos].copy(), off


def encn256v32_stream(values, d1=False, start0=0, scalar=True):
    """What a reference caller writes for n values: p4(D1)Enc256v32 while 256
    remain, then one p4(D1)Enc32 of the rest, each call at the end pointer of
    the previous one (D1 start = the value before the block).  -> bytes"""
    L = lib()
    pre = "tpref_s_" if scalar else "tpref_d_"
    f256 = getattr(L, pre + ("p4d1enc256v32" if d1 else "p4enc256v32"))
    f32 = getattr(L, pre + ("p4d1enc32" if d1 else "p4enc32"))
    v = np.zeros(len(values) + 64, dtype=np.uint32)
    v[: len(values)] = values
    n = len(values)
    out = np.zeros(n * 6 + 4096, dtype=np.uint8)
    base, vp, pos, i, prev = out.ctypes.data, v.ctypes.data, 0, 0, start0 & 0xFFFFFFFF
    while i < n:
        m = min(256, n - i)
        f = f256 if m == 256 else f32
        args = [ctypes.cast(vp + 4 * i, u32p), m, ctypes.cast(base + pos, u8p)] + ([prev] if d1 else [])
        pos = f(*args) - base
        prev = int(v[i + m - 1])
        i += m
    return bytes(out[:pos])
