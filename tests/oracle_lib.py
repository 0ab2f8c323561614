"""ctypes binding of oracle/liborc.so -- the CPU restatement used as the
parity checker.  Test infrastructure only (tests/, smoke(), bench cpu_baseline)."""
import ctypes
import os
import subprocess

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
_lib = None

u8p = ctypes.POINTER(ctypes.c_uint8)
u32p = ctypes.POINTER(ctypes.c_uint32)
u64p = ctypes.POINTER(ctypes.c_uint64)
c_u = ctypes.c_uint


def lib():
    global _lib
    if _lib is None:
        path = os.path.join(ORACLE_DIR, "liborc.so")
        if not os.path.exists(path):
            subprocess.check_call(["make", "-s", "-C", ORACLE_DIR, "liborc.so"])
        L = ctypes.CDLL(path)
        for name, argt in [
            ("orc_p4enc256v32", [u32p, c_u, u8p]), ("orc_p4enc128v32", [u32p, c_u, u8p]),
            ("orc_p4enc32", [u32p, c_u, u8p]),
            ("orc_p4d1enc256v32", [u32p, c_u, u8p, ctypes.c_uint32]),
            ("orc_p4d1enc128v32", [u32p, c_u, u8p, ctypes.c_uint32]),
            ("orc_p4d1enc32", [u32p, c_u, u8p, ctypes.c_uint32]),
            ("orc_p4enc128v64", [u64p, c_u, u8p]), ("orc_p4enc256v64", [u64p, c_u, u8p]),
            ("orc_p4d1enc128v64", [u64p, c_u, u8p, ctypes.c_uint64]),
            ("orc_p4d1enc256v64", [u64p, c_u, u8p, ctypes.c_uint64]),
        ]:
            f = getattr(L, name)
            f.argtypes = argt
            f.restype = ctypes.c_void_p
        for name, argt in [
            ("orc_p4dec256v32", [u8p, c_u, u32p]), ("orc_p4dec128v32", [u8p, c_u, u32p]),
            ("orc_p4dec32", [u8p, c_u, u32p]),
            ("orc_p4d1dec256v32", [u8p, c_u, u32p, ctypes.c_uint32]),
            ("orc_p4d1dec128v32", [u8p, c_u, u32p, ctypes.c_uint32]),
            ("orc_p4d1dec32", [u8p, c_u, u32p, ctypes.c_uint32]),
            ("orc_p4dec128v64", [u8p, c_u, u64p]), ("orc_p4dec256v64", [u8p, c_u, u64p]),
            ("orc_p4d1dec128v64", [u8p, c_u, u64p, ctypes.c_uint64]),
            ("orc_p4d1dec256v64", [u8p, c_u, u64p, ctypes.c_uint64]),
        ]:
            f = getattr(L, name)
            f.argtypes = argt
            f.restype = ctypes.c_void_p
        for name in ["orc_enc256v32_batch"]:
            getattr(L, name).argtypes = [u32p, ctypes.c_uint64, u8p, u64p]
            getattr(L, name).restype = ctypes.c_uint64
        L.orc_d1enc256v32_batch.argtypes = [u32p, ctypes.c_uint64, u8p, u64p, u32p]
        L.orc_d1enc256v32_batch.restype = ctypes.c_uint64
        L.orc_dec256v32_batch.argtypes = [u8p, u64p, ctypes.c_uint64, u32p]
        L.orc_d1dec256v32_batch.argtypes = [u8p, u64p, ctypes.c_uint64, u32p, u32p]
        L.orc_enc256v64_batch.argtypes = [u64p, ctypes.c_uint64, u8p, u64p]
        L.orc_enc256v64_batch.restype = ctypes.c_uint64
        L.orc_d1enc256v64_batch.argtypes = [u64p, ctypes.c_uint64, u8p, u64p, u64p]
        L.orc_d1enc256v64_batch.restype = ctypes.c_uint64
        L.orc_dec256v64_batch.argtypes = [u8p, u64p, ctypes.c_uint64, u64p]
        L.orc_d1dec256v64_batch.argtypes = [u8p, u64p, ctypes.c_uint64, u64p, u64p]
        L.orc_enc32_batch.argtypes = [u32p, ctypes.c_uint64, c_u, u8p, u64p]
        L.orc_enc32_batch.restype = ctypes.c_uint64
        L.orc_d1enc32_batch.argtypes = [u32p, ctypes.c_uint64, c_u, u8p, u64p, u32p]
        L.orc_d1enc32_batch.restype = ctypes.c_uint64
        L.orc_dec32_batch.argtypes = [u8p, u64p, ctypes.c_uint64, c_u, u32p]
        L.orc_d1dec32_batch.argtypes = [u8p, u64p, ctypes.c_uint64, c_u, u32p, u32p]
        L.orc_dec256v32_batch_mt.argtypes = [u8p, u64p, ctypes.c_uint64, u32p, ctypes.c_int]
        L.orc_p4bits32.argtypes = [u32p, c_u, ctypes.POINTER(c_u)]
        L.orc_p4bits32.restype = c_u
        L.orc_p4bits64.argtypes = [u64p, c_u, ctypes.POINTER(c_u)]
        L.orc_p4bits64.restype = c_u
        _lib = L
    return _lib


def ptr(a, t):
    return a.ctypes.data_as(t)


# --- per-block convenience (return python bytes / numpy) --------------------
_FMT = {
    "256v32": (np.uint32, 256), "128v32": (np.uint32, 128), "32": (np.uint32, None),
    "128v64": (np.uint64, 128), "256v64": (np.uint64, 256),
}


def encode(fmt, values, d1=False, start=0):
    dt, blk = _FMT[fmt]
    n = len(values)
    buf = np.zeros(max(n, 256) + 64, dtype=dt)
    buf[:n] = values
    out = np.zeros(n * 10 + 4096, dtype=np.uint8)
    L = lib()
    tp = u32p if dt == np.uint32 else u64p
    name = ("orc_p4d1enc" if d1 else "orc_p4enc") + fmt
    f = getattr(L, name)
    args = [ptr(buf, tp), n, ptr(out, u8p)] + ([start] if d1 else [])
    end = f(*args)
    return bytes(out[: end - out.ctypes.data])


def decode(fmt, enc, n, d1=False, start=0):
    dt, blk = _FMT[fmt]
    src = np.zeros(len(enc) + 64, dtype=np.uint8)
    src[: len(enc)] = np.frombuffer(enc, dtype=np.uint8)
    out = np.zeros(max(n, 256) + 64, dtype=dt)
    L = lib()
    tp = u32p if dt == np.uint32 else u64p
    name = ("orc_p4d1dec" if d1 else "orc_p4dec") + fmt
    f = getattr(L, name)
    args = [ptr(src, u8p), n, ptr(out, tp)] + ([start] if d1 else [])
    end = f(*args)
    return out[:n].copy(), end - src.ctypes.data


# --- batch helpers -----------------------------------------------------------
def enc256v32_batch(vals2d, starts=None):
    """vals2d: (nblocks, 256) uint32 -> (packed uint8 array, offsets uint64[nb+1])"""
    v = np.ascontiguousarray(vals2d, dtype=np.uint32)
    nb = v.shape[0]
    out = np.zeros(nb * 1100 + 2400, dtype=np.uint8)
    off = np.zeros(nb + 1, dtype=np.uint64)
    L = lib()
    if starts is None:
        tot = L.orc_enc256v32_batch(ptr(v, u32p), nb, ptr(out, u8p), ptr(off, u64p))
    else:
        st = np.ascontiguousarray(starts, dtype=np.uint32)
        tot = L.orc_d1enc256v32_batch(ptr(v, u32p), nb, ptr(out, u8p), ptr(off, u64p), ptr(st, u32p))
    return out[:tot].copy(), off


def dec256v32_batch(packed, off, nb, starts=None):
    src = np.zeros(len(packed) + 64, dtype=np.uint8)
    src[: len(packed)] = packed
    out = np.zeros((nb, 256), dtype=np.uint32)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    L = lib()
    if starts is None:
        rc = L.orc_dec256v32_batch(ptr(src, u8p), ptr(off, u64p), nb, ptr(out, u32p))
    else:
        st = np.ascontiguousarray(starts, dtype=np.uint32)
        rc = L.orc_d1dec256v32_batch(ptr(src, u8p), ptr(off, u64p), nb, ptr(out, u32p), ptr(st, u32p))
    assert rc == 0, rc
    return out


def enc256v64_batch(vals2d, starts=None):
    v = np.ascontiguousarray(vals2d, dtype=np.uint64)
    nb = v.shape[0]
    out = np.zeros(nb * 2400 + 4800, dtype=np.uint8)
    off = np.zeros(nb + 1, dtype=np.uint64)
    L = lib()
    if starts is None:
        tot = L.orc_enc256v64_batch(ptr(v, u64p), nb, ptr(out, u8p), ptr(off, u64p))
    else:
        st = np.ascontiguousarray(starts, dtype=np.uint64)
        tot = L.orc_d1enc256v64_batch(ptr(v, u64p), nb, ptr(out, u8p), ptr(off, u64p), ptr(st, u64p))
    return out[:tot].copy(), off


def dec256v64_batch(packed, off, nb, starts=None):
    src = np.zeros(len(packed) + 64, dtype=np.uint8)
    src[: len(packed)] = packed
    out = np.zeros((nb, 256), dtype=np.uint64)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    L = lib()
    if starts is None:
        rc = L.orc_dec256v64_batch(ptr(src, u8p), ptr(off, u64p), nb, ptr(out, u64p))
    else:
        st = np.ascontiguousarray(starts, dtype=np.uint64)
        rc = L.orc_d1dec256v64_batch(ptr(src, u8p), ptr(off, u64p), nb, ptr(out, u64p), ptr(st, u64p))
    assert rc == 0, rc
    return out


def enc32_batch(vals2d, starts=None):
    v = np.ascontiguousarray(vals2d, dtype=np.uint32)
    nb, bn = v.shape
    out = np.zeros(nb * (bn * 5 + 40) + 4096, dtype=np.uint8)
    off = np.zeros(nb + 1, dtype=np.uint64)
    L = lib()
    if starts is None:
        tot = L.orc_enc32_batch(ptr(v, u32p), nb, bn, ptr(out, u8p), ptr(off, u64p))
    else:
        st = np.ascontiguousarray(starts, dtype=np.uint32)
        tot = L.orc_d1enc32_batch(ptr(v, u32p), nb, bn, ptr(out, u8p), ptr(off, u64p), ptr(st, u32p))
    return out[:tot].copy(), off


def dec32_batch(packed, off, nb, bn, starts=None):
    src = np.zeros(len(packed) + 64, dtype=np.uint8)
    src[: len(packed)] = packed
    out = np.zeros((nb, bn), dtype=np.uint32)
    off = np.ascontiguousarray(off, dtype=np.uint64)
    L = lib()
    if starts is None:
        rc = L.orc_dec32_batch(ptr(src, u8p), ptr(off, u64p), nb, bn, ptr(out, u32p))
    else:
        st = np.ascontiguousarray(starts, dtype=np.uint32)
        rc = L.orc_d1dec32_batch(ptr(src, u8p), ptr(off, u64p), nb, bn, ptr(out, u32p), ptr(st, u32p))
    assert rc == 0, rc
    return out


# --- n-variant streams (tpf_p4nenc256v32's layout) ---------------------------
def encn256v32(values, d1=False, start0=0):
    """Any n: the stream a reference caller builds by chaining p4Enc256v32 over
    the full 256-blocks and p4Enc32 over the rest (D1: p4D1* with each block's
    start = the value before it, the first = start0).  -> (packed, offsets)"""
    v = np.ascontiguousarray(values, dtype=np.uint32).reshape(-1)
    n, nf, tail = len(v), len(v) // 256, len(v) % 256
    full = v[: nf * 256].reshape(nf, 256)
    if d1:
        starts = np.concatenate([[start0], full.reshape(-1)[255::256][:-1]]).astype(np.uint32) if nf else None
        packed, off = enc256v32_batch(full, starts) if nf else (np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    else:
        packed, off = enc256v32_batch(full) if nf else (np.zeros(0, np.uint8), np.zeros(1, np.uint64))
    if tail:
        prev = (int(v[nf * 256 - 1]) if nf else start0) & 0xFFFFFFFF
        t = encode("32", v[nf * 256:], d1=d1, start=prev)
        packed = np.concatenate([packed, np.frombuffer(t, dtype=np.uint8)])
        off = np.concatenate([off, [int(off[-1]) + len(t)]]).astype(np.uint64)
    return packed, off
