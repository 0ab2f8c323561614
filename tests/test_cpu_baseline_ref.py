"""bench.py's cpu_baseline legs for C3 and C4 (oracle/_ref/libtpref.so:
tpref_d1dec256v32_stream_mt, tpref_rt256v32_stream_mt) compute what they
claim to time: the reference scalar path decodes the per-block and chained
D1 streams to the original posting list and round-trips C4-style values.
Skipped where oracle/_ref was not built (no /root/reference)."""
import ctypes

import numpy as np
import pytest

import ref_lib

pytestmark = pytest.mark.skipif(not ref_lib.available(), reason="oracle/_ref not built")


def _posting_stream(nb, seed):
    r = np.random.default_rng(seed)
    gaps = r.integers(1, 65, nb * 256).astype(np.uint64)
    big = r.random(nb * 256) < 0.05
    gaps[big] += r.integers(0, 1 << 16, int(big.sum())).astype(np.uint64)
    vals = (np.cumsum(gaps) & 0xFFFFFFFF).astype(np.uint32).reshape(nb, 256)
    starts = np.zeros(nb, np.uint32)
    starts[1:] = vals[:-1, -1]
    L = ref_lib.lib()
    buf = np.zeros(nb * 1100 + 64, np.uint8)
    off = np.zeros(nb + 1, np.uint64)
    base = buf.ctypes.data
    p = base
    for i in range(nb):
        off[i] = p - base
        row = np.ascontiguousarray(vals[i])
        p = L.tpref_s_p4d1enc256v32(row.ctypes.data_as(ref_lib.u32p), 256,
                                    ctypes.cast(p, ref_lib.u8p), int(starts[i]))
    off[nb] = p - base
    return vals, starts, buf, off


@pytest.mark.parametrize("chained", [0, 1])
@pytest.mark.parametrize("threads", [1, 3])
def test_d1dec_stream_mt_scalar(chained, threads):
    nb = 37
    vals, starts, buf, off = _posting_stream(nb, 5 + chained)
    L = ctypes.CDLL(ref_lib.REF_SO)
    f = L.tpref_d1dec256v32_stream_mt
    f.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_uint64, ctypes.c_void_p, ctypes.c_int, ctypes.c_int, ctypes.c_int]
    f.restype = ctypes.c_double
    out = np.zeros((nb, 256), np.uint32)
    assert f(buf.ctypes.data, off.ctypes.data, starts.ctypes.data, nb, out.ctypes.data, threads, 0, chained) >= 0
    np.testing.assert_array_equal(out, vals)


@pytest.mark.parametrize("threads", [1, 4])
def test_rt_stream_mt_scalar(threads):
    r = np.random.default_rng(9)
    nb = 64
    bw = r.integers(1, 33, (nb, 1)).astype(np.uint64)
    v = (r.integers(0, 1 << 32, (nb, 256), dtype=np.uint64) & ((np.uint64(1) << bw) - np.uint64(1)))
    exc = r.random((nb, 256)) < 0.25
    v[exc] = r.integers(0, 1 << 32, int(exc.sum()), dtype=np.uint64)
    v = v.astype(np.uint32)
    L = ctypes.CDLL(ref_lib.REF_SO)
    f = L.tpref_rt256v32_stream_mt
    f.argtypes = [ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p, ctypes.c_uint64, ctypes.c_void_p,
                  ctypes.c_void_p, ctypes.c_int, ctypes.c_int]
    f.restype = ctypes.c_double
    slot = 1088
    scratch = np.zeros(nb * slot + 64, np.uint8)
    off = np.zeros(nb, np.uint64)
    out = np.zeros((nb, 256), np.uint32)
    assert f(v.ctypes.data, nb, scratch.ctypes.data, slot, off.ctypes.data, out.ctypes.data, threads, 0) >= 0
    np.testing.assert_array_equal(out, v)
    # a slot below the largest block is refused
    assert f(v.ctypes.data, nb, scratch.ctypes.data, 1000, off.ctypes.data, out.ctypes.data, threads, 0) < 0
